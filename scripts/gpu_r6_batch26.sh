#!/bin/bash
# Round 6, batch 26: HT moments in two LDS copies (even / odd lanes): tests, phases, A/B.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b26; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ht_sequential.py -m gpu -q --timeout 300 --timeout-method thread > $O/ht_tests.txt 2>&1 || { tail -30 $O/ht_tests.txt; exit 3; }
tail -2 $O/ht_tests.txt
timeout -k 10 300 python scripts/ht_diag.py > $O/ht_diag.txt 2>&1 || { tail -20 $O/ht_diag.txt; exit 3; }
tail -3 $O/ht_diag.txt
OMLDM_HT_REP=1 timeout -k 10 300 python scripts/ht_diag.py > $O/ht_diag_rep1.txt 2>&1 || { tail -20 $O/ht_diag_rep1.txt; exit 3; }
tail -3 $O/ht_diag_rep1.txt
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only HT --quality-rounds 2 > $O/ht_p16.json 2> $O/ht_p16.err || { tail -20 $O/ht_p16.err; exit 3; }
cut -c 1-1200 $O/ht_p16.json
OMLDM_HT_REP=1 timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only HT --quality-rounds 0 > $O/ht_p16_rep1.json 2> $O/ht_p16_rep1.err || { tail -20 $O/ht_p16_rep1.err; exit 3; }
cut -c 1-1200 $O/ht_p16_rep1.json
