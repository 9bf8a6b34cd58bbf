#!/bin/bash
# Round 6, batch 25: HT grouped grace / consumed counts: tests, phases, A/B.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b25; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ht_sequential.py -m gpu -q --timeout 300 --timeout-method thread > $O/ht_tests.txt 2>&1 || { tail -30 $O/ht_tests.txt; exit 3; }
tail -2 $O/ht_tests.txt
timeout -k 10 300 python scripts/ht_diag.py > $O/ht_diag.txt 2>&1 || { tail -20 $O/ht_diag.txt; exit 3; }
tail -3 $O/ht_diag.txt
OMLDM_HT_GROUPCNT=0 timeout -k 10 300 python scripts/ht_diag.py > $O/ht_diag_rowcnt.txt 2>&1 || { tail -20 $O/ht_diag_rowcnt.txt; exit 3; }
tail -3 $O/ht_diag_rowcnt.txt
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only HT --quality-rounds 2 > $O/ht_p16.json 2> $O/ht_p16.err || { tail -20 $O/ht_p16.err; exit 3; }
cut -c 1-1200 $O/ht_p16.json
OMLDM_HT_GROUPCNT=0 timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only HT --quality-rounds 0 > $O/ht_p16_rowcnt.json 2> $O/ht_p16_rowcnt.err || { tail -20 $O/ht_p16_rowcnt.err; exit 3; }
cut -c 1-1200 $O/ht_p16_rowcnt.json
