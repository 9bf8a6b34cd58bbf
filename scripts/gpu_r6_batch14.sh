#!/bin/bash
# Round 6, batch 14: NN per-phase cycles (register-held stamps); the Hoeffding tree with the
# next chunk's rows prefetched: tests, phase cycles, learner rate.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b14; mkdir -p $O
for f in 2 3 0; do
  timeout -k 10 60 ./.probe/mlpp 16 0 $f > $O/mlpp_s16_f$f.txt 2>&1 || { cat $O/mlpp_s16_f$f.txt; exit 3; }
  cat $O/mlpp_s16_f$f.txt
done
timeout -k 10 600 python -u -m pytest tests/test_ht_sequential.py tests/test_kernels_dense.py -m gpu -k "ht or hoeffding" -q --timeout 300 --timeout-method thread > $O/ht_tests.txt 2>&1 || { tail -30 $O/ht_tests.txt; exit 3; }
tail -2 $O/ht_tests.txt
timeout -k 10 300 python scripts/ht_diag.py > $O/ht_diag.txt 2>&1 || { tail -20 $O/ht_diag.txt; exit 3; }
grep -v amdgpu.ids $O/ht_diag.txt | tail -4
OMLDM_MLP_FORM=3 timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only NN --quality-rounds 0 > $O/nn_f3.json 2>&1 && tail -c 300 $O/nn_f3.json
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only HT --quality-rounds 1 > $O/ht_p16.json 2> $O/ht_p16.err || { tail -20 $O/ht_p16.err; exit 3; }
cut -c 1-900 $O/ht_p16.json
