#!/bin/bash
# Round 6, batch 7: NN v2 (simplified GEMM loop) and the MultiClassPA scan with the
# branch-free decide: tests, template diagnostics, phase cycles, learner rates.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py -m gpu -k mlp -x -q --timeout 120 --timeout-method thread > $O/mlp_tests.txt 2>&1 || { tail -30 $O/mlp_tests.txt; exit 3; }
tail -1 $O/mlp_tests.txt
for f in 0 2 1; do
  timeout -k 10 60 ./.probe/mlpp 16 0 $f > $O/mlpp_s16_f$f.txt 2>&1 || { cat $O/mlpp_s16_f$f.txt; exit 3; }
  cat $O/mlpp_s16_f$f.txt
done
for args in "4 8" "8 16" "10 16"; do
  timeout -k 10 300 python scripts/mc_kt_diag.py $args >> $O/mc_kt.txt 2>&1 || { tail -20 $O/mc_kt.txt; exit 3; }
done
cat $O/mc_kt.txt
for k in 4 8 16; do
  timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
timeout -k 10 900 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -v --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1
grep -E "PASSED|FAILED|passed|failed" $O/mc_tests.txt | tail -30
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only NN,MultiClassPA --quality-rounds 1 > $O/learners.json 2> $O/learners.err || { tail -20 $O/learners.err; exit 3; }
cut -c 1-1500 $O/learners.json
