#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b16; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -q --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1
grep -E "passed|failed|FAILED" $O/mc_tests.txt | tail -5
for k in 2 4; do
  timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
