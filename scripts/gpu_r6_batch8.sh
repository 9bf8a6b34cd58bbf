#!/bin/bash
# Round 6, batch 8: MultiClassPA scan with the max-tree decide: tests, phase cycles, rates.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b8
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -x -q --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1 || { tail -40 $O/mc_tests.txt; exit 3; }
tail -2 $O/mc_tests.txt
for k in 4 8 10 16; do
  OMLDM_MC_SCAN_KMAX=16 timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
