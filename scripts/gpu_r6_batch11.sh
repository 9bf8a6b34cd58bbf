#!/bin/bash
# Round 6, batch 11: MultiClassPA scan with fixed-point partials: tests, repeats, cycles.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b11
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -q --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1
grep -E "passed|failed|FAILED" $O/mc_tests.txt | tail -12
timeout -k 10 600 python -u scripts/mc_repeat.py > $O/mc_repeat.txt 2>&1 || { tail -20 $O/mc_repeat.txt; exit 3; }
grep -v amdgpu.ids $O/mc_repeat.txt
for k in 4 8 10 16; do
  OMLDM_MC_SCAN_KMAX=16 timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
