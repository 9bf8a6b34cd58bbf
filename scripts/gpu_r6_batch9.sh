#!/bin/bash
# Round 6, batch 9: MultiClassPA K = 16 template correctness map (padding vs spill).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b9
mkdir -p $O
export OMLDM_MC_SCAN_KMAX=16
timeout -k 10 900 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -q --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1
grep -E "passed|failed|FAILED" $O/mc_tests.txt | tail -12
for args in "8 16" "16 16" "10 16 16 1024" "10 16 4 4096" "12 16" "9 16"; do
  timeout -k 10 300 python scripts/mc_kt_diag.py $args >> $O/mc_kt.txt 2>&1 || { tail -20 $O/mc_kt.txt; exit 3; }
done
grep -v amdgpu.ids $O/mc_kt.txt
