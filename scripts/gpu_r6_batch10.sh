#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b10
mkdir -p $O
timeout -k 10 600 python -u scripts/mc_repeat.py > $O/mc_repeat.txt 2>&1 || { tail -20 $O/mc_repeat.txt; exit 3; }
grep -v amdgpu.ids $O/mc_repeat.txt
