#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b15; mkdir -p $O
timeout -k 10 400 python -u scripts/e2e_dib_diag.py json dib dib > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 3; }
grep -v amdgpu.ids $O/diag.txt
timeout -k 10 400 python -u scripts/e2e_dib_diag.py dib json > $O/diag2.txt 2>&1 || { tail -20 $O/diag2.txt; exit 3; }
grep -v amdgpu.ids $O/diag2.txt
