#!/bin/bash
# Round 6: the whole GPU suite (every failure listed, not just the first).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/r6/suite
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=8 -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/suite/pytest_gpu.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/suite/pytest_gpu.txt | tail -20
exit $rc
