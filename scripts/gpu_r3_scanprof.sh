#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_scanprof -o run -- python3 $GRAFT_REPO_ROOT/scripts/scan_ab.py > $GRAFT_REPO_ROOT/gpurun_out/r3_scanprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_scanprof.log; exit 6; }
find $GRAFT_REPO_ROOT/gpurun_out/r3_scanprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
