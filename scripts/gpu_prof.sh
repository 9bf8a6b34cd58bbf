#!/bin/bash
# rocprofv3 kernel trace of the bench (device-resident and pinned ingest).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for mode in device pinned; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_$mode -o run -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 50 --ingest $mode ${BENCH_ARGS:-} > $R/gpurun_out/prof_$mode.log 2>&1 || { echo "prof $mode failed"; tail -20 $R/gpurun_out/prof_$mode.log; exit 5; }
  tail -1 $R/gpurun_out/prof_$mode.log | cut -c1-200
done
