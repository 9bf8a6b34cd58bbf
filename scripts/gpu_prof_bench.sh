#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the default headline bench, summarised.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 100 ${BENCH_ARGS:-} > $R/gpurun_out/prof_bench.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 5; }
cd $R && python scripts/trace_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && tail -20 gpurun_out/prof_bench_summary.txt
