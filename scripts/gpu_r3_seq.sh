#!/bin/bash
# Round 3: raw-wire Gram-scan kernel — numerics vs CPU, then the headline bench + profile.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rawwire.py -m gpu > gpurun_out/r3_rawwire.log 2>&1 || { tail -40 gpurun_out/r3_rawwire.log; exit 3; }
tail -3 gpurun_out/r3_rawwire.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --latency-samples 500 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -30 gpurun_out/r3_bench.err; exit 4; }
cat gpurun_out/r3_bench.json
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --latency-samples 10 --ingest device --ref off > gpurun_out/r3_bench_dev.json 2> gpurun_out/r3_bench_dev.err || { tail -30 gpurun_out/r3_bench_dev.err; exit 5; }
cat gpurun_out/r3_bench_dev.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --latency-samples 10 --ref off > $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log; exit 6; }
find $GRAFT_REPO_ROOT/gpurun_out/r3_prof -name "*kernel_stats.csv" | head -1 | xargs head -20
