#!/bin/bash
# Round 3: v2 scan kernel — numerics vs CPU (both kernels), the A/B timing, the headline
# bench (pinned + device-resident) with a kernel trace, then this round's new GPU tests.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rawwire.py -m gpu > gpurun_out/r3_scan_tests.log 2>&1 || { tail -60 gpurun_out/r3_scan_tests.log; exit 3; }
tail -3 gpurun_out/r3_scan_tests.log
timeout -k 10 200 python scripts/scan_ab.py > gpurun_out/r3_scan_ab.json 2> gpurun_out/r3_scan_ab.err || { tail -30 gpurun_out/r3_scan_ab.err; exit 4; }
cat gpurun_out/r3_scan_ab.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-samples 500 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -30 gpurun_out/r3_bench.err; exit 6; }
cat gpurun_out/r3_bench.json
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --latency-samples 10 --engine-latency 0 --engine-e2e 0 --ingest device --ref off > gpurun_out/r3_bench_dev.json 2> gpurun_out/r3_bench_dev.err || { tail -30 gpurun_out/r3_bench_dev.err; exit 7; }
cat gpurun_out/r3_bench_dev.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --latency-samples 10 --ref off --engine-latency 0 --engine-e2e 0 > $GRAFT_REPO_ROOT/gpurun_out/r3_prof2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_prof2.log; exit 8; }
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_forecast_server_gpu.py tests/test_no_host_sync_gpu.py -m gpu > gpurun_out/r3_new_tests.log 2>&1 || { tail -60 gpurun_out/r3_new_tests.log; exit 5; }
tail -8 gpurun_out/r3_new_tests.log
