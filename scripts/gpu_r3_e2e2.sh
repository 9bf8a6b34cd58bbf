#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/engine_e2e.py --records 2000000 --batch 131072 --forecast-server auto > gpurun_out/r3_e2e_lazy.json 2> gpurun_out/r3_e2e_lazy.err || { tail -20 gpurun_out/r3_e2e_lazy.err; exit 3; }
cat gpurun_out/r3_e2e_lazy.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_forecast_server_gpu.py -m gpu > gpurun_out/r3_fs_tests.log 2>&1 || { tail -40 gpurun_out/r3_fs_tests.log; exit 5; }
tail -3 gpurun_out/r3_fs_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --latency-samples 500 --ref off > gpurun_out/r3_bench_lat.json 2> gpurun_out/r3_bench_lat.err || { tail -20 gpurun_out/r3_bench_lat.err; exit 4; }
cat gpurun_out/r3_bench_lat.json
