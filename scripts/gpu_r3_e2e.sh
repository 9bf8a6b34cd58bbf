#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for fs in false auto; do
timeout -k 10 300 python bench/engine_e2e.py --records 2000000 --batch 131072 --forecast-server $fs > gpurun_out/r3_e2e_16_$fs.json 2> gpurun_out/r3_e2e_16_$fs.err || { tail -20 gpurun_out/r3_e2e_16_$fs.err; exit 3; }
cat gpurun_out/r3_e2e_16_$fs.json
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_forecast_server_gpu.py -m gpu > gpurun_out/r3_fs_tests.log 2>&1 || { tail -40 gpurun_out/r3_fs_tests.log; exit 5; }
tail -4 gpurun_out/r3_fs_tests.log
