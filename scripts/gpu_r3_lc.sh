#!/bin/bash
# Engine e2e after the per-tick learning-curve read became lagged (no host sync per tick).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 131072 65536; do
  timeout -k 10 120 python bench/engine_e2e.py --records 8000000 --batch $b > gpurun_out/lc_e2e_$b.json 2> gpurun_out/lc_e2e_$b.err || { tail -20 gpurun_out/lc_e2e_$b.err; exit 5; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['wall_s'], d['ticks_timed'])" gpurun_out/lc_e2e_$b.json $b
done
timeout -k 10 120 python bench/engine_e2e.py --records 8000000 --batch 131072 --forecast-frac 0.002 > gpurun_out/lc_e2e_fc.json 2> gpurun_out/lc_e2e_fc.err || { tail -20 gpurun_out/lc_e2e_fc.err; exit 6; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('fc', d['value'], d['forecast_lane'])" gpurun_out/lc_e2e_fc.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lc_gpu_tests.log 2>&1 || { tail -60 gpurun_out/lc_gpu_tests.log; exit 7; }
tail -2 gpurun_out/lc_gpu_tests.log
