#!/bin/bash
# Training throughput with forecasts flowing on the resident serving wave: does the
# persistent wave's hardware queue stall the training streams, and do more HW queues help?
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env, args
  local tag=$1; shift
  env "$@" > "gpurun_out/hwq_$tag.json" 2> "gpurun_out/hwq_$tag.err" || { tail -20 "gpurun_out/hwq_$tag.err"; exit 5; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['predictions'], d['forecast_lane'], d['wall_s'])" "gpurun_out/hwq_$tag.json" "$tag"
}
E="timeout -k 10 120 python bench/engine_e2e.py --records 8000000 --batch 131072"
run base    OMLDM_X=0 $E --forecast-frac 0
run fc_q4   OMLDM_X=0 $E --forecast-frac 0.002
run fc_q8   GPU_MAX_HW_QUEUES=8 $E --forecast-frac 0.002
run base_q8 GPU_MAX_HW_QUEUES=8 $E --forecast-frac 0
run fc_off  OMLDM_X=0 $E --forecast-frac 0.002 --forecast-server false
