#!/bin/bash
# engine e2e at the final state: forecasts flowing on the per-record lane, and 4 pipelines
mkdir -p gpurun_out/r4
e() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench/engine_e2e.py "$@" > gpurun_out/r4/e2e_$n.json 2> gpurun_out/r4/e2e_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d.get('wall_s'), d.get('pipelines'), d.get('predictions'), d.get('forecast_lane'))"
}
e dib_base --records 8000000 --batch 131072 --format dib || exit 3
e dib_fc --records 8000000 --batch 131072 --format dib --forecast-frac 0.002 || exit 4
e dib_p4 --records 8000000 --batch 131072 --format dib --pipelines 4 || exit 5
e json_fc --records 4000000 --batch 131072 --format json --forecast-frac 0.004 || exit 6
