#!/bin/bash
# copies two batches ahead of the round (the pipeline stays primed across the warmup sync)
mkdir -p gpurun_out/r4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/bp_$n.json 2> gpurun_out/r4/bp_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bp_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b a2 || exit 3
b a1 --ahead 1 --ref off || exit 4
b a2b --ref off || exit 5
b a1b --ahead 1 --ref off || exit 6
b s40 --ref off --steps 40 || exit 7
b a2_100 --ref off --steps 100 || exit 8
