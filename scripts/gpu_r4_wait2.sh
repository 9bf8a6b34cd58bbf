#!/bin/bash
# diagnostic: what the round's cross-stream wait on its prep costs
mkdir -p gpurun_out/r4
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/bq_$n.json 2> gpurun_out/r4/bq_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bq_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b wait X=1 --ref off || exit 3
b nowait OMLDM_S3_DIAG_NOWAIT=1 --ref off || exit 4
b wait2 X=1 --ref off || exit 5
b nowait2 OMLDM_S3_DIAG_NOWAIT=1 --ref off || exit 6
