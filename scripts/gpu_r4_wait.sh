#!/bin/bash
mkdir -p gpurun_out/r4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/bq_$n.json 2> gpurun_out/r4/bq_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bq_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b a || exit 3
b b --ref off || exit 4
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_wait -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_wait.log 2>&1 || exit 8
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_wait -name "*kernel_trace.csv" | head -1) --last 22 | cut -c1-100
