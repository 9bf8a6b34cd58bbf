#!/bin/bash
# staging depth (the copy of batch k+slots waits for round k's slot) and prep variants
mkdir -p gpurun_out/r4
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 "$@" > gpurun_out/r4/bs_$n.json 2> gpurun_out/r4/bs_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bs_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'])"
}
b s3 X=1 --slots 3 || exit 3
b s4 X=1 --slots 4 || exit 4
b s6 X=1 --slots 6 || exit 5
b s6k0 X=1 --slots 6 --scan-cus 0 || exit 6
b s6k32 X=1 --slots 6 --scan-cus 32 || exit 7
b s6valu OMLDM_S3_GRAM_VALU=1 --slots 6 || exit 8
b s6dev X=1 --slots 6 --ingest device --pool 6 || exit 9
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_s6 -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 --slots 6 > gpurun_out/r4/prof_s6.log 2>&1 || exit 10
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_s6 -name "*kernel_trace.csv" | head -1) --last 30 | cut -c1-100
