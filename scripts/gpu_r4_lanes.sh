#!/bin/bash
# CU-mask bit -> XCD map, then the headline's lane layout sweep (copy CUs, their layout, CUs
# kept for the scan)
mkdir -p gpurun_out/r4
PYTHONPATH=. timeout -k 10 120 python scripts/cumask_probe.py || exit 3
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 "$@" > gpurun_out/r4/bl_$n.json 2> gpurun_out/r4/bl_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bl_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'])"
}
b base || exit 4
b k0 --scan-cus 0 || exit 5
b lay0 --cu-layout 0 || exit 6
b lay0k0 --cu-layout 0 --scan-cus 0 || exit 7
b i8 --ingest-cus 8 || exit 8
b i32 --ingest-cus 32 || exit 9
b i32k0 --ingest-cus 32 --scan-cus 0 || exit 10
b plain --lane plain || exit 11
b base2 || exit 12
