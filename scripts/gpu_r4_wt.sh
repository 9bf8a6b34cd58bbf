#!/bin/bash
# write-through pull copy vs plain stores, copy CU layouts, CUs kept for the scan
mkdir -p gpurun_out/r4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 "$@" > gpurun_out/r4/bw_$n.json 2> gpurun_out/r4/bw_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bw_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'])"
}
b warm --steps 5 || exit 3
b wt_k0 --scan-cus 0 || exit 4
b pl_k0 --scan-cus 0 --pull-wt 0 || exit 5
b wt_k16 || exit 6
b pl_k16 --pull-wt 0 || exit 7
b wt_lay0k0 --cu-layout 0 --scan-cus 0 || exit 8
b wt_k0b --scan-cus 0 || exit 9
b pl_k0b --scan-cus 0 --pull-wt 0 || exit 10
b wt_k0_i8 --scan-cus 0 --ingest-cus 8 || exit 11
b wt_k0_s4 --scan-cus 0 --slots 4 || exit 12
for f in dib json; do
  timeout -k 10 240 python bench/engine_e2e.py --records 4000000 --batch 131072 --format $f > gpurun_out/r4/e2e_$f.json 2> gpurun_out/r4/e2e_$f.err || exit 13
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$f.json').read().strip().splitlines()[-1])
st=d.get('stages_ms',{}); print('$f', d['value'], d.get('record_bytes'), d.get('wall_s'), {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})"
done
