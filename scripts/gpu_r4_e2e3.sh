#!/bin/bash
# engine e2e with the SIMD record indexer
mkdir -p gpurun_out/r4
e() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench/engine_e2e.py "$@" > gpurun_out/r4/e2e_$n.json 2> gpurun_out/r4/e2e_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$n.json').read().strip().splitlines()[-1])
st=d.get('stages_ms',{}); print('$n', d['value'], d.get('wall_s'), d.get('ticks_timed'), {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})"
}
e dibS --records 8000000 --batch 131072 --format dib --partitions 8 || exit 4
e dibS16 --records 8000000 --batch 131072 --format dib --partitions 16 || exit 5
e jsonS --records 4000000 --batch 131072 --format json --partitions 8 || exit 6
e jsonS16 --records 4000000 --batch 131072 --format json --partitions 16 || exit 7
