#!/bin/bash
# engine e2e: persistent reader pool vs a thread per reader per block, alternated
mkdir -p gpurun_out/r4
e() {  # name, env, args
  n=$1; v=$2; shift 2
  env $v timeout -k 10 240 python bench/engine_e2e.py "$@" > gpurun_out/r4/e2e_$n.json 2> gpurun_out/r4/e2e_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$n.json').read().strip().splitlines()[-1])
st=d.get('stages_ms',{}); print('$n', d['value'], {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if k.startswith('ingest_')})"
}
for r in 1 2; do
  e dpool$r OMLDM_READ_POOL=1 --records 8000000 --batch 131072 --format dib || exit 3
  e dthr$r OMLDM_READ_POOL=0 --records 8000000 --batch 131072 --format dib || exit 4
  e jpool$r OMLDM_READ_POOL=1 --records 4000000 --batch 131072 --format json || exit 5
  e jthr$r OMLDM_READ_POOL=0 --records 4000000 --batch 131072 --format json || exit 6
done
