#!/bin/bash
# engine e2e after the native block fill + one-launch staging copy
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_json_gpu.py tests/test_ingest_pipeline.py tests/test_engine.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/e2e2_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/e2e2_tests.txt; [ $rc -eq 0 ] || exit 3
e() {  # name, env, args
  n=$1; v=$2; shift 2
  env $v timeout -k 10 240 python bench/engine_e2e.py "$@" > gpurun_out/r4/e2e_$n.json 2> gpurun_out/r4/e2e_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$n.json').read().strip().splitlines()[-1])
st=d.get('stages_ms',{}); print('$n', d['value'], d.get('wall_s'), d.get('ticks_timed'), {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})"
}
e dibN X=1 --records 8000000 --batch 131072 --format dib --partitions 8 || exit 4
e dibP OMLDM_NATIVE_FILL=0 --records 8000000 --batch 131072 --format dib --partitions 8 || exit 5
e dibN16 X=1 --records 8000000 --batch 131072 --format dib --partitions 16 || exit 6
e jsonN X=1 --records 4000000 --batch 131072 --format json --partitions 8 || exit 7
e dibN65 X=1 --records 4000000 --batch 65536 --format dib --partitions 8 || exit 8
