#!/bin/bash
# engine e2e: GPU parse on its own stream beside the next block's copy
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_json_gpu.py tests/test_engine.py tests/test_forecast_server_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/e2e4_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/e2e4_tests.txt; [ $rc -eq 0 ] || exit 3
e() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench/engine_e2e.py "$@" > gpurun_out/r4/e2e_$n.json 2> gpurun_out/r4/e2e_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$n.json').read().strip().splitlines()[-1])
st=d.get('stages_ms',{}); print('$n', d['value'], d.get('wall_s'), d.get('ticks_timed'), {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})"
}
e jsonP --records 4000000 --batch 131072 --format json --partitions 8 || exit 4
e dibP2 --records 8000000 --batch 131072 --format dib --partitions 8 || exit 5
e jsonP16 --records 4000000 --batch 131072 --format json --partitions 16 || exit 6
