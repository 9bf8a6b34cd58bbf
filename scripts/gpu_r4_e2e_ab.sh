#!/bin/bash
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_json_gpu.py tests/test_ingest_pipeline.py tests/test_forecast_server_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 4
run() {  # name, env, args...
  n=$1; shift
  timeout -k 10 240 env "$@" > gpurun_out/r4/ab_$n.json 2> gpurun_out/r4/ab_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/ab_$n.json').read().strip().splitlines()[-1])
st=d['stages_ms']; print('$n', d['value'], d['wall_s'], d['ticks_timed'], {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})
"
}
run b131k python bench/engine_e2e.py --records 4000000 --batch 131072 || exit 5
run b65k python bench/engine_e2e.py --records 4000000 --batch 65536 || exit 6
timeout -k 10 200 python scripts/ingest_only_probe.py || exit 7
timeout -k 10 300 python bench/multi_pipeline.py --pipelines 16 --steps 10 --warmup 3 --latency-samples 200 > gpurun_out/r4/multi_exact.json 2> gpurun_out/r4/multi_exact.err && tail -1 gpurun_out/r4/multi_exact.json | cut -c1-700
timeout -k 10 300 python bench/multi_pipeline.py --pipelines 1 --steps 10 --warmup 3 --latency-samples 50 > gpurun_out/r4/multi_exact1.json 2> gpurun_out/r4/multi_exact1.err && tail -1 gpurun_out/r4/multi_exact1.json | cut -c1-300
