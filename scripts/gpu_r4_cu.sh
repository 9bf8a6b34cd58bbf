#!/bin/bash
# scan3 numerics after the branch-free LDS paths + combine changes, the CU-mask → XCD map,
# and the headline bench with / without CUs kept for the scan (trace of the timed loop)
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_scan3.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 3
PYTHONPATH=. timeout -k 10 120 python scripts/cumask_probe.py || exit 4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 "$@" > gpurun_out/r4/bcu_$n.json 2> gpurun_out/r4/bcu_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bcu_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b keep16 || exit 5
b keep0 --scan-cus 0 --ref off --latency-samples 0 || exit 6
b keep32 --scan-cus 32 --ref off --latency-samples 0 || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_bcu -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_bcu.log 2>&1 || exit 8
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_bcu -name "*kernel_trace.csv" | head -1) --last 24 | cut -c1-110
timeout -k 10 200 python -u -m pytest tests/test_json_gpu.py -x -q --timeout 100 --timeout-method thread 2>&1 | tail -2 || exit 9
for f in dib json; do
  timeout -k 10 240 python bench/engine_e2e.py --records 4000000 --batch 131072 --format $f > gpurun_out/r4/e2e_$f.json 2> gpurun_out/r4/e2e_$f.err || exit 10
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$f.json').read().strip().splitlines()[-1])
st=d['stages_ms']; print('$f', d['value'], d['record_bytes'], d['wall_s'], {k: round(v['host_ms']/max(1,v['calls']),2) for k,v in st.items() if v.get('host_ms',0)>1})"
done
