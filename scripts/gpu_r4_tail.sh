#!/bin/bash
# the round's tail in the scan's launch (last scan block): numerics, headline A/B, trace
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_scan3.py tests/test_rawwire.py tests/test_linear.py tests/test_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/tail_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/tail_tests.txt; [ $rc -eq 0 ] || exit 3
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/bt_$n.json 2> gpurun_out/r4/bt_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bt_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b inl X=1 || exit 4
b ker OMLDM_S3_TAIL=kernel --ref off || exit 5
b inl2 X=1 --ref off || exit 6
b ker2 OMLDM_S3_TAIL=kernel --ref off || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_tail -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_tail.log 2>&1 || exit 8
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_tail -name "*kernel_trace.csv" | head -1) --last 16 | cut -c1-100
