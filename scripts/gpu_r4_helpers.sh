#!/bin/bash
# helpers: dense columns owned in reverse field order, margins read the table before writing: numerics, probe, headline
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_scan3.py tests/test_rawwire.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/helpers_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/helpers_tests.txt; [ $rc -eq 0 ] || exit 3
timeout -k 10 120 python scripts/scan3_probe.py > gpurun_out/r4/probe6.json 2>gpurun_out/r4/probe6.err || exit 4
head -c 300 gpurun_out/r4/probe6.json; echo
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/bh_$n.json 2> gpurun_out/r4/bh_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bh_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b a || exit 5
b b --ref off || exit 6
b c --ref off --steps 100 || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_helpers -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_helpers.log 2>&1 || exit 8
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_helpers -name "*kernel_trace.csv" | head -1) --last 22 | cut -c1-100
