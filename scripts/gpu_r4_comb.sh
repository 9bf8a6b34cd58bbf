#!/bin/bash
# in-launch combine: numerics (A/B against the scatter kernel, oracle tests), then the
# headline bench with the combine in the scan's launch vs after it, and a kernel trace
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_scan3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/comb_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r4/comb_tests.txt; [ $rc -eq 0 ] || exit 3
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 "$@" > gpurun_out/r4/bcomb_$n.json 2> gpurun_out/r4/bcomb_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bcomb_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b comb1 OMLDM_S3_COMB=1 || exit 5
b comb0 OMLDM_S3_COMB=0 --ref off --latency-samples 0 || exit 6
b comb2 OMLDM_S3_COMB=2 --ref off --latency-samples 0 || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_comb -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_comb.log 2>&1 || exit 8
f=$(find gpurun_out/r4/prof_comb -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r4/comb_kernel_stats.csv && cut -c1-150 gpurun_out/r4/comb_kernel_stats.csv | head -14
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_comb -name "*kernel_trace.csv" | head -1) --last 16 | cut -c1-110
