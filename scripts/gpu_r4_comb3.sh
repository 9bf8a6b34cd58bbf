#!/bin/bash
# helpers' margins back on exec-masked LDS paths: probe stamps, numerics, headline A/B
mkdir -p gpurun_out/r4
for c in 1 0; do
  OMLDM_S3_COMB=$c timeout -k 10 120 python scripts/scan3_probe.py > gpurun_out/r4/probe3_comb$c.json 2>gpurun_out/r4/probe3_comb$c.err || exit 3
  echo "comb$c $(head -c 400 gpurun_out/r4/probe3_comb$c.json)"
done
timeout -k 10 300 python -u -m pytest tests/test_scan3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/comb3_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/comb3_tests.txt; [ $rc -eq 0 ] || exit 4
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 "$@" > gpurun_out/r4/b3_$n.json 2> gpurun_out/r4/b3_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/b3_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b c1 OMLDM_S3_COMB=1 || exit 5
b c0 OMLDM_S3_COMB=0 --ref off --latency-samples 0 || exit 6
b c1k32 OMLDM_S3_COMB=1 --scan-cus 32 --ref off --latency-samples 0 || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_comb3 -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_comb3.log 2>&1 || exit 8
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_comb3 -name "*kernel_trace.csv" | head -1) --last 12 | cut -c1-110
