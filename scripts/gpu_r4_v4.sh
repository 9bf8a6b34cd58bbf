#!/bin/bash
# no-spill helper loop (precise vmcnt waits) + Grams beside the flags pass: probe, numerics,
# headline A/B, kernel trace
mkdir -p gpurun_out/r4
timeout -k 10 120 python scripts/scan3_probe.py > gpurun_out/r4/probe4.json 2>gpurun_out/r4/probe4.err || exit 3
head -c 420 gpurun_out/r4/probe4.json; echo
timeout -k 10 300 python -u -m pytest tests/test_scan3.py tests/test_rawwire.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/v4_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r4/v4_tests.txt; [ $rc -eq 0 ] || exit 4
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 "$@" > gpurun_out/r4/b4_$n.json 2> gpurun_out/r4/b4_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/b4_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b def X=1 || exit 5
b nosplit OMLDM_S3_PREP_SPLIT=0 --ref off --latency-samples 0 || exit 6
b s4 X=1 --slots 4 --ref off --latency-samples 0 || exit 7
b k0 X=1 --scan-cus 0 --ref off --latency-samples 0 || exit 8
b dev X=1 --ingest device --pool 6 --ref off --latency-samples 0 || exit 9
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_v4 -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_v4.log 2>&1 || exit 10
python scripts/trace_timeline.py $(find gpurun_out/r4/prof_v4 -name "*kernel_trace.csv" | head -1) --last 24 | cut -c1-100
