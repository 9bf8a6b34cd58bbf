#!/bin/bash
# headline bench (v3 default) + kernel trace of the timed loop
mkdir -p gpurun_out/r4
timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 > gpurun_out/r4/bench_v3.json 2> gpurun_out/r4/bench_v3.err || exit 6
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4/bench_v3.json").read().strip().splitlines()[-1])
print("bench_v3", d["value"], d["ms_per_step"], d.get("holdout_accuracy"), d.get("ref_holdout_accuracy"), d.get("accuracy_gap_pt"), d.get("round_kernel"))
PY
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_bench -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_bench.log 2>&1 || exit 8
f=$(find gpurun_out/r4/prof_bench -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r4/bench_kernel_stats.csv && cut -c1-160 gpurun_out/r4/bench_kernel_stats.csv | head -12
