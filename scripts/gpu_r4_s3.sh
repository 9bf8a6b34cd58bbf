#!/bin/bash
# Round 4: v3 table-scan tests, v2 vs v3 headline A/B, kernel trace of v3.
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_scan3.py tests/test_holdout_gpu.py tests/test_kmeans_seq.py tests/test_forecast_server_gpu.py tests/test_rawwire.py tests/test_async_protocols.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/scan3_tests.txt 2>&1
rc=$?; tail -15 gpurun_out/r4/scan3_tests.txt; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.txt 2>&1 || exit 9
OMLDM_SEQ_KERNEL=scan timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 > gpurun_out/r4/bench_v2.json 2> gpurun_out/r4/bench_v2.err || exit 5
timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 > gpurun_out/r4/bench_v3.json 2> gpurun_out/r4/bench_v3.err || exit 6
python - <<'PY'
import json
for n in ("bench_v2", "bench_v3"):
    d = json.loads(open(f"gpurun_out/r4/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d.get("holdout_accuracy"), d.get("ref_holdout_accuracy"), d.get("accuracy_gap_pt"), d.get("round_kernel"))
PY
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_v3 -o prof -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_v3.log 2>&1 || exit 8
f=$(find gpurun_out/r4/prof_v3 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r4/v3_kernel_stats.csv
head -20 gpurun_out/r4/v3_kernel_stats.csv
