#!/bin/bash
# Reducer hot-key aggregation A/B (OMLDM_REDUCE_HOT = lanes that must share a key; 65 =
# off): linear GPU tests, then the device-resident headline step and its kernel times.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linear.py tests/test_compact_wire.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_lin.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_lin.log; [ $rc -eq 0 ] || exit $rc
for h in 65 4 2 8 65 4; do
  rm -rf gpurun_out/hot_$h
  OMLDM_REDUCE_HOT=$h timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hot_$h -o run -- python3 bench.py --ingest device --steps 200 --warmup 20 --latency-samples 10 > gpurun_out/hot_$h.json 2> gpurun_out/hot_$h.err || { tail -5 gpurun_out/hot_$h.err; exit 3; }
  python3 - $h <<'PY'
import csv, json, sys
h = sys.argv[1]
d = json.loads(open(f"gpurun_out/hot_{h}.json").read().strip().splitlines()[-1])
out = [f"hot={h}: {d['ms_per_step']} ms/step"]
for r in csv.DictReader(open(f"gpurun_out/hot_{h}/run_kernel_stats.csv")):
    if "linear_reduce" in r["Name"] or "round_rd" in r["Name"]:
        out.append(f"{r['Name'][:30]} {float(r['AverageNs'])/1e3:.1f}")
print("  ".join(out))
PY
done
