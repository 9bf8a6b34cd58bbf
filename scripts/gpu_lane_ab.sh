#!/bin/bash
# Ingest lanes under the copy: kernel times of the training chain with the copy on a
# 16-CU block and training on the other CUs ("split") vs plain streams ("plain").
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export TMPDIR=/tmp
for ln in split plain; do
  rm -rf gpurun_out/lane_$ln
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lane_$ln -o run -- python3 bench.py --lane $ln --steps 200 --warmup 20 --latency-samples 10 > gpurun_out/lane_$ln.json 2> gpurun_out/lane_$ln.err || { tail -5 gpurun_out/lane_$ln.err; exit 3; }
  python3 - $ln <<'PY'
import csv, json, sys
ln = sys.argv[1]
d = json.loads(open(f"gpurun_out/lane_{ln}.json").read().strip().splitlines()[-1])
out = [f"{ln}: {d['ms_per_step']} ms/step"]
for r in csv.DictReader(open(f"gpurun_out/lane_{ln}/run_kernel_stats.csv")):
    n = r["Name"]
    for k in ("round_rd", "reduce_kernel", "apply_kernel", "pull_copy"):
        if k in n:
            out.append(f"{k} {float(r['AverageNs'])/1e3:.1f}")
print("  ".join(out))
PY
done
