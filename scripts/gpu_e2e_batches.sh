#!/bin/bash
# End-to-end engine bench at the three recorded batch sizes (1 GPU), one JSON line each.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
: > gpurun_out/e2e_batches.json
for b in 65536 131072 32768; do
  timeout -k 10 300 python bench/engine_e2e.py --records 4000000 --batch $b >> gpurun_out/e2e_batches.json 2> gpurun_out/e2e_$b.err || { tail -20 gpurun_out/e2e_$b.err; exit 1; }
done
cat gpurun_out/e2e_batches.json
