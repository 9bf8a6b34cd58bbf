#!/bin/bash
# End-to-end engine + learners benches (1 GPU).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench/engine_e2e.py --records ${E2E_RECORDS:-4000000} --batch ${E2E_BATCH:-65536} > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
if [ -n "${LEARNERS:-}" ]; then
  timeout -k 10 300 python bench/learners.py > gpurun_out/learners.json 2> gpurun_out/learners.err || { tail -20 gpurun_out/learners.err; exit 2; }
  cat gpurun_out/learners.json
fi
if [ -n "${FORECAST:-}" ]; then
  timeout -k 10 300 python bench/engine_e2e.py --records 4000000 --batch 65536 --forecast-frac $FORECAST > gpurun_out/e2e_fc.json 2> gpurun_out/e2e_fc.err || { tail -20 gpurun_out/e2e_fc.err; exit 3; }
  cat gpurun_out/e2e_fc.json
fi
