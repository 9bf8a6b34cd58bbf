#!/bin/bash
# BASELINE config 2 (logistic regression, bf16 model, 2^20 hashed features): pinned-host
# stream and HBM-resident ingest.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 240 python bench.py --learner LogisticRegression --steps 200 --warmup 20 > gpurun_out/cfg2_pinned.json 2> gpurun_out/cfg2_pinned.err || { tail -20 gpurun_out/cfg2_pinned.err; exit 3; }
timeout -k 10 240 python bench.py --learner LogisticRegression --ingest device --steps 200 --warmup 20 > gpurun_out/cfg2_device.json 2> gpurun_out/cfg2_device.err || { tail -20 gpurun_out/cfg2_device.err; exit 3; }
cat gpurun_out/cfg2_pinned.json gpurun_out/cfg2_device.json
