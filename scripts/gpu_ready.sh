#!/bin/bash
# The prep's ready word (OMLDM_S3_READY=1, default) vs the cross-stream event wait (0):
# device-ingest and pinned headline, config 5, and the tests that run preps made ahead.
set -e
O=gpurun_out/r5/ready
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan3.py tests/test_multi_pipeline_gpu.py tests/test_round_split.py tests/test_engine_defaults_gpu.py > $O/tests.txt 2>&1
A="--steps 100 --warmup 10 --engine-e2e 0 --engine-latency 0 --latency-samples 0"
for R in 1 0; do
  OMLDM_S3_READY=$R timeout -k 10 200 python bench.py $A --ingest device > $O/dev_r$R.json 2> $O/dev_r$R.err
  OMLDM_S3_READY=$R timeout -k 10 200 python bench.py $A > $O/pinned_r$R.json 2> $O/pinned_r$R.err
done
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 16 > $O/m16.json 2> $O/m16.err
