#!/bin/bash
# In-scan combine (OMLDM_S3_INSCAN: 1 auto = when the combiners' grid exceeds one workgroup
# per CU, 0 never, 2 always) across pipeline counts, the device-ingest headline, tests.
set -e
O=gpurun_out/r5/inscan4
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan3.py tests/test_multi_pipeline_gpu.py > $O/tests.txt 2>&1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --ingest device --engine-e2e 0 --engine-latency 0 --latency-samples 0 > $O/dev_i1.json 2> $O/dev_i1.err
for M in 16 8 6 4; do
  for I in 1 0; do
    OMLDM_S3_INSCAN=$I timeout -k 10 200 python bench/multi_pipeline.py --pipelines $M > $O/m${M}_i$I.json 2> $O/m${M}_i$I.err
  done
done
