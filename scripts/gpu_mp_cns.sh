#!/bin/bash
# Multi-pipeline: spokes per combiner workgroup (OMLDM_S3_CNS), latency form.
set -e
mkdir -p gpurun_out/r5
for c in 1 2 4; do
  for m in 16 8; do
    OMLDM_S3_CNS=$c timeout -k 10 200 python bench/multi_pipeline.py --pipelines $m > gpurun_out/r5/mp_cns${c}_m${m}.json 2> gpurun_out/r5/mp_cns${c}_m${m}.err
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_multi_pipeline_gpu.py > gpurun_out/r5/t_mp.txt 2>&1
