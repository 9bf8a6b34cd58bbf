#!/bin/bash
# Multi-pipeline (BASELINE config 5) A/B: launch forms and pipeline counts.
set -e
mkdir -p gpurun_out/r5
for f in "$@"; do
  for m in 16 8 4 1; do
    OMLDM_S3_FORM=$f timeout -k 10 200 python bench/multi_pipeline.py --pipelines $m --ref 0 > gpurun_out/r5/mp_form${f}_m${m}.json 2> gpurun_out/r5/mp_form${f}_m${m}.err
  done
done
