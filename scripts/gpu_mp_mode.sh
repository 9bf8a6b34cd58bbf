#!/bin/bash
# Config 5 A/B: round mode 3 (the scan workgroup's helpers gather w0: no w0-margin
# workgroups, 32 workgroups per pipeline) vs mode 4 (48 per pipeline) at M = 16 / 8 / 1.
set -e
O=gpurun_out/r5/mpmode2
mkdir -p $O
for M in 16 12 8 1; do
  for MODE in 3 4; do
    OMLDM_S3_MODE=$MODE timeout -k 10 200 python bench/multi_pipeline.py --pipelines $M > $O/mode${MODE}_m$M.json 2> $O/mode${MODE}_m$M.err
  done
done
