#!/bin/bash
# One apply launch for the pipelines of a fused round: tests and config 5.
set -e
O=gpurun_out/r5/applym
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_multi_pipeline_gpu.py tests/test_matrix.py -k "multi or Multi or SVM" > $O/tests.txt 2>&1
for M in 16 8 4; do
  timeout -k 10 200 python bench/multi_pipeline.py --pipelines $M > $O/m$M.json 2> $O/m$M.err
done
