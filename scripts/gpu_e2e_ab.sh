#!/bin/bash
# Engine end-to-end A/B (records/s of JSON and DIB topics through the whole engine).
# Each tag is a comma-separated list of VAR=value settings (empty tag: defaults);
# E2E_BATCH sets the records per tick.
set -e
mkdir -p gpurun_out/r5
for tag in "$@"; do
  name=$(echo "$tag" | tr '=,-' '___')
  env $(echo "$tag" | tr ',' ' ') bash -c 'timeout -k 10 200 python bench.py --steps 3 --warmup 1 --latency-samples 0 --engine-latency 0 --ref off --e2e-batch ${E2E_BATCH:-524288}' > gpurun_out/r5/e2e_${name}.json 2> gpurun_out/r5/e2e_${name}.err
done
