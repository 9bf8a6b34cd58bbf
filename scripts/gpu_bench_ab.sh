#!/bin/bash
# bench.py A/B: each argument is a tag of extra bench flags (commas for spaces).
set -e
mkdir -p gpurun_out/r5
for tag in "$@"; do
  name=$(echo "$tag" | tr '=,-' '___')
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 $(echo "$tag" | tr ',' ' ') > gpurun_out/r5/bab_${name}.json 2> gpurun_out/r5/bab_${name}.err
done
