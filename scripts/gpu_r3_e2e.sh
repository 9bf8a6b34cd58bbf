#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for fs in false auto; do
timeout -k 10 300 python bench/engine_e2e.py --records 2000000 --batch 131072 --forecast-server $fs > gpurun_out/r3_e2e_16_$fs.json 2> gpurun_out/r3_e2e_16_$fs.err || { tail -20 gpurun_out/r3_e2e_16_$fs.err; exit 3; }
cat gpurun_out/r3_e2e_16_$fs.json
done
