#!/bin/bash
# Device-ingest headline: CUs kept off the prep stream for the scan (--scan-cus).
set -e
mkdir -p gpurun_out/r5/scancus
for c in 0 32 48 64 96; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --ingest device --engine-e2e 0 --engine-latency 0 --latency-samples 0 --ref off --scan-cus $c > gpurun_out/r5/scancus/dev_$c.json 2> gpurun_out/r5/scancus/dev_$c.err
done
for c in 0 48; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --engine-e2e 0 --engine-latency 0 --latency-samples 0 --ref off --scan-cus $c > gpurun_out/r5/scancus/pin_$c.json 2> gpurun_out/r5/scancus/pin_$c.err
done
