#!/bin/bash
# Device-ingest headline: CUs kept free of the next round's prep (--scan-cus) and the
# price of the cross-stream wait (scripts/devgap_probe.py, measurement only).
set -e
O=gpurun_out/r5/devgap2
mkdir -p $O
A="--steps 100 --warmup 10 --ingest device --engine-e2e 0 --engine-latency 0 --latency-samples 0"
for C in 0 48 64 96; do
  timeout -k 10 200 python bench.py $A --scan-cus $C > $O/base_c$C.json 2> $O/base_c$C.err
done
timeout -k 10 200 python scripts/devgap_probe.py $A --scan-cus 64 > $O/nowait_c64.json 2> $O/nowait_c64.err
timeout -k 10 200 python scripts/devgap_probe.py $A > $O/nowait_c0.json 2> $O/nowait_c0.err
