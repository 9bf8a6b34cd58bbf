#!/bin/bash
# Engine e2e with the training topic in 8 vs 16 partitions (one reader per partition region).
set -e
O=gpurun_out/r5/e2eparts
mkdir -p $O
A="--steps 20 --warmup 5 --engine-latency 0 --latency-samples 0"
for P in 16 8; do
  OMLDM_E2E_PARTS=$P timeout -k 10 400 python bench.py $A > $O/p$P.json 2> $O/p$P.err
done
