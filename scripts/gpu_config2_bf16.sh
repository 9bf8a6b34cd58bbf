#!/bin/bash
# BASELINE config 2 as named: online logistic regression with a bf16 model.
set -e
O=gpurun_out/r5/final
mkdir -p $O
A="--steps 50 --warmup 10 --learner LogisticRegression --engine-e2e 0 --engine-latency 0 --latency-samples 0"
timeout -k 10 200 python bench.py $A --model-dtype bf16 > $O/config2_logreg_bf16.json 2> $O/config2_logreg_bf16.err
timeout -k 10 200 python bench.py $A --model-dtype bf16 --ingest device > $O/config2_logreg_bf16_device.json 2> $O/config2_logreg_bf16_device.err
