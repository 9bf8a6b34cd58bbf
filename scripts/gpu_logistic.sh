#!/bin/bash
# The logistic chain on ρ with lr·y in the Grams' columns: tests and BASELINE config 2.
set -e
O=gpurun_out/r5/logistic
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan3.py tests/test_engine_defaults_gpu.py -k "LOGISTIC or logistic or Logistic or rare_workgroup or shrinking or prep_matches" > $O/tests.txt 2>&1
A="--steps 50 --warmup 10 --learner LogisticRegression --engine-e2e 0 --engine-latency 0 --latency-samples 0"
timeout -k 10 200 python bench.py $A > $O/config2.json 2> $O/config2.err
timeout -k 10 200 python bench.py $A --ingest device > $O/config2_device.json 2> $O/config2_device.err
timeout -k 10 200 python bench.py $A --model-dtype bf16 > $O/config2_bf16.json 2> $O/config2_bf16.err
