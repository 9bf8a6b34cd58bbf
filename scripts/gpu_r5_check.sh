#!/bin/bash
# Round-5 GPU check: default bench, config-5 multi-pipeline (fused / per-stream), GPU suite.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out/r5
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_default.json 2> gpurun_out/r5/bench_default.err
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 16 > gpurun_out/r5/config5_fused_m16.json 2> gpurun_out/r5/config5_fused_m16.err
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 16 --fused 0 --ref 0 > gpurun_out/r5/config5_streams_m16.json 2> gpurun_out/r5/config5_streams_m16.err
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 4 > gpurun_out/r5/config5_fused_m4.json 2> gpurun_out/r5/config5_fused_m4.err
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r5/gpu_suite.txt 2>&1
