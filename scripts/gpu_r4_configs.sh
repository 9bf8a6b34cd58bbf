#!/bin/bash
# BASELINE configs 2, 4, 5 on one GPU at the round's kernels (exact semantics)
set -u
mkdir -p gpurun_out/r4
timeout -k 10 300 python bench.py --learner LogisticRegression --engine-e2e 0 --engine-latency 0 --latency-samples 200 > gpurun_out/r4/config2_logreg.json 2> gpurun_out/r4/config2_logreg.err || { echo c2 failed; tail -5 gpurun_out/r4/config2_logreg.err; exit 3; }
tail -c 700 gpurun_out/r4/config2_logreg.json; echo
timeout -k 10 300 python bench/orr_fgm.py > gpurun_out/r4/config4_orr_fgm.json 2> gpurun_out/r4/config4_orr_fgm.err || { echo c4 failed; tail -5 gpurun_out/r4/config4_orr_fgm.err; exit 4; }
tail -c 900 gpurun_out/r4/config4_orr_fgm.json; echo
timeout -k 10 300 python bench/multi_pipeline.py --mode exact --pipelines 16 --steps 20 --warmup 3 > gpurun_out/r4/config5_multi_exact.json 2> gpurun_out/r4/config5_multi_exact.err || { echo c5 failed; tail -5 gpurun_out/r4/config5_multi_exact.err; exit 5; }
tail -c 1200 gpurun_out/r4/config5_multi_exact.json; echo
timeout -k 10 300 python bench/multi_pipeline.py --mode exact --pipelines 4 --steps 20 --warmup 3 --latency-samples 200 > gpurun_out/r4/config5_multi_exact_m4.json 2> gpurun_out/r4/config5_multi_exact_m4.err || { echo c5b failed; tail -5 gpurun_out/r4/config5_multi_exact_m4.err; exit 6; }
tail -c 600 gpurun_out/r4/config5_multi_exact_m4.json; echo
