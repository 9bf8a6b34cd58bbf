#!/bin/bash
# Round-5 numbers for profiles/round5: headline (pinned + device ingest), config 2 / 5,
# the engine end to end, and a kernel-trace summary of the headline. Each GPU step has its
# own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out/r5/final
O=gpurun_out/r5/final
timeout -k 10 400 python bench.py --steps 100 --warmup 10 > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --ingest device --engine-e2e 0 --engine-latency 0 --latency-samples 0 > $O/bench_device.json 2> $O/bench_device.err
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --learner LogisticRegression --engine-e2e 0 --engine-latency 0 --latency-samples 0 > $O/config2_logreg.json 2> $O/config2_logreg.err
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 16 > $O/config5_m16.json 2> $O/config5_m16.err
timeout -k 10 200 python bench/multi_pipeline.py --pipelines 4 > $O/config5_m4.json 2> $O/config5_m4.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 50 --warmup 5 --engine-e2e 0 --engine-latency 0 --latency-samples 0 --ref off > $O/prof_bench.out 2>&1
