#!/bin/bash
# Kernel trace + stats of BASELINE config 5 (16 pipelines, one launch, in-scan combine).
set -e
O=gpurun_out/r5/mptrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench/multi_pipeline.py --pipelines 16 --steps 20 --warmup 5 --ref 0 --latency-samples 0 > $O/kt.out 2>&1
