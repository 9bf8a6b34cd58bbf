#!/bin/bash
# Kernel trace of the device-ingest headline (the step is the round): per-dispatch start /
# end, to place the scan, the apply and the next round's prep on one timeline.
set -e
O=gpurun_out/r5/devtrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 50 --warmup 10 --ingest device --engine-e2e 0 --engine-latency 0 --latency-samples 0 --ref off > $O/kt.out 2>&1
