#!/bin/bash
# two-rank rehearsal of the bench's multi-GPU path (both ranks on the one GPU, gloo),
# with the engine measurements on (rank-local communicator)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
OMLDM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --latency-samples 200 --engine-e2e 262144 > gpurun_out/r4/bench2.json 2> gpurun_out/r4/bench2.err || { tail -30 gpurun_out/r4/bench2.err; exit 8; }
tail -c 2500 gpurun_out/r4/bench2.json
