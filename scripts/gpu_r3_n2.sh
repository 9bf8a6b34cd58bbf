#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
OMLDM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r3_bench2_full.json 2> gpurun_out/r3_bench2_full.err || { tail -30 gpurun_out/r3_bench2_full.err; exit 8; }
cat gpurun_out/r3_bench2_full.json
