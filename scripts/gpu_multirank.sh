#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo; the driver runs the real N-GPU RCCL scaling).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_multirank_gpu.py -m gpu -q -x > gpurun_out/pytest_multirank.log 2>&1 || { tail -30 gpurun_out/pytest_multirank.log; exit 2; }
tail -1 gpurun_out/pytest_multirank.log
OMLDM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus 2 --steps 10 --warmup 2 --latency-samples 50 > gpurun_out/bench_2rank.log 2>&1 || { tail -30 gpurun_out/bench_2rank.log; exit 3; }
tail -1 gpurun_out/bench_2rank.log
