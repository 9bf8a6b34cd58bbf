#!/bin/bash
# Whole GPU suite, then a 4-rank gloo rehearsal of the bench on one GPU.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
OMLDM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NR:-4} --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus ${NR:-4} --steps 10 --warmup 2 --latency-samples 50 > gpurun_out/bench_nrank.log 2>&1 || { tail -30 gpurun_out/bench_nrank.log; exit 3; }
tail -1 gpurun_out/bench_nrank.log
