#!/bin/bash
# NN round kernels under rocprofv3 --kernel-trace (fp32 and bf16 operands, learner bench).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
CASES='[["NN",0,{"hiddenLayers":[64,64]},512],["NN@bf16",0,{"hiddenLayers":[64,64],"matmulDtype":"bf16"},512]]'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nn -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 50 > $R/gpurun_out/prof_nn.log 2>&1 || { tail -20 $R/gpurun_out/prof_nn.log; exit 5; }
cd $R && python scripts/trace_summary.py gpurun_out/prof_nn mlp_round > gpurun_out/prof_nn_summary.txt; head -20 gpurun_out/prof_nn_summary.txt; tail -3 gpurun_out/prof_nn.log
