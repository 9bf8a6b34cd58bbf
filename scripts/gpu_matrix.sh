#!/bin/bash
# Engine configuration matrix on the GPU (tests/test_matrix.py, 64 cases).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_matrix.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/matrix_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/matrix_gpu.log; exit $rc
