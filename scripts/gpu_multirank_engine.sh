#!/bin/bash
# Whole-engine two-rank jobs with both ranks on the box's one GPU (gloo between them).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_engine_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/multirank_engine.log 2>&1; rc=$?; tail -40 gpurun_out/multirank_engine.log; exit $rc
