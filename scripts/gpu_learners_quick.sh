#!/bin/bash
# GPU tests of the spoke kernels + learner throughput table (bench/learners.py).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_linear.py tests/test_compact_wire.py tests/test_kernels_dense.py tests/test_serving.py tests/test_multi_pipeline.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/learners.py ${LEARNER_ARGS:-} > gpurun_out/learners.log 2>&1 || { echo learners failed; tail -20 gpurun_out/learners.log; exit 3; }
tail -20 gpurun_out/learners.log
