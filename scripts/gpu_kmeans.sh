#!/bin/bash
# K-means: GPU numerics tests, then the learner bench with the matrix-core assign and
# with the scalar kernel (OMLDM_KMEANS_MFMA=0) for an A/B.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py -m gpu -q -x -k kmeans --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_km.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/learners.py --only K-means > gpurun_out/km_mfma.log 2>&1 || { tail -20 gpurun_out/km_mfma.log; exit 3; }
OMLDM_KMEANS_MFMA=0 timeout -k 10 200 python bench/learners.py --only K-means > gpurun_out/km_scalar.log 2>&1 || { tail -20 gpurun_out/km_scalar.log; exit 3; }
cat gpurun_out/km_mfma.log gpurun_out/km_scalar.log
