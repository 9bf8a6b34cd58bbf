#!/bin/bash
# MultiClassPA kernels: GPU tests + learner bench (compact wire rd vs table kernel).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py tests/test_linear.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mc.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_mc.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_mc.log | head -20; exit $rc; }
for rd in 1 0; do
  OMLDM_MC_RD=$rd timeout -k 10 200 python bench/learners.py ${LEARNER_ARGS:-} > gpurun_out/learners_mc$rd.log 2>&1 || { echo learners failed; tail -20 gpurun_out/learners_mc$rd.log; exit 3; }
  echo "rd=$rd: $(tail -1 gpurun_out/learners_mc$rd.log)"
done
