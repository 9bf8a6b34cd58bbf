#!/bin/bash
# ORR Gram kernels: GPU tests, config-4 bench (ORR + PolynomialFeatures + FGM) v2 vs v1,
# and a kernel trace of the v2 run.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py tests/test_protocols.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gram.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gram.log; [ $rc -eq 0 ] || exit $rc
for v in fused unfused v1; do
  case $v in fused) E="";; unfused) E="OMLDM_FUSE_POLY=0";; v1) E="OMLDM_FUSE_POLY=0 OMLDM_GRAM_V1=1";; esac
  env $E timeout -k 10 200 python bench/orr_fgm.py > gpurun_out/orr_fgm_$v.log 2>&1 || { echo "orr_fgm $v failed"; tail -20 gpurun_out/orr_fgm_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/orr_fgm_$v.log | cut -c1-330)"
done
timeout -k 10 120 python bench/learners.py --only ORR > gpurun_out/orr_learner.log 2>&1 && tail -1 gpurun_out/orr_learner.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_orr
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_orr -o run -- python3 $R/bench/orr_fgm.py --steps 20 > $R/gpurun_out/prof_orr.log 2>&1 || { echo prof failed; tail -20 $R/gpurun_out/prof_orr.log; exit 4; }
cd $R && python scripts/trace_summary.py gpurun_out/prof_orr > gpurun_out/prof_orr_summary.txt && head -12 gpurun_out/prof_orr_summary.txt
