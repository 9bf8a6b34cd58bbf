#!/bin/bash
# NN round kernel: MLP numerics tests, then a spoke sweep of the learner bench with the
# default library and with each variant in omldm_amd/_native/variants/ (A/B on one box).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py -k mlp -x -q --timeout 120 --timeout-method thread > gpurun_out/nn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/nn_tests.log; [ $rc -eq 0 ] || exit $rc
CASES='[["NN",0,{"hiddenLayers":[64,64]},512],["NN@s1024",0,{"hiddenLayers":[64,64]},1024],["NN@bf16",0,{"hiddenLayers":[64,64],"matmulDtype":"bf16"},512],["NN@bf16s1024",0,{"hiddenLayers":[64,64],"matmulDtype":"bf16"},1024],["NN@bf16s256",0,{"hiddenLayers":[64,64],"matmulDtype":"bf16"},256]]'
timeout -k 10 200 python bench/learners.py --cases "$CASES" > gpurun_out/nn_ab_default.json 2>gpurun_out/nn_ab.err || { tail -20 gpurun_out/nn_ab.err; exit 3; }
cat gpurun_out/nn_ab_default.json
for v in omldm_amd/_native/variants/*.so; do
  [ -e "$v" ] || continue
  cp omldm_amd/_native/libomldm_hip.so /tmp/libomldm_hip_default.so
  cp "$v" omldm_amd/_native/libomldm_hip.so
  timeout -k 10 200 python bench/learners.py --cases "$CASES" > gpurun_out/nn_ab_$(basename $v .so).json 2>>gpurun_out/nn_ab.err || { tail -20 gpurun_out/nn_ab.err; exit 4; }
  echo "== $v"; cat gpurun_out/nn_ab_$(basename $v .so).json
  cp /tmp/libomldm_hip_default.so omldm_amd/_native/libomldm_hip.so
done
