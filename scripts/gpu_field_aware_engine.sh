#!/bin/bash
# Compatibility check: the engine / Kafka / dense-kernel GPU tests with the engine's default
# categorical wire switched to field-aware (uint16 slots) for this run only (117 passed).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
# one-off: the engine's default categorical wire flipped to field-aware for this run only
sed -i 's/    fieldAware: bool = False /    fieldAware: bool = True  /' omldm_amd/utils/config.py
grep -n "fieldAware: bool" omldm_amd/utils/config.py
timeout -k 10 600 python -u -m pytest tests/test_engine.py tests/test_kafka.py tests/test_kernels_dense.py tests/test_multi_pipeline.py tests/test_examples.py tests/test_ingest_pipeline.py tests/test_holdout_gpu.py tests/test_fault.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1; rc=$?; tail -15 gpurun_out/fa_tests.log; exit $rc
