#!/bin/bash
# Round 6, batch 1: HT persistent kernel (diagnostics, tests, rates), the native forecast
# lane tests and the bench's engine forecast lane measurement.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/b1
mkdir -p $O
cd $R
timeout -k 10 200 python scripts/ht_diag.py > $O/ht_diag.txt 2>&1 || { tail -20 $O/ht_diag.txt; exit 3; }
cat $O/ht_diag.txt
timeout -k 10 300 python -u -m pytest tests/test_forecast_native_gpu.py tests/test_forecast_server_gpu.py -x -q --timeout 120 --timeout-method thread > $O/fs_tests.txt 2>&1; rc=$?; tail -15 $O/fs_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_ht_sequential.py tests/test_kernels_dense.py -m gpu -x -q -k "ht or HT" --timeout 300 --timeout-method thread > $O/ht_tests.txt 2>&1; rc=$?; tail -5 $O/ht_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/learners.py --preset p16 --steps 5 --only HT --cases '[["HT", 2, {"nClasses": 4, "exactDevice": true}, 16], ["HT@hostloop", 2, {"nClasses": 4}, 16], ["HT@check1024", 2, {"nClasses": 4, "checkEvery": 1024}, 16]]' > $O/ht_learners.json 2> $O/ht_learners.err || { tail -20 $O/ht_learners.err; exit 3; }
cat $O/ht_learners.json
timeout -k 10 300 python bench.py --engine-e2e 0 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 3; }
cat $O/bench.json
