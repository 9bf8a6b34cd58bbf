#!/bin/bash
# Hoeffding tree: the persistent exact kernel vs the host-driven loop and the oracle, its
# phase diagnostics, then the P = 16 rates.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/ht
mkdir -p $O
cd $R
timeout -k 10 200 python scripts/ht_diag.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 3; }
cat $O/diag.txt
timeout -k 10 400 python -u -m pytest tests/test_ht_sequential.py tests/test_kernels_dense.py -m gpu -x -q -k "ht or HT" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/learners.py --preset p16 --steps 5 --only HT --cases '[["HT", 2, {"nClasses": 4, "exactDevice": true}, 16], ["HT@hostloop", 2, {"nClasses": 4}, 16], ["HT@check1024", 2, {"nClasses": 4, "checkEvery": 1024}, 16]]' > $O/learners.json 2> $O/learners.err || { tail -20 $O/learners.err; exit 3; }
cat $O/learners.json
