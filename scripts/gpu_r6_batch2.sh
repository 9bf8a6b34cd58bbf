#!/bin/bash
# Round 6, batch 2: the headline bench with its new fields (device copy / round ms, fp64
# parity row, native forecast lane), the engine e2e with an SVM and a K-means pipeline, the
# learner table at P = 16, and the GPU tests touched this round.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/b2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_scan3.py tests/test_multirank_gpu.py tests/test_kmeans_seq.py tests/test_ht_sequential.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 3; }
cat $O/bench.json
timeout -k 10 300 python bench/engine_e2e.py --records 4000000 --batch 524288 --partitions 16 --learners "SVM,K-means:k=16" > $O/e2e_svm_kmeans.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 3; }
cat $O/e2e_svm_kmeans.json
timeout -k 10 400 python bench/learners.py --preset p16 --steps 5 > $O/learners_p16.json 2> $O/learners.err || { tail -20 $O/learners.err; exit 3; }
cat $O/learners_p16.json
