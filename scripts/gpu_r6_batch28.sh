#!/bin/bash
# Round 6, batch 28: exact K-means with 1/(n+1) ahead of the argmin
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b28; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmeans_seq.py tests/test_kernels_dense.py -m gpu -k "kmeans" -q --timeout 300 --timeout-method thread > $O/km_tests.txt 2>&1 || { tail -30 $O/km_tests.txt; exit 3; }
tail -2 $O/km_tests.txt
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only K-means --quality-rounds 0 > $O/km_p16.json 2> $O/km_p16.err || { tail -20 $O/km_p16.err; exit 3; }
cut -c 1-600 $O/km_p16.json
