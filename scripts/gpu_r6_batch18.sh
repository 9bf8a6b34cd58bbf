#!/bin/bash
# Round 6, batch 18: exact K-means with the branch-free centroid update, and MultiClassPA
# K = 2 on the binary scan: tests and rates.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b18; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmeans_seq.py tests/test_kernels_dense.py -m gpu -k "kmeans" -q --timeout 300 --timeout-method thread > $O/km_tests.txt 2>&1 || { tail -30 $O/km_tests.txt; exit 3; }
tail -2 $O/km_tests.txt
timeout -k 10 600 python -u -m pytest tests/test_scan3.py -m gpu -k "multiclass" -q --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1 || { tail -30 $O/mc_tests.txt; exit 3; }
tail -2 $O/mc_tests.txt
timeout -k 10 300 python bench/learners.py --preset p16 --steps 10 --only K-means --quality-rounds 0 > $O/km_p16.json 2> $O/km_p16.err || { tail -20 $O/km_p16.err; exit 3; }
cut -c 1-600 $O/km_p16.json
timeout -k 10 300 python bench/learners.py --preset p16 --steps 20 --only MultiClassPA --quality-rounds 2 > $O/mc_p16.json 2> $O/mc_p16.err || { tail -20 $O/mc_p16.err; exit 3; }
cut -c 1-900 $O/mc_p16.json
OMLDM_MC_BINARY=0 timeout -k 10 300 python bench/learners.py --preset p16 --steps 20 --only MultiClassPA --quality-rounds 2 > $O/mc_p16_k.json 2> $O/mc_p16_k.err || { tail -20 $O/mc_p16_k.err; exit 3; }
cut -c 1-900 $O/mc_p16_k.json
