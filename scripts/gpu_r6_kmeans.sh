#!/bin/bash
# Exact sequential k-means: the fast one-wave form vs the CPU oracle and vs the earlier
# forms, then the P = 16 learner rates of both forms.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/km
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kmeans_seq.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/learners.py --preset p16 --steps 5 --only K-means > $O/fast.json 2> $O/fast.err || { tail -20 $O/fast.err; exit 3; }
cat $O/fast.json
OMLDM_KMEANS_FAST=0 timeout -k 10 200 python bench/learners.py --preset p16 --steps 3 --only K-means > $O/old.json 2> $O/old.err || { tail -20 $O/old.err; exit 3; }
cat $O/old.json
