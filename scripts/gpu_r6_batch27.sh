#!/bin/bash
# Round 6, batch 27: kernel trace of the single-learner kernels at P = 16 (MultiClassPA
# K = 2 / 4, HT, K-means, NN).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b27; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o learners -- python3 $R/bench/learners.py --preset p16 --steps 5 --quality-rounds 0 --only MultiClassPA,HT,K-means,NN > $O/prof.log 2>&1 || { tail -5 $O/prof.log; echo "trace failed"; exit 3; }
find $O/prof -name "*kernel_stats.csv" | head -2
