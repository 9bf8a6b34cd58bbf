#!/bin/bash
# Round-6 baseline: headline bench, the slow learners at P = 16, and a kernel trace of the
# single-learner rounds (K-means, HT).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/base
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cat $O/bench.json
timeout -k 10 300 python bench/learners.py --preset p16 --steps 5 --only K-means,HT,NN,MultiClassPA > $O/learners.json 2> $O/learners.err || { tail -20 $O/learners.err; exit 3; }
cat $O/learners.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o km -- python3 $R/bench/learners.py --preset p16 --steps 3 --only K-means,HT > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
find $O/prof -name "*kernel_stats.csv" | head -3
