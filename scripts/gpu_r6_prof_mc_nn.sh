#!/bin/bash
# Kernel traces of the MultiClassPA (K = 4) and NN rounds at P = 16.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/prof_mc_nn
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o mcnn -- python3 $R/bench/learners.py --preset p16 --steps 5 --only MultiClassPA,NN > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 3; }
tail -3 $O/log.txt
find $O/prof -name "*kernel_stats.csv" -exec head -30 {} \;
