#!/bin/bash
# Round 6, batch 3: kernel traces of the MultiClassPA (K = 4) and NN rounds; BASELINE
# config 5 through the engine (16 heterogeneous pipelines) at 1 / 2 / 4 pipeline streams,
# and a kernel trace of the 2-stream run.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6/b3
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_mcnn -o mcnn -- python3 $R/bench/learners.py --preset p16 --steps 5 --only MultiClassPA,NN > $O/mcnn.log 2>&1 || { tail -20 $O/mcnn.log; exit 3; }
tail -2 $O/mcnn.log
cd $R
for s in 1 2 4; do
  timeout -k 10 300 python bench/config5_engine.py --streams $s --solo $([ $s = 2 ] && echo 1 || echo 0) > $O/config5_s$s.json 2> $O/config5_s$s.err || { tail -20 $O/config5_s$s.err; exit 3; }
  cut -c 1-400 $O/config5_s$s.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python3 $R/bench/config5_engine.py --streams 2 --solo 0 > $O/c5prof.log 2>&1 || { tail -20 $O/c5prof.log; exit 3; }
find $O -name "*kernel_stats.csv" | head
