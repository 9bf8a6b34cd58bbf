#!/bin/bash
# Round 6, batch 19: BASELINE config 5 through the engine with MultiClassPA K = 2 on the
# binary scan: 1 / 2 / 4 pipeline streams (2: every pipeline against its solo run) + trace.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b19; mkdir -p $O
for s in 1 2 4; do
  timeout -k 10 300 python bench/config5_engine.py --streams $s --solo $([ $s = 2 ] && echo 1 || echo 0) > $O/config5_s$s.json 2> $O/config5_s$s.err || { tail -20 $O/config5_s$s.err; exit 3; }
  cut -c 1-700 $O/config5_s$s.json
done
timeout -k 10 400 python -u bench/config5_engine.py --streams 2 --solo 0 --trace $O/config5_kernels.txt > $O/config5_traced.json 2> $O/config5_traced.err || { tail -20 $O/config5_traced.err; exit 3; }
head -30 $O/config5_kernels.txt
