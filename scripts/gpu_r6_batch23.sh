#!/bin/bash
# Round 6, batch 23: closing numbers — smoke(), bench.py at N = 1 (default flags), every
# learner at P = 16 with the GPU-vs-CPU holdout quality, and a kernel trace of bench.py.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b23; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 3; }
tail -1 $O/smoke.txt
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 3; }
tail -c 600 $O/bench_default.json
timeout -k 10 700 python -u bench/learners.py --preset p16 --steps 10 > $O/learners_p16.json 2> $O/learners_p16.err || { tail -20 $O/learners_p16.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/learners_p16.json'))
for k,v in d['learners'].items(): print(k, v.get('examples_per_s'), v.get('ms_per_round'), (v.get('quality') or {}).get('score_gap'))"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py --steps 50 --warmup 10 --engine-e2e 0 > $O/benchprof.log 2>&1 || { tail -5 $O/benchprof.log; echo "bench trace failed"; }
find $O/prof_bench -name "*kernel_stats.csv" | head -2
