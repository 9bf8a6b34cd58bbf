#!/bin/bash
# Kernel trace of the learner throughput table (per-kernel time vs the wall-clock round).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learners -o run -- python3 bench/learners.py --steps 20 > gpurun_out/prof_learners.log 2>&1 || { tail -20 gpurun_out/prof_learners.log; exit 3; }
S=$(find gpurun_out/prof_learners -name '*kernel_stats.csv' | head -1)
python3 - "$S" > gpurun_out/prof_learners_summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:45]:
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e3:10.1f} {float(r["AverageNs"])/1e3:8.2f}')
PY
cat gpurun_out/prof_learners_summary.txt
tail -1 gpurun_out/prof_learners.log
