#!/bin/bash
# Round 6, batch 29: closing per-learner record at P = 16 (with the GPU-vs-CPU quality).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b29; mkdir -p $O
timeout -k 10 700 python -u bench/learners.py --preset p16 --steps 10 > $O/learners_p16.json 2> $O/learners_p16.err || { tail -20 $O/learners_p16.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/learners_p16.json'))
for k,v in d['learners'].items(): print(k, v.get('examples_per_s'), v.get('ms_per_round'), (v.get('quality') or {}).get('score_gap'))"
