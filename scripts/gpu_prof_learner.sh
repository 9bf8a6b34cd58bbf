#!/bin/bash
# rocprofv3 kernel trace of one learner in bench/learners.py (LEARNER=name), summarised.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_learner
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_learner -o run -- python3 $R/bench/learners.py --only ${LEARNER:-MultiClassPA} --steps 10 > $R/gpurun_out/prof_learner.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_learner.log; exit 5; }
cd $R && python scripts/trace_summary.py gpurun_out/prof_learner > gpurun_out/prof_learner_summary.txt && head -14 gpurun_out/prof_learner_summary.txt
