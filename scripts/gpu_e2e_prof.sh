#!/bin/bash
# End-to-end engine profile: roctx ranges (marker trace) + kernel trace, one tick's timeline.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_e2e
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e -o run -- python3 $R/bench/engine_e2e.py --records ${E2E_RECORDS:-1000000} --batch 65536 > $R/gpurun_out/prof_e2e.log 2>&1 || { echo prof failed; tail -20 $R/gpurun_out/prof_e2e.log; exit 2; }
tail -1 $R/gpurun_out/prof_e2e.log | cut -c1-400
cd $R && python scripts/tick_timeline.py gpurun_out/prof_e2e 8 > gpurun_out/e2e_tick.txt && cat gpurun_out/e2e_tick.txt | head -80
