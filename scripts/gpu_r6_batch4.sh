#!/bin/bash
# Round 6, batch 4: the signal plane of the Asynchronous / SSP PS (GPU tests + the 2-rank
# rehearsal), then BASELINE config 5 through the engine at 1 / 2 / 4 pipeline streams and a
# kernel trace of the 2-stream run.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_r6_async.sh || { tail -30 gpurun_out/r6/async/*.txt gpurun_out/r6/async/*.err; exit 3; }
cut -c 1-1500 gpurun_out/r6/async/rehearsal.json
O=$R/gpurun_out/r6/b4
mkdir -p $O
for s in 1 2 4; do
  timeout -k 10 300 python bench/config5_engine.py --streams $s --solo $([ $s = 2 ] && echo 1 || echo 0) > $O/config5_s$s.json 2> $O/config5_s$s.err || { tail -20 $O/config5_s$s.err; exit 3; }
  cut -c 1-400 $O/config5_s$s.json
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python3 $R/bench/config5_engine.py --streams 2 --solo 0 > $O/c5prof.log 2>&1 || { tail -20 $O/c5prof.log; exit 3; }
echo done
