#!/bin/bash
# End-to-end engine profile: roctx ranges (marker trace) + kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 60 python -c "from omldm_amd.utils import tracing; print('roctx:', bool(tracing._load_roctx()))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e -o run -- python3 $R/bench/engine_e2e.py --records 200000 --batch 65536 > $R/gpurun_out/prof_e2e.log 2>&1 || { echo prof failed; tail -20 $R/gpurun_out/prof_e2e.log; exit 2; }
ls $R/gpurun_out/prof_e2e
tail -1 $R/gpurun_out/prof_e2e.log | cut -c1-300
