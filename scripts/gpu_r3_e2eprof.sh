#!/bin/bash
# Engine e2e kernel trace: GPU busy time per tick next to the host stages.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e2eprof -o e2e -- python3 bench/engine_e2e.py --records 8000000 --batch 131072 > gpurun_out/e2eprof_prof.json 2> gpurun_out/e2eprof_prof.err || { tail -20 gpurun_out/e2eprof_prof.err; exit 6; }
ls -R gpurun_out/e2eprof | head -20
