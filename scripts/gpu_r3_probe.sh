#!/bin/bash
# Round 3: Gram-scan phase breakdown vs spokes, then the whole GPU test suite.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/seq_phase_probe.py > gpurun_out/r3_probe.json 2> gpurun_out/r3_probe.err || { tail -30 gpurun_out/r3_probe.err; exit 4; }
cat gpurun_out/r3_probe.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3_gpu_tests.log; exit 5; }
tail -5 gpurun_out/r3_gpu_tests.log
