#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rawwire.py -m gpu > gpurun_out/r3_rawwire.log 2>&1 || { tail -40 gpurun_out/r3_rawwire.log; exit 3; }
tail -2 gpurun_out/r3_rawwire.log
timeout -k 10 200 python scripts/seq_phase_probe.py > gpurun_out/r3_probe.json 2> gpurun_out/r3_probe.err || { tail -30 gpurun_out/r3_probe.err; exit 4; }
cat gpurun_out/r3_probe.json
