#!/bin/bash
# Round 3: v2 scan kernel — numerics vs CPU (both kernels), then the A/B timing.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rawwire.py -m gpu > gpurun_out/r3_scan_tests.log 2>&1 || { tail -60 gpurun_out/r3_scan_tests.log; exit 3; }
tail -3 gpurun_out/r3_scan_tests.log
timeout -k 10 200 python scripts/scan_ab.py > gpurun_out/r3_scan_ab.json 2> gpurun_out/r3_scan_ab.err || { tail -30 gpurun_out/r3_scan_ab.err; exit 4; }
cat gpurun_out/r3_scan_ab.json
