#!/bin/bash
# Signal plane of the Asynchronous / SSP PS: GPU tests, then the 2-rank rehearsal bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6/async
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_async_protocols.py -m gpu -k signal -x -v \
  --timeout 150 --timeout-method thread > $O/tests_signal.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_async_protocols.py -m gpu -k "not signal" -x -v \
  --timeout 150 --timeout-method thread > $O/tests_device.txt 2>&1 &&
timeout -k 10 300 python -u bench/async_rehearsal.py --seconds 3 > $O/rehearsal.json 2> $O/rehearsal.err &&
timeout -k 10 300 python -u bench/async_rehearsal.py --seconds 3 --slow 20 > $O/rehearsal_slow.json 2> $O/rehearsal_slow.err
