#!/bin/bash
# Full GPU check: pytest -m gpu, smoke, default bench, rocprofv3 kernel-trace summary.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log | grep -E "passed|failed|FAILED|Error" ; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 100 ${BENCH_ARGS:-} > $R/gpurun_out/prof_bench.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 5; }
  cd $R && python scripts/trace_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && cat gpurun_out/prof_bench_summary.txt | tail -16
fi
