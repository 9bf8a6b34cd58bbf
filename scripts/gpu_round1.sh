#!/bin/bash
# GPU check: kernel numerics tests, smoke, bench, rocprofv3 kernel stats.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
if [ -n "${PROFILE:-}" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 100 ${BENCH_ARGS:-} > $R/gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 $R/gpurun_out/prof.log; exit 5; }
  find $R/gpurun_out/prof -name "*stats*" | head
fi
