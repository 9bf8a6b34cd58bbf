#!/bin/bash
# full GPU suite, smoke, default bench (headline + engine e2e + engine latency)
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4/gpu_suite.txt 2>&1
rc=$?; tail -5 gpurun_out/r4/gpu_suite.txt; [ $rc -eq 0 ] || exit 4
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.txt 2>&1 || exit 5
tail -1 gpurun_out/r4/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_default.json 2> gpurun_out/r4/bench_default.err || exit 6
tail -1 gpurun_out/r4/bench_default.json
