#!/bin/bash
# v3 scan: GPU tests, per-phase probe, and a kernel trace of the probe (standalone passes)
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_scan3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4/scan3_quick.txt 2>&1
rc=$?; tail -3 gpurun_out/r4/scan3_quick.txt; [ $rc -eq 0 ] || exit 4
timeout -k 10 200 python scripts/scan3_probe.py | tee gpurun_out/r4/probe.json || exit 5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_probe -o probe -- python scripts/scan3_probe.py > gpurun_out/r4/prof_probe.log 2>&1 || exit 6
f=$(find gpurun_out/r4/prof_probe -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r4/probe_kernel_stats.csv && head -12 gpurun_out/r4/probe_kernel_stats.csv
