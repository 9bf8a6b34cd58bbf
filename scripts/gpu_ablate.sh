#!/bin/bash
# Kernel phase ablation sweep + config sweep (diagnostics).
# SWEEP: space-separated configs; inside a config use ',' between flags; 'x' = defaults.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_linear.py -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
run() { timeout -k 10 120 python bench.py --steps 30 --warmup 5 --latency-samples 200 "$@" > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 3; }; python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['ms_per_step'], round(d['value']/1e6,1),'M/s', 'acc',d['holdout_accuracy'],'ovf',d['lds_table_overflow'],'p50',d['p50_predict_latency_us'])" "$@"; }
for a in ${SWEEP:-x --ingest=device --ingest=device,--ablate=1 --ingest=device,--ablate=2}; do
  if [ "$a" = "x" ]; then run; else run ${a//,/ }; fi
done
