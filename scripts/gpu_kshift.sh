#!/bin/bash
set -u
mkdir -p gpurun_out
run() { timeout -k 10 120 env "$@" > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 3; }; python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['ms_per_step'], round(d['value']/1e6,1),'M/s', d['holdout_accuracy'], 'ovf', d['lds_table_overflow'])" "$@"; }
for K in 12 13 14; do
  run OMLDM_KSHIFT=$K python bench.py --steps 30 --warmup 5 --latency-samples 50 --ingest device
  run OMLDM_KSHIFT=$K python bench.py --steps 30 --warmup 5 --latency-samples 50 --ingest device --ablate 1
done
run OMLDM_KSHIFT=13 python bench.py --steps 30 --warmup 5 --latency-samples 50
run OMLDM_KSHIFT=14 python bench.py --steps 30 --warmup 5 --latency-samples 50
