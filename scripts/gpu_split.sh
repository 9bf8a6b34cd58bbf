#!/bin/bash
# Sweep of reduce blocks per key group (OMLDM_REDUCE_SPLIT): device-resident step (the
# training chain alone), the default H2D step, and kernel times under the copy (rocprofv3).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
run() { timeout -k 10 120 env "$@" > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 3; }; python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['ms_per_step'], round(d['value']/1e6,1),'M/s', d['holdout_accuracy'], 'ovf', d['lds_table_overflow'])" "$@"; }
for SP in ${SPLITS:-1 2 4 8}; do
  run OMLDM_REDUCE_SPLIT=$SP python bench.py --steps 40 --warmup 5 --latency-samples 50 --ingest device
  run OMLDM_REDUCE_SPLIT=$SP python bench.py --steps 40 --warmup 5 --latency-samples 50
done
for SP in ${PROF_SPLITS:-1 4}; do
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/prof_sp$SP
  OMLDM_REDUCE_SPLIT=$SP timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_sp$SP -o run -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 50 > $R/gpurun_out/prof_sp$SP.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_sp$SP.log; exit 5; }
  cd $R && echo "== split $SP" && python scripts/trace_summary.py gpurun_out/prof_sp$SP | head -8
done
