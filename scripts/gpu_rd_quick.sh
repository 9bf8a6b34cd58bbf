#!/bin/bash
# Quick device-resident + pinned timing of the headline bench, and a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
for ing in device pinned; do
  timeout -k 10 120 python bench.py --ingest $ing --latency-samples 200 ${BENCH_ARGS:-} > gpurun_out/q_${ing}.log 2>&1 || { echo "bench $ing failed"; tail -20 gpurun_out/q_${ing}.log; exit 2; }
  echo "ingest=$ing: $(python -c "import json,sys; d=json.loads(open('gpurun_out/q_${ing}.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms/step', round(d['value']/1e6,1), 'M ex/s acc', d['holdout_accuracy'], 'p50', d['p50_predict_latency_us'])")"
done
cd /tmp && export TMPDIR=/tmp
for ing in device pinned; do
rm -rf $R/gpurun_out/prof_q_$ing
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_q_$ing -o run -- python3 $R/bench.py --ingest $ing --steps 20 --warmup 5 --latency-samples 50 ${BENCH_ARGS:-} > $R/gpurun_out/prof_q_$ing.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_q_$ing.log; exit 3; }
(cd $R && python scripts/trace_summary.py gpurun_out/prof_q_$ing > gpurun_out/prof_q_${ing}_summary.txt && echo "== $ing" && head -6 gpurun_out/prof_q_${ing}_summary.txt && tail -2 gpurun_out/prof_q_${ing}_summary.txt)
done
