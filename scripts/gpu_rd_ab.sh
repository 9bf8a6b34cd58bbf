#!/bin/bash
# A/B of the linear round kernels on the headline config: register-dedup (default on the
# field-aware wire) vs the LDS-hash-table kernel (OMLDM_LINEAR_RD=0); device-resident and
# with the H2D copy in the loop; then a kernel trace of each.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
for rd in 1 0; do
  for ing in device pinned; do
    OMLDM_LINEAR_RD=$rd timeout -k 10 120 python bench.py --ingest $ing --latency-samples 200 ${BENCH_ARGS:-} > gpurun_out/rd${rd}_${ing}.log 2>&1 || { echo "bench rd=$rd $ing failed"; tail -20 gpurun_out/rd${rd}_${ing}.log; exit 2; }
    echo "rd=$rd ingest=$ing: $(python -c "import json,sys; d=json.loads(open('gpurun_out/rd${rd}_${ing}.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms/step', round(d['value']/1e6,1), 'M ex/s acc', d['holdout_accuracy'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for rd in 1 0; do
  rm -rf $R/gpurun_out/prof_rd$rd
  OMLDM_LINEAR_RD=$rd timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rd$rd -o run -- python3 $R/bench.py --steps 20 --warmup 5 --latency-samples 50 ${BENCH_ARGS:-} > $R/gpurun_out/prof_rd$rd.log 2>&1 || { echo "prof rd=$rd failed"; tail -20 $R/gpurun_out/prof_rd$rd.log; exit 3; }
  (cd $R && python scripts/trace_summary.py gpurun_out/prof_rd$rd > gpurun_out/prof_rd${rd}_summary.txt && echo "== rd=$rd" && head -8 gpurun_out/prof_rd${rd}_summary.txt && tail -2 gpurun_out/prof_rd${rd}_summary.txt)
done
