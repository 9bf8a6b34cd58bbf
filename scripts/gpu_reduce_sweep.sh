#!/bin/bash
# Reduce-kernel geometry sweep (OMLDM_REDUCE_SPLIT × OMLDM_REDUCE_THREADS) on the headline
# bench: ms/step device-resident and with the H2D copy, and the reduce kernel's time.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/sweep
cd /tmp && export TMPDIR=/tmp
for sp in ${SPLITS:-1 2 4}; do for nt in ${THREADS:-256 512 1024}; do for ing in device pinned; do
  d=$R/gpurun_out/sweep/s${sp}_t${nt}_$ing; rm -rf $d
  OMLDM_REDUCE_SPLIT=$sp OMLDM_REDUCE_THREADS=$nt timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $R/bench.py --ingest $ing --steps 30 --warmup 5 --latency-samples 20 --lane split > $d.log 2>&1 || { echo "run $sp $nt $ing failed"; tail -5 $d.log; exit 2; }
  ms=$(python3 -c "import json; d=json.loads(open('$d.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")
  red=$(python3 -c "
import csv
rows=[r for r in csv.DictReader(open('$d/run_kernel_stats.csv'))]
for r in rows:
    if r['Name'].startswith('void omldm::linear_reduce') or 'linear_reduce_kernel' in r['Name']: print(round(float(r['AverageNs'])/1e3,1), end=' ')
    if 'linear_round_rd' in r['Name']: print('round', round(float(r['AverageNs'])/1e3,1), end=' ')
")
  echo "split=$sp threads=$nt $ing: $ms ms/step | reduce $red us"
done; done; done
