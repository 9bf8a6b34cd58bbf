#!/bin/bash
# K-means matrix-core assign: kernel time with the flush / the LDS sums ablated.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export TMPDIR=/tmp
for ab in 0 1 2 3; do
  OMLDM_KMEANS_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/km_ab_$ab -o run -- python3 bench/learners.py --only K-means --steps 20 > gpurun_out/km_ab_$ab.log 2>&1 || { tail -20 gpurun_out/km_ab_$ab.log; exit 3; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/km_ab_$ab/run_kernel_stats.csv')):
    if 'mfma' in r['Name']: print('ablate=$ab', r['Name'][:40], r['Calls'], r['AverageNs'])
"
done
