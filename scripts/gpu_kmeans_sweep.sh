#!/bin/bash
# K-means assign: block-count sweep of the matrix-core kernel (kernel time via rocprofv3).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
export TMPDIR=/tmp
for nb in ${BLOCKS:-512 256 128}; do
  OMLDM_KMEANS_BLOCKS=$nb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/km_sweep_$nb -o run -- python3 bench/learners.py --only K-means --steps 20 > gpurun_out/km_sweep_$nb.log 2>&1 || { tail -20 gpurun_out/km_sweep_$nb.log; exit 3; }
  echo "blocks=$nb"; grep -h kmeans $(find gpurun_out/km_sweep_$nb -name '*kernel_stats.csv') | cut -d, -f1-5
done
