#!/bin/bash
# Kernel trace + L2 counters of the multi-pipeline launch (BASELINE config 5) at M = 16 and
# M = 4: where the 16-pipeline step goes. Each pass has its own time limit.
set -e
O=gpurun_out/r5/mpprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for M in 16 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$M -o kt -- python3 bench/multi_pipeline.py --pipelines $M --steps 10 --warmup 3 --ref 0 > $O/kt$M.out 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch$M -o f -- python3 bench/multi_pipeline.py --pipelines $M --steps 10 --warmup 3 --ref 0 > $O/fetch$M.out 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc$M -o t -- python3 bench/multi_pipeline.py --pipelines $M --steps 10 --warmup 3 --ref 0 > $O/tcc$M.out 2>&1
done
