#!/bin/bash
# Gram pass ablations under rocprofv3 (kernel trace + stats only).
set -e
mkdir -p gpurun_out/r5/gram
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 1 2 4 7; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/gram/a$a -o g -- python3 scripts/gram_ablate.py $a > gpurun_out/r5/gram/a$a.out 2>&1
done
