#!/bin/bash
# A/B: engine staging copy by the pull kernel vs SDMA (hipMemcpyAsync), 2 reps each.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for b in 65536 131072; do for cp in pull sdma; do
  v=$(timeout -k 10 200 python bench/engine_e2e.py --records 4000000 --batch $b --ingest-copy $cp 2>/dev/null | python -c "import json,sys; print(round(json.loads(sys.stdin.read().strip().splitlines()[-1])['value']/1e6,1))") || exit 1
  echo "rep $rep batch $b ingestCopy $cp: $v M rec/s"
done; done; done
