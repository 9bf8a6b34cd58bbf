#!/bin/bash
# NUMA placement A/B for the headline bench (1 GPU): bound to the GPU's node (default),
# unbound, and forced onto the remote socket.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
remote=$(python - <<'PY'
import torch
from omldm_amd.utils.topology import pci_address, device_locality
node, _ = device_locality(pci_address(0))
print("64-127" if node == 0 else "0-63")
PY
)
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --latency-samples 3000 > gpurun_out/numa_bound_$rep.json || exit 1
  OMLDM_NUMA_BIND=0 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --latency-samples 3000 > gpurun_out/numa_unbound_$rep.json || exit 1
  OMLDM_NUMA_BIND=0 timeout -k 10 120 taskset -c $remote python bench.py --steps 200 --warmup 20 --latency-samples 3000 > gpurun_out/numa_remote_$rep.json || exit 1
done
for f in gpurun_out/numa_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value']/1e6, d['p50_predict_latency_us'], d.get('numa'))"; done
