#!/bin/bash
# Register-dedup round kernel: occupancy sensitivity (device-resident headline step with
# library variants built with -DOMLDM_RD_OCC=4/6/8; the in-tree library is occupancy 5).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
cp omldm_amd/_native/libomldm_hip.so .probe/libhip_occ5.so
for occ in 5 4 6 8 5; do
  cp .probe/libhip_occ$occ.so omldm_amd/_native/libomldm_hip.so
  OMLDM_NO_AUTOBUILD=1 timeout -k 10 120 python bench.py --ingest device --steps 200 --warmup 20 --latency-samples 10 > gpurun_out/rd_occ$occ.json 2>gpurun_out/rd_occ$occ.err || { tail -5 gpurun_out/rd_occ$occ.err; exit 3; }
  python3 -c "import json; d=json.load(open('gpurun_out/rd_occ$occ.json')); print('occ=$occ', d['ms_per_step'], round(d['value']/1e6))"
done
