#!/bin/bash
# Engine e2e: reader variants (split reads, persistent pool, reader count).
set -e
mkdir -p gpurun_out/r5/read
for tag in "A=0" "OMLDM_READ_SPLIT=1,OMLDM_READ_POOL=1,OMLDM_READERS=16" "OMLDM_READ_SPLIT=1,OMLDM_READ_POOL=1,OMLDM_READERS=32" "OMLDM_READ_POOL=1"; do
  name=$(echo "$tag" | tr '=,' '__')
  env $(echo "$tag" | tr ',' ' ') timeout -k 10 200 python scripts/e2e_run.py dib 8388608 524288 > gpurun_out/r5/read/$name.json 2> gpurun_out/r5/read/$name.err
done
