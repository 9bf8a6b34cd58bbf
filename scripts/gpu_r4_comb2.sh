#!/bin/bash
# isolated scan timing (probe: prep and run serialised) with / without the in-launch combine,
# and the headline with more CUs kept for the scan's launch (16 scan + 16 combiner blocks)
mkdir -p gpurun_out/r4
for c in 0 1; do
  OMLDM_S3_COMB=$c timeout -k 10 120 python scripts/scan3_probe.py > gpurun_out/r4/probe_comb$c.json 2>gpurun_out/r4/probe_comb$c.err || exit 3
  echo "comb$c $(cat gpurun_out/r4/probe_comb$c.json)"
done
b() {  # name, env, args
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 "$@" > gpurun_out/r4/bcomb_$n.json 2> gpurun_out/r4/bcomb_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bcomb_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'])"
}
b c1k32 OMLDM_S3_COMB=1 --scan-cus 32 || exit 5
b c1k48 OMLDM_S3_COMB=1 --scan-cus 48 || exit 6
b c0k16 OMLDM_S3_COMB=0 --scan-cus 16 || exit 7
b c1plain OMLDM_S3_COMB=1 --lane plain || exit 8
b c0plain OMLDM_S3_COMB=0 --lane plain || exit 9
