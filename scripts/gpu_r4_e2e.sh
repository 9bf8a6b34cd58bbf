#!/bin/bash
mkdir -p gpurun_out/r4
for b in 65536 131072; do
  timeout -k 10 240 python bench/engine_e2e.py --records 1500000 --batch $b > gpurun_out/r4/e2e_$b.json 2> gpurun_out/r4/e2e_$b.err || exit 5
  python -c "
import json; d=json.loads(open('gpurun_out/r4/e2e_$b.json').read().strip().splitlines()[-1])
print($b, d['value'], d['wall_s'], d['ticks_timed']); st=d['stages_ms']
for k,v in sorted(st.items(), key=lambda kv: -kv[1].get('total_ms',0))[:12]: print('  ', k, v)
"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_e2e -o e2e -- python bench/engine_e2e.py --records 1000000 --batch 131072 > gpurun_out/r4/prof_e2e.log 2>&1 || exit 8
f=$(find gpurun_out/r4/prof_e2e -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r4/e2e_kernel_stats.csv && cut -c1-150 gpurun_out/r4/e2e_kernel_stats.csv | head -20
