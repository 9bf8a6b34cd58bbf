#!/bin/bash
# the copy stream without device-side waits (the host waits for the slot's last round)
mkdir -p gpurun_out/r4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --latency-samples 0 "$@" > gpurun_out/r4/ba_$n.json 2> gpurun_out/r4/ba_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/ba_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('holdout_accuracy'), d.get('accuracy_gap_pt'))"
}
b hw1 || exit 3
b hw0 --host-ahead-wait 0 --ref off || exit 4
b hw1b --ref off || exit 5
b hw0b --host-ahead-wait 0 --ref off || exit 6
b hw1s4 --ref off --slots 4 || exit 7
b hw1_100 --ref off --steps 100 || exit 8
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_ahead -o bench -- python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 --steps 10 > gpurun_out/r4/prof_ahead.log 2>&1 || exit 9
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r4/prof_ahead/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
cp=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in rows if 'pull_copy' in r['Kernel_Name'])
print('copy gaps', [round((cp[i+1][0]-cp[i][1])/1e3,1) for i in range(max(0,len(cp)-8),len(cp)-1)])
PY
