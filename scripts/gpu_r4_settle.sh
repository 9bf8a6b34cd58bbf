#!/bin/bash
# fresh box: does a clock settle before the warmup remove the first process's slowdown?
mkdir -p gpurun_out/r4
b() {  # name, args
  n=$1; shift
  timeout -k 10 240 python bench.py --engine-e2e 0 --engine-latency 0 --ref off --latency-samples 0 "$@" > gpurun_out/r4/bst_$n.json 2> gpurun_out/r4/bst_$n.err || return 1
  python -c "
import json; d=json.loads(open('gpurun_out/r4/bst_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'])"
}
b first_settle || exit 3
b second_nosettle --settle-ms 0 || exit 4
b third_settle || exit 5
b steps100 --steps 100 || exit 6
