#!/bin/bash
# H2D engine comparison with SDMA explicitly enabled vs default.
set -u
mkdir -p gpurun_out
one() { timeout -k 10 120 env "$@" > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 3; }; python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['ms_per_step'], round(d['value']/1e6,1),'M/s')" "$@"; }
one HSA_ENABLE_SDMA=1 python bench.py --steps 30 --warmup 5 --latency-samples 100 --h2d sdma
one HSA_ENABLE_SDMA=1 python bench.py --steps 30 --warmup 5 --latency-samples 100 --h2d engine --copy-streams 1
one HSA_ENABLE_SDMA=1 python bench.py --steps 30 --warmup 5 --latency-samples 100 --h2d engine --copy-streams 2
one HSA_ENABLE_SDMA=1 python bench.py --steps 30 --warmup 5 --latency-samples 100
one HSA_ENABLE_SDMA=0 python bench.py --steps 30 --warmup 5 --latency-samples 100 --h2d engine --copy-streams 1
one HSA_ENABLE_SDMA=1 HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=1 python bench.py --steps 30 --warmup 5 --latency-samples 100 --h2d engine --copy-streams 1
