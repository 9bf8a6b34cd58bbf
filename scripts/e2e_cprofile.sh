#!/bin/bash
# Host profile of the engine's tick thread during the end-to-end bench (cProfile, main
# thread only), top functions by cumulative and own time.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/e2e.prof bench/engine_e2e.py --records 4000000 --batch 65536 > gpurun_out/e2e_cprof.json 2> gpurun_out/e2e_cprof.err || { tail -20 gpurun_out/e2e_cprof.err; exit 1; }
cat gpurun_out/e2e_cprof.json
python - <<'PY' > gpurun_out/e2e_cprof.txt
import pstats
p = pstats.Stats("gpurun_out/e2e.prof")
p.sort_stats("tottime").print_stats(35)
p.sort_stats("cumulative").print_stats(45)
PY
head -120 gpurun_out/e2e_cprof.txt
