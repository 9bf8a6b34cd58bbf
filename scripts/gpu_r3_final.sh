#!/bin/bash
# Round 3 final: the whole GPU suite, smoke, the driver's default bench, a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_final_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3_final_gpu_tests.log; exit 5; }
tail -3 gpurun_out/r3_final_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final_smoke.log 2>&1 || { tail -20 gpurun_out/r3_final_smoke.log; exit 6; }
tail -1 gpurun_out/r3_final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3_final_bench.json 2> gpurun_out/r3_final_bench.err || { tail -20 gpurun_out/r3_final_bench.err; exit 7; }
cat gpurun_out/r3_final_bench.json
# multi-rank rehearsal of the bench on the one GPU (both ranks on cuda:0 over gloo)
OMLDM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --engine-latency 0 --engine-e2e 0 --latency-samples 0 > gpurun_out/r3_final_bench2.json 2> gpurun_out/r3_final_bench2.err || { tail -30 gpurun_out/r3_final_bench2.err; exit 8; }
cat gpurun_out/r3_final_bench2.json
