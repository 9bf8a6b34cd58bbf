#!/bin/bash
# Round 3: the whole GPU test suite, smoke, then PMC counters of the headline kernels.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gpu_tests_full.log 2>&1 || { tail -60 gpurun_out/r3_gpu_tests_full.log; exit 5; }
tail -3 gpurun_out/r3_gpu_tests_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 6; }
tail -1 gpurun_out/r3_smoke.log
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --latency-samples 0 --ref off --engine-latency 0 --engine-e2e 0 --ingest device"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_sq -o run -- $B > $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_sq.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_sq.log; exit 7; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_tcc -o run -- $B > $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_tcc.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_tcc.log; exit 8; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INSTS_SMEM --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_lds -o run -- $B > $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_lds.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r3_pmc_lds.log; exit 9; }
echo pmc-ok
