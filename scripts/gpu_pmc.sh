#!/bin/bash
# PMC counter passes (own runs, --kernel-trace only alongside --pmc).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --latency-samples 10 --ingest device --latency-mode copy"
[ -n "${SKIP_SQ:-}" ] || timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc_sq -o run -- $B > $R/gpurun_out/pmc_sq.log 2>&1 || { echo pmc1 failed; tail -20 $R/gpurun_out/pmc_sq.log; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- $B > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo pmc2 failed; tail -20 $R/gpurun_out/pmc_fetch.log; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc_tcc -o run -- $B > $R/gpurun_out/pmc_tcc.log 2>&1 || { echo pmc2b failed; tail -20 $R/gpurun_out/pmc_tcc.log; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mlp -o run -- python3 $R/bench/learners.py --only NN,ORR --steps 5 > $R/gpurun_out/pmc_mlp.log 2>&1 || { echo pmc3 failed; tail -20 $R/gpurun_out/pmc_mlp.log; exit 4; }
find $R/gpurun_out/pmc_* -name "*.csv" | head -20
