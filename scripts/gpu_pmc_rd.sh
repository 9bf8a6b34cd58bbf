#!/bin/bash
# SQ counters of the device-resident headline round (one pass, kernel trace only beside it).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --latency-samples 10 --ingest device --latency-mode copy ${BENCH_ARGS:-}"
rm -rf $R/gpurun_out/pmc_rd
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_rd -o run -- $B > $R/gpurun_out/pmc_rd.log 2>&1 || { echo pmc failed; tail -20 $R/gpurun_out/pmc_rd.log; exit 2; }
rm -rf $R/gpurun_out/pmc_rd2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_rd2 -o run -- $B > $R/gpurun_out/pmc_rd2.log 2>&1 || { echo pmc2 failed; tail -20 $R/gpurun_out/pmc_rd2.log; exit 3; }
cd $R
for d in pmc_rd pmc_rd2; do f=$(find gpurun_out/$d -name "*counter_collection.csv" | head -1); python scripts/pmc_summary.py $f; done
