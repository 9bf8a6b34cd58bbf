#!/bin/bash
# current headline: kernel trace + PMC passes (one counter group per run, --kernel-trace only)
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/r4
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 3 --latency-samples 0 --ref off --engine-e2e 0 --engine-latency 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4/prof_head -o bench -- $B > $R/gpurun_out/r4/prof_head.log 2>&1 || { echo trace failed; tail -5 $R/gpurun_out/r4/prof_head.log; exit 2; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r4/pmc_sq -o run -- $B > $R/gpurun_out/r4/pmc_sq.log 2>&1 || { echo pmc1 failed; tail -5 $R/gpurun_out/r4/pmc_sq.log; exit 3; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r4/pmc_fetch -o run -- $B > $R/gpurun_out/r4/pmc_fetch.log 2>&1 || { echo pmc2 failed; tail -5 $R/gpurun_out/r4/pmc_fetch.log; exit 4; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum --output-format csv -d $R/gpurun_out/r4/pmc_tcc -o run -- $B > $R/gpurun_out/r4/pmc_tcc.log 2>&1 || { echo pmc3 failed; tail -5 $R/gpurun_out/r4/pmc_tcc.log; exit 5; }
cd $R
for d in pmc_sq pmc_fetch pmc_tcc; do
  f=$(find gpurun_out/r4/$d -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/pmc_summary.py $f > gpurun_out/r4/$d.txt && head -12 gpurun_out/r4/$d.txt | cut -c1-200
done
f=$(find gpurun_out/r4/prof_head -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r4/head_kernel_stats.csv
python3 scripts/trace_timeline.py $(find gpurun_out/r4/prof_head -name "*kernel_trace.csv" | head -1) --last 24 > gpurun_out/r4/head_timeline.txt
cut -c1-100 gpurun_out/r4/head_timeline.txt | tail -14
