#!/bin/bash
# Secondary BASELINE configs on one GPU: multi-pipeline serving (config 5), ORR+poly FGM
# (config 4), NN/HT learner throughput, and the reference-class CPU baseline.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench/multi_pipeline.py ${MP_ARGS:-} > gpurun_out/multi_pipeline.json 2> gpurun_out/multi_pipeline.err || { echo multi failed; tail -20 gpurun_out/multi_pipeline.err; exit 3; }
cat gpurun_out/multi_pipeline.json
timeout -k 10 300 python bench/orr_fgm.py ${ORR_ARGS:-} > gpurun_out/orr_fgm.json 2> gpurun_out/orr_fgm.err || { echo orr failed; tail -20 gpurun_out/orr_fgm.err; exit 4; }
cat gpurun_out/orr_fgm.json
if [ -f bench/learners.py ]; then
  timeout -k 10 300 python bench/learners.py > gpurun_out/learners.json 2> gpurun_out/learners.err || { echo learners failed; tail -20 gpurun_out/learners.err; exit 5; }
  cat gpurun_out/learners.json
fi
timeout -k 10 300 python bench/cpu_reference.py --threads 16 > gpurun_out/cpu_reference.json 2>&1 || { echo cpu ref failed; exit 6; }
cat gpurun_out/cpu_reference.json
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_multi -o run -- python3 $R/bench/multi_pipeline.py --steps 10 --warmup 2 --latency-samples 50 > $R/gpurun_out/prof_multi.log 2>&1 || { echo prof multi failed; exit 7; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_orr -o run -- python3 $R/bench/orr_fgm.py --steps 20 --warmup 2 > $R/gpurun_out/prof_orr.log 2>&1 || { echo prof orr failed; exit 8; }
  cd $R && python scripts/trace_summary.py gpurun_out/prof_multi > gpurun_out/prof_multi_summary.txt && python scripts/trace_summary.py gpurun_out/prof_orr > gpurun_out/prof_orr_summary.txt
  tail -12 gpurun_out/prof_multi_summary.txt; tail -12 gpurun_out/prof_orr_summary.txt
fi
