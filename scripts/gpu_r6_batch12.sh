#!/bin/bash
# Round 6, batch 12: PMC counters of the NN round kernel v2 at P = 16 (three passes, each its
# own run with --kernel-trace only), then the Async / SSP 2-rank rehearsal on the bench wire.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b12; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
CASES='[["NN",0,{"hiddenLayers":[64,64]},16]]'
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/pmc1 -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 5 --quality-rounds 0 > $O/pmc1.log 2>&1 || { echo pass1 failed; tail -5 $O/pmc1.log; exit 2; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 5 --quality-rounds 0 > $O/pmc2.log 2>&1 || { echo pass2 failed; tail -5 $O/pmc2.log; exit 3; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_ANY --output-format csv -d $O/pmc3 -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 5 --quality-rounds 0 > $O/pmc3.log 2>&1 || { echo pass3 failed; tail -5 $O/pmc3.log; }
cd $R && python3 - <<'PY' > $O/pmc_summary.txt
import csv, glob, collections
tot = collections.defaultdict(float)
for d in ("pmc1", "pmc2", "pmc3"):
    for f in glob.glob(f"gpurun_out/r6/b12/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mlp_round2" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
print("mlp_round2_kernel<8> (P = 16, 5 timed + 18 warm-up rounds), summed over dispatches:")
for k, v in sorted(tot.items()):
    print(f"  {k:28s} {v:.4e}")
if tot.get("SQ_WAVE_CYCLES"):
    w = tot["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if k in tot:
            print(f"  {k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
if tot.get("GRBM_GUI_ACTIVE") and tot.get("SQ_VALU_MFMA_BUSY_CYCLES"):
    print(f"  SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE = {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / tot['GRBM_GUI_ACTIVE']:.3f}")
PY
cat $O/pmc_summary.txt
mkdir -p gpurun_out/r6/async
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 > gpurun_out/r6/async/rehearsal_fa.json 2> gpurun_out/r6/async/rehearsal_fa.err || { tail -20 gpurun_out/r6/async/rehearsal_fa.err; exit 3; }
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 --slow 2 > gpurun_out/r6/async/rehearsal_fa_slow.json 2> gpurun_out/r6/async/rehearsal_fa_slow.err || { tail -20 gpurun_out/r6/async/rehearsal_fa_slow.err; exit 3; }
cut -c 1-2500 gpurun_out/r6/async/rehearsal_fa.json
