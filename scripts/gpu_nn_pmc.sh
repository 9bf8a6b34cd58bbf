#!/bin/bash
# NN round kernel counters (own runs, --kernel-trace only alongside --pmc).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
CASES='[["NN@bf16",0,{"hiddenLayers":[64,64],"matmulDtype":"bf16"},512]]'
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc_nn1 -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 5 > $R/gpurun_out/pmc_nn1.log 2>&1 || { echo pass1 failed; tail -5 $R/gpurun_out/pmc_nn1.log; exit 2; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_nn2 -o run -- python3 $R/bench/learners.py --cases "$CASES" --steps 5 > $R/gpurun_out/pmc_nn2.log 2>&1 || { echo pass2 failed; tail -5 $R/gpurun_out/pmc_nn2.log; exit 3; }
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc_nn1", "gpurun_out/pmc_nn2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no counter file"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if "mlp_round" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]]["v"] += float(r["Counter_Value"])
    print(d, {k: "%.3e" % v["v"] for k, v in acc.items()})
PY
