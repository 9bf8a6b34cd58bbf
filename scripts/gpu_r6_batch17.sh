#!/bin/bash
# Round 6, batch 17: signal plane with fenced cached mailbox reads (tests + rehearsal), and
# the config-5 engine run with an in-process kernel summary.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R
O=$R/gpurun_out/r6/b17; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_async_protocols.py -m gpu -v --timeout 150 --timeout-method thread > $O/async_tests.txt 2>&1 || { tail -30 $O/async_tests.txt; exit 3; }
grep -E "PASSED|FAILED|passed|failed" $O/async_tests.txt | tail -6
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 > $O/rehearsal_fa.json 2> $O/rehearsal_fa.err || { tail -20 $O/rehearsal_fa.err; exit 3; }
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 --slow 2 --protos Asynchronous,SSP --planes signal > $O/rehearsal_fa_slow.json 2> $O/rehearsal_fa_slow.err || { tail -20 $O/rehearsal_fa_slow.err; exit 3; }
python3 - <<'PY'
import json
for f in ("rehearsal_fa.json", "rehearsal_fa_slow.json"):
    d = json.load(open("gpurun_out/r6/b17/" + f))
    for k, v in d["runs"].items():
        print(f, k, v.get("rounds_per_s_total"), v.get("rounds_per_s"), v.get("pushes_per_s"), v.get("acc"))
PY
timeout -k 10 400 python -u bench/config5_engine.py --streams 2 --solo 0 --trace $O/config5_kernels.txt > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 3; }
head -30 $O/config5_kernels.txt
