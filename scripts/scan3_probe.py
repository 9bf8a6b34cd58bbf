#!/usr/bin/env python3
"""v3 table scan at the headline geometry (16 spokes × 8192 rows, 2^20 slots): device time
of the prepare (passes 1-3) and of the run (scan + combine) per round, and the scan
kernel's per-phase cycles per chunk (linear_scan3.hip stamps). Diagnostics only (GPU)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402
from omldm_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
space = FeatureSpace(13, 0, 26, 1 << 20)
rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
S, R = 16, 8192
L.SEQ_KERNEL = "scan3"
b = synth_raw(space, S * R, seed=25)
b = type(b)(b.num.to(dev), b.tok.to(dev), b.y.to(torch.int8).to(dev))
w = torch.zeros(space.dim, device=dev)
dacc = torch.zeros(space.dim + 2, device=dev)
cum = torch.zeros(8, dtype=torch.float64, device=dev)
for _ in range(3):
    L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
    L.linear_apply(w, None, dacc)
torch.cuda.synchronize()
n = 10
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
tp = tr = 0.0
for _ in range(n):
    ev[0].record()
    b.prep = L.linear_scan3_prepare(b, R, S, space.dim, True, rule)
    ev[1].record()
    L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
    L.linear_apply(w, None, dacc)
    ev[2].record()
    torch.cuda.synchronize()
    tp += ev[0].elapsed_time(ev[1])
    tr += ev[1].elapsed_time(ev[2])
    b.prep = None
lib = native.hip().cdll
lib.omldm_scan3_stamps.argtypes = [ctypes.c_void_p]
st = torch.zeros((S, 16), dtype=torch.int64, device=dev)
lib.omldm_scan3_stamps(st.data_ptr())
L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
torch.cuda.synchronize()
lib.omldm_scan3_stamps(None)
m = st.double().mean(0)
nch = (R + 63) // 64 + 2
names = ["scan_tail", "scan_bar", "h_top_wait", "h_issue", "h_margins", "h_lds_prefetch",
         "h_scatter", "h_bar", "scan_head", "scan_chain"]
print(json.dumps({"prepare_ms": round(tp / n, 4), "run_ms": round(tr / n, 4),
                  "Mex_s": round(S * R / ((tp + tr) / n) / 1e3, 1),
                  "stamps_cycles_per_chunk": {names[k]: round(float(m[k]) / nch, 1)
                                              for k in range(10)}}), flush=True)

# latency experiment: every gather reads w[0] (wrong model, timing only)
lib.omldm_scan3_debug.argtypes = [ctypes.c_int]
lib.omldm_scan3_debug(1)
st.zero_()
lib.omldm_scan3_stamps(st.data_ptr())
L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
torch.cuda.synchronize()
lib.omldm_scan3_stamps(None)
lib.omldm_scan3_debug(0)
m = st.double().mean(0)
print(json.dumps({"gathers_hit_w0": {names[k]: round(float(m[k]) / nch, 1)
                                     for k in range(10)}}), flush=True)

# per helper wave (g_s3_debug = 16 + wave selects the stamped helper): which helper sets
# the chunk period (waves 4 and 8 share the scanner's SIMD)
per = {}
for wv in range(1, 12):
    lib.omldm_scan3_debug(16 + wv)
    st.zero_()
    lib.omldm_scan3_stamps(st.data_ptr())
    L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
    torch.cuda.synchronize()
    lib.omldm_scan3_stamps(None)
    m = st.double().mean(0)
    per[wv] = {names[k]: round(float(m[k]) / nch) for k in range(2, 8)}
lib.omldm_scan3_debug(0)
print(json.dumps({"helper_waves": per}), flush=True)
if os.environ.get("PROBE_HPRIO"):
    lib.omldm_scan3_hprio.argtypes = [ctypes.c_int]
    for v in (0, 1, 0, 1):
        lib.omldm_scan3_hprio(v)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(n):
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
            L.linear_apply(w, None, dacc)
        ev[1].record()
        torch.cuda.synchronize()
        print(json.dumps({"hprio": v, "run_ms": round(ev[0].elapsed_time(ev[1]) / n, 4)}),
              flush=True)
    lib.omldm_scan3_hprio(0)
if os.environ.get("PROBE_DENSE_ORDERS"):
    lib.omldm_scan3_dense_order.argtypes = [ctypes.c_int]
    for order in (0, 1):
        lib.omldm_scan3_dense_order(order)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(n):
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, cum=cum)
            L.linear_apply(w, None, dacc)
        ev[1].record()
        torch.cuda.synchronize()
        print(json.dumps({"dense_order": order, "run_ms": round(ev[0].elapsed_time(ev[1]) / n, 4)}),
              flush=True)
    lib.omldm_scan3_dense_order(0)
