#!/usr/bin/env python3
"""A/B of the two exact sequential round kernels (linear_seq.hip "seq" vs linear_scan.hip
"scan") on the headline geometry: max |Δw| against each other after 3 rounds, and the
device time per round. Diagnostics only (GPU)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402

dev = torch.device("cuda", 0)
space = FeatureSpace(13, 0, 26, 1 << 20)
rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
for S, R in [(16, 8192), (16, 2048), (32, 8192)]:
    B = S * R
    b = synth_raw(space, B, seed=25)
    b = type(b)(b.num.to(dev), b.tok.to(dev), b.y.to(torch.int8).to(dev))
    res = {}
    for kern in ("seq", "scan"):
        L.SEQ_KERNEL = kern
        w = torch.zeros(space.dim, device=dev)
        dacc = torch.zeros(space.dim + 2, device=dev)
        rep = torch.empty((S, space.dim), device=dev)
        L.linear_seq_broadcast(w, rep)
        for _ in range(3):
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
            L.linear_seq_apply(w, rep, dacc)
        torch.cuda.synchronize()
        n = 10
        t = time.perf_counter()
        for _ in range(n):
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
            L.linear_seq_apply(w, rep, dacc)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / n * 1e3
        w3 = torch.zeros(space.dim, device=dev)
        L.linear_seq_broadcast(w3, rep)
        for _ in range(3):
            L.linear_seq_round(w3, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
            L.linear_seq_apply(w3, rep, dacc)
        torch.cuda.synchronize()
        res[kern] = (ms, w3.cpu())
    d = float((res["seq"][1] - res["scan"][1]).abs().max())
    print(json.dumps({"geom": f"{S}x{R}", "ms_seq": round(res["seq"][0], 3),
                      "ms_scan": round(res["scan"][0], 3),
                      "Mex_s_scan": round(B / res["scan"][0] / 1e3, 1),
                      "max_abs_dw": d, "w_norm": float(res["seq"][1].norm())}), flush=True)

# per-phase cycles of the scan kernel (linear_scan.hip stamps), headline geometry
import ctypes  # noqa: E402

from omldm_amd.ops import native  # noqa: E402

lib = native.hip().cdll
lib.omldm_linear_scan_stamps.argtypes = [ctypes.c_void_p]
L.SEQ_KERNEL = "scan"
S, R = 16, 8192
b = synth_raw(space, S * R, seed=25)
b = type(b)(b.num.to(dev), b.tok.to(dev), b.y.to(torch.int8).to(dev))
w = torch.zeros(space.dim, device=dev)
dacc = torch.zeros(space.dim + 2, device=dev)
rep = torch.empty((S, space.dim), device=dev)
L.linear_seq_broadcast(w, rep)
L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
L.linear_seq_apply(w, rep, dacc)
st = torch.zeros((S, 16), dtype=torch.int64, device=dev)
lib.omldm_linear_scan_stamps(st.data_ptr())
L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
torch.cuda.synchronize()
lib.omldm_linear_scan_stamps(None)
m = st.double().mean(0)
it = max(float(m[8]), 1.0)
names = ["scan", "scan_bar", "h_top_wait", "h_issue", "h_margins", "h_lds", "h_scatter", "h_bar"]
print(json.dumps({"stamps_cycles_per_chunk": {names[k]: round(float(m[k]) / it, 1)
                                              for k in range(8)}, "iterations": it}), flush=True)
