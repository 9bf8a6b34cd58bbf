#!/usr/bin/env python3
"""Per-phase cycle breakdown of the Gram-scan round (linear_seq.hip diagnostics stamps)
and round time vs spokes. Diagnostics only (GPU)."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402
from omldm_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
space = FeatureSpace(13, 0, 26, 1 << 20)
rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
lib = native.hip().cdll
lib.omldm_linear_seq_stamps.argtypes = [ctypes.c_void_p]
out = {}
for S, R in [(16, 8192), (64, 8192), (256, 2048), (256, 8192)]:
    B = S * R
    b = synth_raw(space, B, seed=25)
    b = type(b)(b.num.to(dev), b.tok.to(dev), b.y.to(torch.int8).to(dev))
    w = torch.zeros(space.dim, device=dev)
    dacc = torch.zeros(space.dim + 2, device=dev)
    rep = torch.empty((S, space.dim), device=dev)
    L.linear_seq_broadcast(w, rep)
    for _ in range(3):
        L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
        L.linear_seq_apply(w, rep, dacc)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 10
    for _ in range(n):
        L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
        L.linear_seq_apply(w, rep, dacc)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / n * 1e3
    st = torch.zeros((S, 16), dtype=torch.int64, device=dev)
    lib.omldm_linear_seq_stamps(st.data_ptr())
    L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S, replicas=rep)
    L.linear_seq_apply(w, rep, dacc)
    torch.cuda.synchronize()
    lib.omldm_linear_seq_stamps(None)
    m = st.double().mean(0)
    ch = float(m[5])
    names = ["scan", "scan_wait", "post_scan", "-", "produce", "chunks", "prod_wait",
             "-", "p_fence_hash", "p_gather_issue", "p_group", "p_bar1", "p_mfma", "p_bar2",
             "p_reset", "p_gather_use"]
    out[f"{S}x{R}"] = {"ms_per_round": round(ms, 3), "Mex_per_s": round(B / ms / 1e3, 1),
                       "cycles_per_chunk": {names[k]: round(float(m[k]) / max(ch, 1), 1)
                                            for k in range(16) if k not in (3, 5, 7)}, "chunks": ch}
    print(json.dumps({f"{S}x{R}": out[f"{S}x{R}"]}), flush=True)
