#!/usr/bin/env python3
"""Diagnostics: the same MultiClassPA rounds through two K templates of the v3 scan
(OMLDM_MC_KT forces the wider one; the key-major shadow is padded to it), and each against
the CPU oracle: max |ΔW|. Usage: python scripts/mc_kt_diag.py NCLASS KT [S R]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models import make_learner  # noqa: E402
from omldm_amd.models.base import RoundContext  # noqa: E402
from omldm_amd.ops import dense as D  # noqa: E402

nclass, kt = int(sys.argv[1]), int(sys.argv[2])
S, R = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (16, 4096)
space = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
out = {}
for tag, env in (("cpu", None), ("native", "0"), ("kt", str(kt))):
    os.environ["OMLDM_MC_KT"] = env or "0"
    dev = "cpu" if tag == "cpu" else "cuda"
    lrn = make_learner("MultiClassPA", {"nClasses": nclass}, space, dev)
    if dev == "cuda" and tag == "kt":  # pad the shadow to the forced template
        lrn.Wt = torch.zeros((space.dim, max(kt, D.class_pad(nclass))), device=dev)
        lrn.on_state_loaded()
    for k in range(2):
        b = synth_batch(space, S * R - 11, start=k * S * R, task=2, n_classes=nclass, seed=43)
        lrn.fit(b.to(dev) if dev != "cpu" else b, RoundContext(spokes=S, inv_p=1.0 / S))
    if dev == "cuda":
        torch.cuda.synchronize()
    out[tag] = lrn.W.detach().float().cpu()
for a, b in (("native", "cpu"), ("kt", "cpu"), ("kt", "native")):
    d = (out[a] - out[b]).abs()
    print(f"nclass={nclass} KT={kt} S={S} R={R}: max|{a} - {b}| = {float(d.max()):.3e}, "
          f"n > 1e-4: {int((d > 1e-4).sum())}, first bad column: "
          f"{int((d > 1e-4).any(0).nonzero()[0]) if (d > 1e-4).any() else -1}", flush=True)
