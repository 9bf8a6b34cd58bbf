#!/usr/bin/env python3
"""Diagnostics: the K = 10 multiclass scan against the CPU oracle several times in one
process (default template cap 8 at import, raised to 16 around each run, as the test)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models import make_learner  # noqa: E402
from omldm_amd.models.base import RoundContext  # noqa: E402
from omldm_amd.ops import dense as D  # noqa: E402

space = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
cases = [(4, 16, 4096), (8, 16, 4096), (10, 16, 4096), (10, 16, 4096), (16, 16, 4096),
         (10, 16, 4096), (10, 5, 300), (10, 16, 4096)]
ref = {}
for K, S, R in cases:
    D._MC_SCAN_KMAX = 16
    res = {}
    for d in ("cpu", "cuda"):
        if d == "cpu" and (K, S, R) in ref:
            res[d] = ref[(K, S, R)]
            continue
        lrn = make_learner("MultiClassPA", {"nClasses": K, "variant": "PA-I", "C": 1.0}, space, d)
        for k in range(3):
            b = synth_batch(space, S * R - 11, start=k * S * R, task=2, n_classes=K, seed=43)
            lrn.fit(b.to(d) if d != "cpu" else b, RoundContext(spokes=S, inv_p=1.0 / S))
        if d == "cuda":
            torch.cuda.synchronize()
        res[d] = lrn.W.detach().float().cpu()
    ref[(K, S, R)] = res["cpu"]
    diff = (res["cuda"] - res["cpu"]).abs()
    print(f"K={K} S={S} R={R}: max|gpu - cpu| = {float(diff.max()):.3e}, "
          f"bad = {int((diff > 1e-4).sum())}", flush=True)
    D._MC_SCAN_KMAX = 8
