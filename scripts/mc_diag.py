#!/usr/bin/env python3
"""Phase cycles of the MultiClassPA v3 scan (csrc/kernels/linear_scan3.hip s3mc_scan_kernel,
g_s3mc_dbg): per chunk of 64 rows, the scanner's chain and barrier wait, and the helper
waves' scatter / base-margin / staging / barrier phases (per helper wave), at P = 16 ×
8192 rows on the engine's field-aware wire.

    python scripts/mc_diag.py [--classes 4 --rounds 5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models import make_learner  # noqa: E402
from omldm_amd.models.base import RoundContext  # noqa: E402
from omldm_amd.ops import native  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--classes", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=131072)
    a = ap.parse_args()
    dev = torch.device("cuda")
    space = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
    ring = [synth_batch(space, a.batch, start=k * a.batch, seed=25, task=2,
                        n_classes=a.classes).to(dev) for k in range(3)]
    L = make_learner("MultiClassPA", {"nClasses": a.classes}, space, dev)
    ctx = RoundContext(spokes=16)
    for k in range(6):
        ring[k % 3].prep = None
        L.fit(ring[k % 3], ctx)
    torch.cuda.synchronize()
    h = native.hip()
    S = 16
    dbg = torch.zeros(S * 8, dtype=torch.int64, device=dev)
    native.check(h.omldm_scan3mc_debug(dbg.data_ptr()), "omldm_scan3mc_debug")
    t = time.perf_counter()
    for k in range(a.rounds):
        ring[k % 3].prep = None
        L.fit(ring[k % 3], ctx)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / a.rounds
    native.check(h.omldm_scan3mc_debug(None), "omldm_scan3mc_debug")
    d = dbg.view(S, 8).double().cpu()
    ch = d[:, 0].clamp(min=1)
    nh = 11  # helper waves (s3::NH)
    per = {"chunks_per_spoke": float(d[:, 0].mean() / a.rounds),
           "scanner_chain_cyc_per_chunk": float((d[:, 1] / ch).mean()),
           "scanner_wait_cyc_per_chunk": float((d[:, 2] / ch).mean()),
           "helper_scatter_cyc_per_chunk": float((d[:, 3] / ch / nh).mean()),
           "helper_margin_cyc_per_chunk": float((d[:, 4] / ch / nh).mean()),
           "helper_stage_cyc_per_chunk": float((d[:, 5] / ch / nh).mean()),
           "helper_wait_cyc_per_chunk": float((d[:, 6] / ch / nh).mean()),
           "spilled_spokes": float(d[:, 7].sum() / a.rounds),
           "ms_per_round": round(el * 1e3, 3), "classes": a.classes}
    print(json.dumps(per))
    return 0


if __name__ == "__main__":
    sys.exit(main())
