#!/usr/bin/env python3
"""Per-learner training throughput on one GPU (every reference learner + extension):
one round = the learner's fit on a micro-batch with S virtual spokes (where the learner
has them), HBM-resident synthetic data, model update included. One JSON line per run
with examples/s per learner — the regression guard for the non-headline kernels.

    python bench/learners.py [--batch 131072 --steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace, HashedBatch  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models import make_learner  # noqa: E402
from omldm_amd.models.base import RoundContext  # noqa: E402

# (name, task, hyper, spokes[, wire]); wire "compact" = the field-aware uint16 wire of the
# headline bench (the register-dedup kernels run there with ≤ 16 rows per spoke)
CASES = [
    ("PA", 0, {}, 4096),
    ("SVM", 0, {"modelDtype": "bf16", "tableLog2": 11}, 4096),
    ("RegressorPA", 1, {}, 4096),
    ("LogisticRegression", 0, {}, 4096),
    ("PA@compact", 0, {}, 8192, "compact"),
    ("SVM@compact", 0, {"modelDtype": "bf16"}, 8192, "compact"),
    ("RegressorPA@compact", 1, {}, 8192, "compact"),
    ("LogisticRegression@compact", 0, {}, 8192, "compact"),
    ("MultiClassPA", 2, {"nClasses": 4}, 8192),
    ("MultiClassPA@4096", 2, {"nClasses": 4}, 4096),
    ("MultiClassPA@compact", 2, {"nClasses": 4}, 8192, "compact"),
    ("ORR", 1, {}, 1),
    ("K-means", 0, {"k": 16}, 1),
    ("K-means@k256", 0, {"k": 256}, 1),  # matrix-core distances (k >= 32)
    # 512 spokes × 256 rows: fastest of 256..2048 (bench/sweep_cases_nn.json)
    ("NN", 0, {"hiddenLayers": [64, 64]}, 512),
    ("NN@bf16", 0, {"hiddenLayers": [64, 64], "matmulDtype": "bf16"}, 512),
    ("HT", 2, {"nClasses": 4}, 1),
]

# --preset p16: every learner at the reference's parallelism (16 spokes per GPU,
# DefaultJobParameters.scala:5), 131072-row rounds = 8192 rows per spoke, the engine's
# field-aware wire (the hashed-linear learners take the v3 table scan there; SVM's L2
# shrink, Pegasos and bf16 models the spoke-table round)
P16_CASES = [
    ("PA", 0, {}, 16, "compact"),
    ("SVM", 0, {}, 16, "compact"),
    ("SVM@l2", 0, {"lambda": 1e-4}, 16, "compact"),
    ("SVM@pegasos", 0, {"variant": "Pegasos", "lambda": 1e-4}, 16, "compact"),
    ("SVM@bf16", 0, {"modelDtype": "bf16"}, 16, "compact"),
    ("RegressorPA", 1, {}, 16, "compact"),
    ("LogisticRegression", 0, {}, 16, "compact"),
    ("MultiClassPA", 2, {"nClasses": 4}, 16, "compact"),
    ("MultiClassPA@k2", 2, {"nClasses": 2}, 16, "compact"),  # the binary-scan form
    ("ORR", 1, {}, 16),
    ("K-means", 0, {"k": 16}, 16),
    ("NN", 0, {"hiddenLayers": [64, 64]}, 16),
    ("HT", 2, {"nClasses": 4}, 16),                     # per-point split checks (default)
    ("HT@check1024", 2, {"nClasses": 4, "checkEvery": 1024}, 16),
    ("HT@hostloop", 2, {"nClasses": 4, "exactDevice": False}, 16),  # the host-driven A/B
    ("K-means@k256", 0, {"k": 256}, 16),               # the workgroup form (k > 64)
]


def _quality(base, task, hyper, space, ring, spokes, dev, rounds):
    """Holdout quality of the GPU learner against the same learner on the CPU (the
    reference-semantics host path), both trained on the same ``rounds`` rounds of the
    bench's stream at the bench's spokes: the learner's own evaluate() — loss per point
    and score per point (accuracy for classifiers, the learner's score otherwise)."""
    hold = synth_batch(space, 16384, start=10 ** 8, seed=26, task=task,
                       n_classes=int(hyper.get("nClasses", 4)))
    if base == "NN":
        hold = HashedBatch(hold.num, hold.cat, torch.where(hold.y > 0, 1.0, -1.0))
    ctx = RoundContext(spokes=spokes)
    out = {}
    for where in (dev, torch.device("cpu")):
        L = make_learner(base, hyper, space, where)
        t = time.perf_counter()
        for k in range(rounds):
            b = ring[k % 3]
            b.prep, b._padded = None, None
            L.fit(b if where == dev else b.to("cpu"), ctx)
        loss, score, n = L.evaluate(hold.to(where))
        n = max(1, int(n))
        out[where.type] = {"loss": round(float(loss) / n, 6), "score": round(float(score) / n, 6),
                           "fit_s": round(time.perf_counter() - t, 3)}
    out["score_gap"] = round(out[dev.type]["score"] - out["cpu"]["score"], 6)
    out["rounds"] = rounds
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--preset", default="", choices=["", "p16"],
                    help="p16: every learner at 16 spokes (the reference's parallelism)")
    ap.add_argument("--quality-rounds", type=int, default=2,
                    help="rounds of the GPU-vs-CPU holdout quality check per learner (0: off)")
    ap.add_argument("--cases", default="",
                    help='JSON list of [name, task, hyper, spokes] replacing the default cases '
                         '(geometry sweeps)')
    a = ap.parse_args(argv)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    spaces = {"wide": FeatureSpace(13, 0, 26, 1 << 20),
              "compact": FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)}
    res = {}
    cases = [tuple(c) for c in json.loads(a.cases)] if a.cases else (
        P16_CASES if a.preset == "p16" else CASES)
    for case in cases:
        name, task, hyper, spokes = case[:4]
        space = spaces[case[4] if len(case) > 4 else "wide"]
        if a.only and name.split("@")[0] not in a.only.split(","):
            continue
        ring = []
        for k in range(3):
            b = synth_batch(space, a.batch, start=k * a.batch, seed=25, task=task,
                            n_classes=int(hyper.get("nClasses", 4)))
            if name.split("@")[0] in ("NN",):
                b = HashedBatch(b.num, b.cat, torch.where(b.y > 0, 1.0, -1.0))
            ring.append(b.to(dev))
        L = make_learner(name.split("@")[0], hyper, space, dev)
        ctx = RoundContext(spokes=spokes)
        try:
            # warm every v3 prep workspace set of the ring (ops.linear S3_SLOT_RING) too
            for k in range(18):
                ring[k % 3].prep, ring[k % 3]._padded = None, None
                L.fit(ring[k % 3], ctx)
        except RuntimeError as e:  # a geometry the host guards refuse (sweeps)
            res[name] = {"error": str(e), "spokes": spokes}
            continue
        if dev.type == "cuda":
            torch.cuda.synchronize()
        from omldm_amd.ops import linear as OL

        if dev.type == "cuda":  # out of the idle clocks the host-side setup left behind
            xs = torch.randn(2048, 2048, device=dev)
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                xs = torch.tanh(xs @ xs)
                torch.cuda.synchronize()
            del xs
        v3_before = OL.SCAN3_ROUNDS
        t = time.perf_counter()
        for k in range(a.steps):
            b = ring[k % 3]
            b.prep, b._padded = None, None  # every round makes its own v3 prep (a new batch)
            L.fit(b, ctx)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        el = time.perf_counter() - t
        res[name] = {"examples_per_s": round(a.steps * a.batch / el, 1),
                     "ms_per_round": round(el / a.steps * 1e3, 3), "spokes": spokes,
                     "rows_per_spoke": -(-a.batch // spokes),
                     "v3_table_scan": OL.SCAN3_ROUNDS > v3_before}
        tot = L.running_totals() if hasattr(L, "running_totals") else {}
        if "overflow" in tot:
            res[name]["overflow"] = tot["overflow"]
        if a.quality_rounds > 0 and dev.type == "cuda":
            try:
                res[name]["quality"] = _quality(name.split("@")[0], task, hyper, space, ring,
                                                spokes, dev, a.quality_rounds)
            except (RuntimeError, NotImplementedError, ValueError) as e:
                res[name]["quality"] = {"error": str(e)[:200]}
            print(name, res[name], file=sys.stderr, flush=True)
    print(json.dumps({"metric": "per-learner training examples/s (1 GPU, 1 pipeline)",
                      "batch": a.batch, "steps": a.steps, "device": str(dev),
                      "learners": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
