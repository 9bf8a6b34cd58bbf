#!/usr/bin/env python3
"""Statistical efficiency of the Synchronous linear-SVM round vs its geometry.

Holdout accuracy after a fixed number of examples of the raw Criteo-shaped stream, for
S spokes × R rows per round (exact sequential PA-I per spoke, replicas averaged per
round — csrc/host/rawwire.cpp, the same semantics as the GPU kernel). The reference
runs P = 16 sequential spokes (omldm/utils/DefaultJobParameters.scala:5); a GPU geometry
with many more spokes averages more replicas per example and learns slower per example.

    python bench/accuracy_sweep.py [--examples 4000000] [--geoms 16x4096,16x8192,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402


def run(space, S, R, examples, pool_batches, seed=25, checkpoints=()):
    B = S * R
    rounds = max(1, examples // B)
    pool = [synth_raw(space, B, start=k * B, seed=seed) for k in range(pool_batches)]
    test = synth_raw(space, 20000, start=10**10, seed=seed)
    testh = test.hashed(space)
    w = torch.zeros(space.dim)
    dacc = torch.zeros(space.dim + 2)
    rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
    curve = []
    t0 = time.perf_counter()
    for k in range(rounds):
        L.linear_seq_round(w, pool[k % pool_batches], R, S, dacc, rule, 1.0 / S)
        L.linear_apply(w, None, dacc)
        n = (k + 1) * B
        if any(n - B < c <= n for c in checkpoints) or k == rounds - 1:
            acc = float(((L.linear_predict(w, testh) >= 0).float() * 2 - 1 == testh.y).float().mean())
            curve.append((n, round(acc, 4)))
    return curve, time.perf_counter() - t0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=4_000_000)
    ap.add_argument("--geoms", default="16x4096,16x8192,32x4096,64x2048,256x512,1024x128,8192x16")
    ap.add_argument("--pool", type=int, default=0, help="distinct batches replayed (0: no replay)")
    ap.add_argument("--dim-log2", type=int, default=20)
    a = ap.parse_args(argv)
    space = FeatureSpace(13, 0, 26, 1 << a.dim_log2)
    cps = [a.examples // 8 * i for i in range(1, 9)]
    for g in a.geoms.split(","):
        S, R = (int(v) for v in g.split("x"))
        B = S * R
        pool = a.pool or max(1, a.examples // B)
        curve, el = run(space, S, R, a.examples, pool, checkpoints=cps)
        print(json.dumps({"spokes": S, "rows": R, "curve": curve, "cpu_s": round(el, 1)}), flush=True)


if __name__ == "__main__":
    main()
