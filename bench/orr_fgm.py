#!/usr/bin/env python3
"""BASELINE config 4: online ridge regression with a polynomial feature map, FGM-style
asynchronous synchronisation over RCCL.

A real engine pipeline (Request → PolynomialFeatures(degree 2) → ORR, protocol FGM) is
driven round by round: per step and GPU, B rows → poly expansion kernel (13 → 104
features) → MFMA Gram update of [x, 1, y] → FGM monitoring (one fused drift-norm pass +
an 8-byte all-reduce) → a full model sync only when the safe zone is left. Data:
synthetic y = a·x + xᵀQx + noise (HBM-resident ring), so the degree-2 map is exact.

    python bench/orr_fgm.py [--steps 50 --warmup 5 --batch 262144]
    torchrun --nproc-per-node N bench/orr_fgm.py ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace, HashedBatch  # noqa: E402
from omldm_amd.api.schemas import Request  # noqa: E402
from omldm_amd.engine.pipeline import Pipeline  # noqa: E402
from omldm_amd.parallel.comm import init_distributed  # noqa: E402


def make_stream(space, B, n, rank, device, seed=11):
    g = torch.Generator().manual_seed(seed)
    d = space.dn
    a = torch.randn(d, generator=g)
    Q = torch.randn(d, d, generator=g) * 0.1
    out = []
    for k in range(n):
        gk = torch.Generator().manual_seed(seed * 1000 + rank * 100 + k)
        x = torch.randn(B, d, generator=gk)
        y = x @ a + ((x @ Q) * x).sum(1) + 0.01 * torch.randn(B, generator=gk)
        out.append(HashedBatch(x, torch.zeros((B, 0), dtype=torch.int32), y).to(device))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=262144, help="rows per GPU per step")
    ap.add_argument("--ring", type=int, default=4)
    ap.add_argument("--epsilon", type=float, default=0.05)
    a = ap.parse_args(argv)

    comm, device = init_distributed()
    rank, world = comm.rank, comm.world
    on_gpu = device.type == "cuda"
    space = FeatureSpace(13, 0, 0, 1 << 12)
    req = Request.from_json({
        "id": 1, "request": "Create", "learner": {"name": "ORR",
                                                  "hyperParameters": {"lambda": 1.0}},
        "preProcessors": [{"name": "PolynomialFeatures", "hyperParameters": {"degree": 2}}],
        "trainingConfiguration": {"protocol": "FGM", "epsilon": a.epsilon}})
    pipe = Pipeline(req, space, comm, device, spokes=1, parallelism=max(2, world))
    ring = make_stream(space, a.batch, a.ring, rank, device)

    def sync():
        if on_gpu:
            torch.cuda.synchronize(device)
        comm.barrier()

    for k in range(a.warmup):
        pipe.train(ring[k % a.ring])
    sync()
    st0 = dict(pipe.protocol.stats.as_dict())
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        pipe.train(ring[k % a.ring])
    sync()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=device if on_gpu else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    pipe.protocol.finalize()
    test = make_stream(space, 20000, 1, 999, device, seed=11)[0]
    rmse = float(((pipe.predict(test) - test.y) ** 2).mean().sqrt())
    st = pipe.protocol.stats.as_dict()
    if rank == 0:
        ex = a.steps * a.batch * world
        print(json.dumps({
            "metric": "training examples/s (whole node), ORR + PolynomialFeatures(2), FGM",
            "value": round(ex / elapsed, 1), "unit": "examples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "dtype": "fp32",
            "data": "synthetic quadratic regression stream, HBM-resident ring",
            "config": {"model": "ORR on degree-2 polynomial map of 13 features (104 dims)",
                       "global_batch": a.batch * world, "parallelism": f"dp{world}",
                       "protocol": "FGM"},
            "fgm": {"full_syncs": st["syncs"] - st0["syncs"],
                    "rounds": st["rounds"] - st0["rounds"],
                    "subrounds": getattr(pipe.protocol, "subrounds", None),
                    "bytes_shipped": st["bytesShipped"] - st0["bytesShipped"],
                    "small_messages": st["smallMessages"] - st0["smallMessages"]},
            "holdout_rmse": round(rmse, 5),
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
