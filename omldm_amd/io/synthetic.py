"""Synthetic training/forecasting streams (there is no network for real datasets).

``synth_batch`` produces a Criteo-shaped hashed batch straight into (pinned) host
memory with the C++ generator (csrc/host/ingest.cpp: omldm_synth_batch). Example i is
a pure function of (seed, i), so rank r of G can generate its own shard of a global
stream independently. ``synth_json_records`` renders the same kind of points as
DataInstance JSON for end-to-end tests through the parser (small volumes only).
"""
from __future__ import annotations

import json
import os
import zlib

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch, RawBatch
from omldm_amd.ops import native
from omldm_amd.ops.native import ptr

TASK_BINARY, TASK_REGRESSION, TASK_MULTICLASS = 0, 1, 2


def synth_batch(space: FeatureSpace, B: int, start: int = 0, seed: int = 25, task: int = 0,
                n_classes: int = 4, noise: float = 0.1, pin: bool = False,
                out: HashedBatch | None = None, threads: int | None = None) -> HashedBatch:
    if out is None:
        out = HashedBatch.empty(space, B, pin=pin)
    assert out.B == B and not out.y.is_cuda and out.num.dtype == torch.float32
    assert out.cat.dtype == space.cat_dtype
    threads = threads or min(16, os.cpu_count() or 1)
    native.host().omldm_synth_batch(seed, start, B, space.dn, space.dc, space.dim, task,
                                    n_classes, noise, space.cat_span, ptr(out.num), ptr(out.cat),
                                    ptr(out.y), threads)
    return out


def synth_raw(space: FeatureSpace, B: int, start: int = 0, seed: int = 25, task: int = 0,
              n_classes: int = 4, noise: float = 0.1, missing: float = 0.0, pin: bool = False,
              out: RawBatch | None = None, threads: int | None = None) -> RawBatch:
    """Criteo-shaped stream on the raw binary wire (csrc/host/rawwire.cpp:
    omldm_synth_raw): categorical values are 32-bit token ids, labels come from a hidden
    model over (field, token). Example i is a pure function of (seed, start + i)."""
    if out is None:
        out = RawBatch.empty(space, B, pin=pin)
    assert out.B == B and out.num.dtype == torch.float32 and out.tok.dtype == torch.int32
    assert out.y.dtype == torch.float32 and not out.y.is_cuda
    threads = threads or min(16, os.cpu_count() or 1)
    native.host().omldm_synth_raw(seed, start, B, space.dn, space.dc, task, n_classes, noise,
                                  missing, ptr(out.num), ptr(out.tok), ptr(out.y), threads)
    return out


def synth_json_records(n: int, space: FeatureSpace, start: int = 0, seed: int = 25,
                       operation: str = "training", task: int = 0) -> list[str]:
    """DataInstance JSON lines (numerical/discrete/categorical features + target); record i
    is a pure function of (seed, start, i) in every process (a stable CRC of each category
    string, not Python's per-process salted ``hash``)."""
    rng = np.random.default_rng(seed * 1_000_003 + start)
    wn = np.random.default_rng(seed).normal(size=space.n_numerical + space.n_discrete)
    out = []
    for i in range(n):
        xn = rng.normal(size=space.n_numerical).round(6)
        xd = rng.integers(0, 5, size=space.n_discrete)
        cats = [f"c{j}_{int(rng.integers(0, 10 ** (1 + j % 4)) ** 1)}"
                for j in range(space.n_categorical)]
        s = float(np.dot(wn, np.concatenate([xn, xd]))) + sum(
            (zlib.crc32(c.encode()) % 7 - 3) * 0.1 for c in cats)
        rec = {"numericalFeatures": xn.tolist(), "discreteFeatures": xd.tolist(),
               "categoricalFeatures": cats, "operation": operation}
        if operation == "training":
            rec["target"] = (1.0 if s >= 0 else -1.0) if task == 0 else s
        out.append(json.dumps(rec))
    return out


def ring_of_batches(space: FeatureSpace, n_batches: int, B: int, rank: int = 0, seed: int = 25,
                    task: int = 0, pin: bool = True) -> list[HashedBatch]:
    """Pre-generated pinned pool replayed by the benchmark like a Kafka log."""
    pool = []
    for k in range(n_batches):
        start = (k * 4096 + rank) * B  # disjoint stream segments per (batch, rank)
        pool.append(synth_batch(space, B, start=start, seed=seed, task=task, pin=pin))
    return pool


def device_of(pool: list[HashedBatch]) -> torch.device:
    return pool[0].y.device
