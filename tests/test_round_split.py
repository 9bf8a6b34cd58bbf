"""Ticks larger than ``roundRows`` rows per spoke train in several Synchronous rounds
(engine/job.py: Job._round_split): round i gives spoke s its rows [i·rr, (i+1)·rr) in
stream order — equal shards as strided views, unequal ones by index."""
from types import SimpleNamespace

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.io.synthetic import synth_batch


def _split(batch, shards, rr):
    batch.shards = tuple(shards)
    me = SimpleNamespace(cfg=SimpleNamespace(roundRows=rr), spokes=len(shards))
    return Job._round_split(me, batch)


def _rows(b):
    return [tuple(r) for r in torch.cat([b.num, b.cat.float(), b.y[:, None]], 1).tolist()]


def test_equal_shards_split_in_stream_order():
    sp = FeatureSpace(3, 0, 4, 1 << 10, field_aware=True)
    b = synth_batch(sp, 4 * 300, seed=1)
    parts = _split(b, [300] * 4, 128)
    assert [p.shards for p in parts] == [(128,) * 4, (128,) * 4, (44,) * 4]
    rows = _rows(b)
    for i, p in enumerate(parts):
        lo, hi = 128 * i, min(300, 128 * (i + 1))
        want = [rows[s * 300 + r] for s in range(4) for r in range(lo, hi)]
        assert _rows(p) == want


def test_unequal_shards_and_no_split():
    sp = FeatureSpace(2, 0, 3, 1 << 10, field_aware=True)
    sh = [100, 260, 0, 129]
    b = synth_batch(sp, sum(sh), seed=2)
    parts = _split(b, sh, 128)
    assert [p.shards for p in parts] == [(100, 128, 0, 128), (0, 128, 0, 1), (0, 4, 0, 0)]
    rows, starts = _rows(b), np.concatenate([[0], np.cumsum(sh)[:-1]])
    for i, p in enumerate(parts):
        want = [rows[a + r] for a, n in zip(starts, sh) for r in range(128 * i, min(n, 128 * (i + 1)))]
        assert _rows(p) == want
    assert sum(p.B for p in parts) == b.B
    assert _split(b, sh, 0) == [b] and _split(b, sh, 260) == [b]
