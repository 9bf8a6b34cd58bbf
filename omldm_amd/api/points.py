"""Point types of the reference's math API (``mlAPI.math`` Point,
LabeledPoint(target, num, disc, cat, raw), UnlabeledPoint, TrainingPoint,
ForecastingPoint, DenseVector, SparseVector — built by DataPointParser,
omldm/utils/parsers/dataStream/DataPointParser.scala:21-46).

The engine never materialises per-point objects: points travel as columnar micro-batches
(``HashedBatch``: numerical ∥ discrete block + hashed categorical slots + targets). These
classes are the per-point view for users and tests, with exact conversion to and from
the columnar form through the same C++ hashing as the parser.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.ops import native


@dataclass
class Point:
    numerical: list[float] = field(default_factory=list)
    discrete: list[int] = field(default_factory=list)
    categorical: list[str] = field(default_factory=list)
    raw: str | None = None

    def dense(self) -> list[float]:
        """numerical ∥ discrete→double (DataPointParser.scala:21-36)."""
        return [float(v) for v in self.numerical] + [float(v) for v in self.discrete]


@dataclass
class LabeledPoint(Point):
    target: float = 0.0


@dataclass
class UnlabeledPoint(Point):
    pass


@dataclass
class TrainingPoint:
    point: LabeledPoint


@dataclass
class ForecastingPoint:
    point: UnlabeledPoint


def to_batch(points: list[Point], space: FeatureSpace) -> HashedBatch:
    """Columnar micro-batch of points (unlabelled points get a NaN target)."""
    B = len(points)
    b = HashedBatch.empty(space, B)
    lib = native.host()
    for i, p in enumerate(points):
        d = p.dense()[: space.dn]
        b.num[i, : len(d)] = torch.tensor(d, dtype=torch.float32)
        for j in range(space.dc):
            if j >= len(p.categorical):
                b.cat[i, j] = -1
                continue
            tok = p.categorical[j].encode()
            if space.cat_span:
                v = lib.omldm_hash_cat16(tok, len(tok), j, space.cat_span)
                b.cat[i, j] = v if v < 0x8000 else v - 0x10000
            else:
                b.cat[i, j] = lib.omldm_hash_cat(tok, len(tok), j, space.dn, space.dim)
        b.y[i] = float(p.target) if isinstance(p, LabeledPoint) else float("nan")
    b.raw = [p.raw for p in points]
    return b


def sparse_vector(batch: HashedBatch, i: int) -> tuple[list[int], list[float]]:
    """(indices, values) of row i in the model's slot space (SparseVector view)."""
    idx, val = [], []
    for j in range(batch.num.shape[1]):
        v = float(batch.num[i, j])
        if v != 0.0:
            idx.append(j)
            val.append(v)
    slot, sign, valid = batch.cat_slots()
    for s, g, ok in zip(slot[i].tolist(), sign[i].tolist(), valid[i].tolist()):
        if ok:
            idx.append(int(s))
            val.append(float(g))
    return idx, val
