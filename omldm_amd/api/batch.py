"""Device-friendly micro-batch of data points.

Reference: a data point is a ``LabeledPoint``/``UnlabeledPoint`` built from
(numerical DenseVector, discrete→double DenseVector, categorical String[])
(omldm/utils/parsers/dataStream/DataPointParser.scala:21-46). Here a micro-batch of
points is three flat arrays (see csrc/host/ingest.cpp for the exact layout):

* ``num`` [B, dn] float32 — numerical then discrete features (slot j = feature j)
* ``cat`` [B, dc] int32   — hashed categorical slot | sign bit, -1 = absent
* ``y``   [B]     float32 — target, NaN for forecasting points / skipped rows

Keeping the batch columnar and fixed-width is what lets a training micro-batch
travel as three pinned ``hipMemcpyAsync`` copies and be consumed by one kernel launch.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch


@dataclass(frozen=True)
class FeatureSpace:
    """Shape of the hashed feature space shared by every pipeline of a job."""

    n_numerical: int = 13
    n_discrete: int = 0
    n_categorical: int = 26
    dim: int = 1 << 20
    # Compact wire format: field-aware hashing, categorical slot carried as uint16
    # {sign, local} with slot = dn + field·cat_span + local (half the PCIe bytes).
    field_aware: bool = False

    @property
    def dn(self) -> int:
        return self.n_numerical + self.n_discrete

    @property
    def dc(self) -> int:
        return self.n_categorical

    @property
    def cat_span(self) -> int:
        if not self.field_aware or self.dc == 0:
            return 0
        return min(32767, (self.dim - self.dn - 1) // self.dc)

    @property
    def cat_dtype(self):
        return torch.int16 if self.field_aware else torch.int32

    def __post_init__(self):
        if self.dim <= self.dn:
            raise ValueError("hash dimension must exceed the number of dense slots")
        if self.dim >= 2**31:
            raise ValueError("hash dimension must fit in 31 bits")
        if self.field_aware and self.dc and (self.dim - self.dn - 1) // self.dc < 1:
            raise ValueError("hash dimension too small for field-aware hashing")


def index_tensor(idx, device) -> torch.Tensor:
    """Host index array (ndarray / CPU tensor) → int64 tensor on ``device``. On GPUs the
    copy goes through a pinned block of the caching host allocator and is
    non-blocking: a pageable ``.to(device)`` would wait for the whole stream (the
    previous round's kernels) before returning."""
    if isinstance(idx, np.ndarray):
        idx = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64))
    device = torch.device(device)
    if idx.device == device:
        return idx
    if device.type == "cuda" and idx.device.type == "cpu":
        return idx.to(torch.int64).pin_memory().to(device, non_blocking=True)
    return idx.to(device)


@dataclass
class HashedBatch:
    num: torch.Tensor
    cat: torch.Tensor
    y: torch.Tensor
    raw: list | None = field(default=None, compare=False)  # optional raw records (forecasting)
    cat_span: int = 0  # > 0: compact uint16 field-aware categorical format (int16 storage)
    # rows per virtual spoke of a spoke-major batch (engine/holdout.py routes a tick into
    # one), or None; a plain attribute, not carried by slicing / selection
    shards = None
    # a v3 scan prep made for this batch (ops.linear.Scan3Prep), shared by the pipelines
    # that train on it within a tick; a plain attribute like ``shards``
    prep = None
    # (spokes, padded batch): spoke_padded's result, made once per tick (engine/job.py may
    # make it ahead on its prep stream)
    _padded = None

    @property
    def B(self) -> int:
        return int(self.y.shape[0])

    @property
    def dn(self) -> int:
        return int(self.num.shape[1])

    @property
    def dc(self) -> int:
        return int(self.cat.shape[1])

    @property
    def device(self):
        return self.y.device

    def __len__(self):
        return self.B

    @staticmethod
    def empty(space: FeatureSpace, B: int = 0, device="cpu", pin: bool = False,
              num_dtype=torch.float32) -> "HashedBatch":
        kw = dict(device=device)
        if pin and torch.cuda.is_available():
            kw["pin_memory"] = True
        return HashedBatch(
            torch.zeros((B, space.dn), dtype=num_dtype, **kw),
            torch.full((B, space.dc), -1, dtype=space.cat_dtype, **kw),
            torch.full((B,), float("nan"), dtype=torch.float32, **kw),
            cat_span=space.cat_span,
        )

    def _like(self, num, cat, y, raw) -> "HashedBatch":
        return HashedBatch(num, cat, y, raw, self.cat_span)

    def to(self, device, non_blocking: bool = False) -> "HashedBatch":
        out = self._like(self.num.to(device, non_blocking=non_blocking),
                         self.cat.to(device, non_blocking=non_blocking),
                         self.y.to(device, non_blocking=non_blocking), self.raw)
        out.shards = self.shards  # the same rows: the spoke layout travels with them
        return out

    def slice(self, a: int, b: int) -> "HashedBatch":
        return self._like(self.num[a:b], self.cat[a:b], self.y[a:b],
                          None if self.raw is None else self.raw[a:b])

    def select(self, idx) -> "HashedBatch":
        raw = None
        if self.raw is not None:
            host = idx if isinstance(idx, np.ndarray) else idx.cpu().numpy()
            raw = [self.raw[int(i)] for i in host]
        idx = index_tensor(idx, self.y.device)
        return self._like(self.num[idx], self.cat[idx], self.y[idx], raw)

    @staticmethod
    def cat_batches(batches: list["HashedBatch"]) -> "HashedBatch":
        batches = [b for b in batches if b is not None]
        raw = None
        if any(b.raw is not None for b in batches):
            raw = []
            for b in batches:
                raw.extend(b.raw if b.raw is not None else [None] * b.B)
        return HashedBatch(torch.cat([b.num for b in batches]), torch.cat([b.cat for b in batches]),
                           torch.cat([b.y for b in batches]), raw, batches[0].cat_span)

    def without_raw(self) -> "HashedBatch":
        return self._like(self.num, self.cat, self.y, None)

    def contiguous(self) -> "HashedBatch":
        return self._like(self.num.contiguous(), self.cat.contiguous(), self.y.contiguous(),
                          self.raw)

    def cat_slots(self) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(slot [B, dc] int64, sign [B, dc] float, valid [B, dc] bool) for either format."""
        if self.cat_span > 0:
            c = self.cat.long() & 0xFFFF
            valid = c != 0xFFFF
            f = torch.arange(self.dc, device=c.device).unsqueeze(0)
            slot = self.dn + f * self.cat_span + (c & 0x7FFF)
            sign = torch.where((c & 0x8000) != 0, -1.0, 1.0)
            return slot, sign, valid
        c = self.cat.long()
        return c & 0x7FFFFFFF, torch.where(c < 0, -1.0, 1.0), c != -1

    def to_wide(self) -> "HashedBatch":
        """Compact uint16 categorical form → int32 signed-slot form (no-op if wide)."""
        if self.cat_span == 0:
            return self
        slot, sign, valid = self.cat_slots()
        c = torch.where(sign < 0, slot | 0x80000000, slot)
        c = torch.where(valid, c, torch.full_like(c, -1)).to(torch.int64)
        c32 = ((c + 2**31) % 2**32 - 2**31).to(torch.int32)
        return HashedBatch(self.num, c32.contiguous(), self.y, self.raw, 0)

    def spoke_padded(self, spokes: int) -> "HashedBatch":
        """A spoke-major batch (``shards`` = rows per spoke) laid out as spokes × R rows,
        R = max(shards): spoke s's rows at [s·R, s·R + shards[s]), the rest unlabeled
        (y NaN, no features — the linear rounds skip them). Sharding it in R-row blocks
        then trains every row on the spoke that routed it. Unchanged when the shards are
        equal (or absent / of another spoke count)."""
        sh = self.shards
        if sh is None or len(sh) != spokes or len(set(sh)) <= 1 or not self.B:
            return self
        if self._padded is not None and self._padded[0] == spokes:
            return self._padded[1]
        R = max(sh)
        idx = np.full(spokes * R, self.B, dtype=np.int64)  # row B: the blank row
        o = 0
        for s, n in enumerate(sh):
            idx[s * R:s * R + n] = np.arange(o, o + n)
            o += n
        ix = index_tensor(idx, self.y.device)
        num = torch.cat([self.num, self.num.new_zeros((1, self.dn))])
        cat = torch.cat([self.cat, self.cat.new_full((1, self.dc), -1)])
        y = torch.cat([self.y, self.y.new_full((1,), float("nan"))])
        out = HashedBatch(num[ix], cat[ix], y[ix], None, self.cat_span)
        out.shards = (R,) * spokes
        self._padded = (spokes, out)
        return out

    def dense(self, dim: int | None = None) -> torch.Tensor:
        """Materialise [B, dim] dense features (tests / small dense learners only)."""
        dim = dim or (self.dn + 1)
        B = self.B
        out = torch.zeros((B, dim), dtype=torch.float32, device=self.y.device)
        dn = min(self.dn, dim)
        out[:, :dn] = self.num[:, :dn].float()
        slot, sign, valid = self.cat_slots()
        valid = valid & (slot < dim)
        rows = torch.arange(B, device=out.device).unsqueeze(1).expand_as(slot)
        out.index_put_((rows[valid], slot[valid]), sign[valid], accumulate=True)
        return out


@dataclass
class PolyBatch(HashedBatch):
    """A training batch whose dense learner input is PolynomialFeatures(2) of ``num`` —
    ``[num, num[:, a]·num[:, b] for (a, b) in pairs]`` — left unexpanded. The pipeline hands
    it to learners that fuse the expansion into their update (ORR's Gram kernel reads the
    d raw values per row instead of the d + d(d+1)/2 expanded ones); ``expanded()`` is the
    materialised batch for everything else."""

    pairs: torch.Tensor | None = field(default=None, compare=False)  # int32 [np, 2]

    def _like(self, num, cat, y, raw) -> "PolyBatch":
        return PolyBatch(num, cat, y, raw, self.cat_span, self.pairs)

    def expanded(self) -> HashedBatch:
        from omldm_amd.ops.preprocess import poly_expand

        x = self.num.float().contiguous()
        num = poly_expand(x, self.pairs) if self.B else torch.zeros(
            (0, x.shape[1] + self.pairs.shape[0]), dtype=torch.float32, device=x.device)
        return HashedBatch(num, self.cat, self.y, self.raw, self.cat_span)


ABSENT_TOKEN = 0xFFFFFFFF


@dataclass
class RawBatch:
    """A micro-batch on the raw binary wire: categorical values travel as 32-bit token
    ids and are hashed on the device inside the training kernel (csrc/kernels/
    linear_seq.hip), so feature hashing is part of the timed hot path.

    * ``num`` [B, dn] float32 — numerical then discrete features
    * ``tok`` [B, dc] int32   — raw token id per field (bit pattern of a uint32;
      0xFFFFFFFF = absent); hashed like ``hash_cat`` of its 4 little-endian bytes
    * ``y``   [B]     float32 (NaN = no target) or int8 (±1 classification labels)
    """

    num: torch.Tensor
    tok: torch.Tensor
    y: torch.Tensor
    # passes 1-3 of the v3 round made ahead of the round (ops.linear.Scan3Prep), or None
    prep: object = None
    # > 0: ``tok`` holds the engine's compact int16 field-aware slots (HashedBatch.cat with
    # this cat_span) instead of tokens — the v3 round reads them as they are; their slots
    # start at ``cbase`` (the feature space's dense slot count: a preprocessor that widens
    # ``num`` does not move them)
    span: int = 0
    cbase: int = 0

    @property
    def B(self) -> int:
        return int(self.y.shape[0])

    @property
    def dn(self) -> int:
        return int(self.num.shape[1])

    @property
    def dc(self) -> int:
        return int(self.tok.shape[1])

    @property
    def device(self):
        return self.y.device

    def __len__(self):
        return self.B

    @staticmethod
    def empty(space: FeatureSpace, B: int = 0, device="cpu", pin: bool = False,
              y_dtype=torch.float32) -> "RawBatch":
        kw = dict(device=device)
        if pin and torch.cuda.is_available():
            kw["pin_memory"] = True
        return RawBatch(torch.zeros((B, space.dn), dtype=torch.float32, **kw),
                        torch.full((B, space.dc), -1, dtype=torch.int32, **kw),
                        torch.zeros((B,), dtype=y_dtype, **kw))

    def to(self, device, non_blocking: bool = False) -> "RawBatch":
        return RawBatch(self.num.to(device, non_blocking=non_blocking),
                        self.tok.to(device, non_blocking=non_blocking),
                        self.y.to(device, non_blocking=non_blocking))

    def slice(self, a: int, b: int) -> "RawBatch":
        return RawBatch(self.num[a:b], self.tok[a:b], self.y[a:b])

    def hashed(self, space: FeatureSpace) -> HashedBatch:
        """The wide hashed form (int32 signed slots) every learner reads."""
        from omldm_amd.ops.ingest import hash_raw

        return HashedBatch(self.num, hash_raw(self.tok, space), self.y.float(), None, 0)
