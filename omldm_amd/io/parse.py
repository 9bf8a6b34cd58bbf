"""DataInstance JSON → HashedBatch (C++ multi-threaded scanner, csrc/host/ingest.cpp).

Reference: DataInstanceParser (skip "EOS", drop malformed records silently,
omldm/utils/parsers/DataInstanceParser.scala:12-22) + DataPointParser
(omldm/utils/parsers/dataStream/DataPointParser.scala:16-55). Dropped records are
counted instead of silently swallowed.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.ops import native

OP_TRAINING, OP_FORECASTING, OP_INVALID = 0, 1, -1


def hash_categorical(token: str, field: int, space: FeatureSpace) -> int:
    b = token.encode()
    if space.cat_span:
        return int(native.host().omldm_hash_cat16(b, len(b), field, space.cat_span))
    return int(native.host().omldm_hash_cat(b, len(b), field, space.dn, space.dim))


class RawView:
    """Lazy per-record view of a parsed block (the raw text is only materialised for
    the records that need it: forecasts echo their point in the Prediction)."""

    __slots__ = ("buf", "offs", "ends")

    def __init__(self, buf, offs: np.ndarray, ends: np.ndarray | None = None):
        self.buf, self.offs, self.ends = buf, offs, ends

    def __len__(self):
        return len(self.offs) - 1

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        i = int(i)
        e = self.offs[i + 1] if self.ends is None else self.ends[i]
        r = self.buf[int(self.offs[i]):int(e)]
        if not isinstance(r, bytes):  # a view of a pinned staging slot
            r = r.tobytes()
        return r.rstrip(b"\n")

    def __iter__(self):
        return (self[i] for i in range(len(self)))


def parse_block(buf, offs: np.ndarray, space: FeatureSpace, threads: int | None = None):
    """Parses buf[offs[i]:offs[i+1]] for every i (``buf``: bytes or a uint8 ndarray,
    e.g. a staging slot). Returns (batch, op, n_valid)."""
    n = len(offs) - 1
    num = torch.zeros((n, space.dn), dtype=torch.float32)
    cat = torch.full((n, space.dc), -1, dtype=space.cat_dtype)
    y = torch.full((n,), float("nan"), dtype=torch.float32)
    op = np.full(n, -1, dtype=np.int8)
    valid = 0
    if n > 0:
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        threads = threads or min(8, os.cpu_count() or 1)
        src = buf if isinstance(buf, bytes) else \
            C.cast(C.c_void_p(np.ascontiguousarray(buf).ctypes.data), C.c_char_p)
        valid = native.host().omldm_parse_instances(
            src, offs.ctypes.data, n, space.n_numerical, space.n_discrete, space.dc, space.dim,
            space.cat_span, num.data_ptr(), cat.data_ptr(), y.data_ptr(), op.ctypes.data,
            threads)
    return HashedBatch(num, cat, y, RawView(buf, offs), space.cat_span), op, int(valid)


def parse_records(records: list, space: FeatureSpace, threads: int | None = None,
                  keep_raw: bool = True):
    """Returns (batch, op[int8 ndarray], n_valid). Invalid rows have op == -1."""
    n = len(records)
    enc = [r if isinstance(r, (bytes, bytearray)) else str(r).encode() for r in records]
    off = np.zeros(n + 1, dtype=np.int64)
    if n:
        np.cumsum([len(e) for e in enc], out=off[1:])
    buf = b"".join(enc)
    num = torch.zeros((n, space.dn), dtype=torch.float32)
    cat = torch.full((n, space.dc), -1, dtype=space.cat_dtype)
    y = torch.full((n,), float("nan"), dtype=torch.float32)
    op = np.full(n, -1, dtype=np.int8)
    valid = 0
    if n:
        threads = threads or min(8, os.cpu_count() or 1)
        valid = native.host().omldm_parse_instances(
            buf, off.ctypes.data, n, space.n_numerical, space.n_discrete, space.dc, space.dim,
            space.cat_span, num.data_ptr(), cat.data_ptr(), y.data_ptr(), op.ctypes.data,
            threads)
    raw = None
    if keep_raw:
        # DIB records (io/dib.py) stay bytes: their payload is not text
        raw = [e.decode() if isinstance(e, (bytes, bytearray)) and not (e and e[0] == 0xB1)
               else e for e in enc]
    return HashedBatch(num, cat, y, raw, space.cat_span), op, int(valid)
