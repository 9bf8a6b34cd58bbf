"""Holdout test sets of the virtual spokes of one rank, kept on the device.

Reference (omldm/operators/spoke/FlinkSpoke.scala:38-41,95-104): EVERY spoke runs its own
counter 0..9 over the training points it receives; its points 8 and 9 of every 10 are
appended to its own FIFO test set of ``testSetSize``; when that FIFO is full the evicted
(oldest) point is trained on instead. A query scores each spoke's test set (:160-163, the
−1 query :136-138) and ResponseConstructor averages the P spoke answers
(omldm/utils/ResponseConstructor.scala:32-52).

Micro-batch form. A rank runs S virtual spokes; the tick's B training rows are dealt to
them in contiguous shards (spoke s: rows [s·⌈B/S⌉, (s+1)·⌈B/S⌉)), the order the round
itself shards a batch in. Each spoke classifies its shard's positions with its own
counter; held rows enter its ring in order; rows they evict (and, once the ring is full,
the earliest held rows of the same shard) join that spoke's training rows. The training
batch is spoke-major — spoke s's rows are contiguous — and records each spoke's row
count (``HashedBatch.shards``), so the round trains spoke s's rows on spoke s.

Which rows are held depends only on the counters, so the host computes one small
descriptor per spoke and two kernels move the rows (csrc/kernels/holdout.hip,
``omldm_holdout_route_spokes``): no index arrays, no host synchronisation.
"""
from __future__ import annotations

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch, index_tensor

DESC_W = 12  # int64 words per spoke descriptor (csrc/kernels/holdout.hip: SpokeDesc)


def held_before(x: int) -> int:
    """Held positions among counter values [0, x): 8 and 9 of every ten."""
    return (x // 10) * 2 + max(0, x % 10 - 8)


def nonheld_row(r: np.ndarray, c: int) -> np.ndarray:
    q = min(c, 8) + r
    return (q // 8) * 10 + (q % 8) - c


def held_row(r: np.ndarray, c: int) -> np.ndarray:
    q = max(c - 8, 0) + r
    return (q // 2) * 10 + 8 + (q % 2) - c


class HoldoutSet:
    def __init__(self, space: FeatureSpace, size: int, device, num_dtype=torch.float32,
                 spokes: int = 1):
        self.size = int(size)
        self.spokes = max(1, int(spokes))
        self.device = torch.device(device)
        self.space = space
        S = self.spokes
        # spoke s's ring: rows [s·size, (s+1)·size)
        self.ring = HashedBatch.empty(space, S * self.size, device=self.device,
                                      num_dtype=num_dtype)
        self.count = np.zeros(S, dtype=np.int64)   # reference counter (mod 10), per spoke
        self.head = np.zeros(S, dtype=np.int64)    # next write position, per spoke
        self.filled = np.zeros(S, dtype=np.int64)
        # descriptor staging: a ring of pinned host slots (the H2D copy reads a slot when
        # the stream runs it; the slot is reused RING ticks later, after its event)
        self._ring = None
        self._ring_i = 0

    _held_before = staticmethod(held_before)

    # ------------------------------------------------------------------ routing
    def shard_bounds(self, B: int) -> list[tuple[int, int]]:
        """Spoke s's rows of a B-row tick: [s·⌈B/S⌉, (s+1)·⌈B/S⌉) ∩ [0, B)."""
        S = self.spokes
        R = -(-B // S) if B else 0
        return [(min(s * R, B), min(s * R + R, B)) for s in range(S)]

    @staticmethod
    def _held_before_v(x: np.ndarray) -> np.ndarray:
        return (x // 10) * 2 + np.maximum(0, x % 10 - 8)

    def _plan(self, B: int, out: np.ndarray | None = None) -> np.ndarray:
        """One descriptor per spoke (b0, n0, n1, r1, n2, s2, ns, hs, rw, o0, c, 0) and the
        advanced counters / heads / fills — vectorised over the spokes (the tick's host
        cost). n0 non-held rows, n1 evicted ring rows from r1, n2 held rows from
        hold-ordinal s2 that never fit; ns held rows from ordinal hs written to the ring
        from rw."""
        S, size = self.spokes, self.size
        R = -(-B // S) if B else 0
        a = np.minimum(np.arange(S, dtype=np.int64) * R, B)
        Bs = np.minimum(a + R, B) - a
        c, head, filled = self.count, self.head, self.filled
        n_hold = self._held_before_v(c + Bs) - self._held_before_v(c)
        n0 = Bs - n_hold
        r1 = (head - filled) % size
        full = n_hold >= size
        n1 = np.where(full, filled, np.maximum(0, filled + n_hold - size))
        n2 = np.where(full, n_hold - size, 0)
        ns = np.where(full, size, n_hold)
        hs = np.where(full, n_hold - size, 0)
        rw = np.where(full, 0, head)
        n_out = n0 + n1 + n2
        o = np.concatenate([[0], np.cumsum(n_out)[:-1]])
        desc = out if out is not None else np.zeros((S, DESC_W), dtype=np.int64)
        for j, v in enumerate((a, n0, n1, r1, n2, np.zeros_like(a), ns, hs, rw, o, c)):
            desc[:, j] = v
        desc[:, 11] = 0
        self.count = (c + Bs) % 10
        self.head = np.where(full, 0, (head + n_hold) % size)
        self.filled = np.where(full, size, np.minimum(size, filled + n_hold))
        return desc

    def _route_device(self, batch: HashedBatch, desc: np.ndarray) -> HashedBatch:
        from omldm_amd.ops import native

        S = self.spokes
        n = desc[:, 1] + desc[:, 2] + desc[:, 4]
        n_out = int(n.sum())
        out = HashedBatch(torch.empty((n_out, batch.dn), dtype=batch.num.dtype, device=self.device),
                          torch.empty((n_out, batch.dc), dtype=batch.cat.dtype, device=self.device),
                          torch.empty(n_out, dtype=torch.float32, device=self.device),
                          cat_span=batch.cat_span)
        # descriptors: a pinned ring slot → its device twin on the compute stream (no
        # host sync, no allocation per tick)
        host, dev, ev = self._slot()
        host.numpy()[:] = desc
        st = torch.cuda.current_stream(self.device)
        dev.copy_(host, non_blocking=True)
        ev.record(st)
        p = native.ptr
        rc = native.hip().omldm_holdout_route_spokes(
            p(batch.num), p(batch.cat), p(batch.y), batch.B, p(self.ring.num), p(self.ring.cat),
            p(self.ring.y), self.size, S, p(out.num), p(out.cat), p(out.y), n_out,
            host.numpy().ctypes.data, p(dev), batch.dn, batch.dc, batch.num.element_size(),
            batch.cat.element_size(), st.cuda_stream)
        native.check(rc, "omldm_holdout_route_spokes")
        return out

    RING = 8

    def _slot(self):
        if self._ring is None:
            self._ring = [(torch.zeros((self.spokes, DESC_W), dtype=torch.int64).pin_memory(),
                           torch.zeros((self.spokes, DESC_W), dtype=torch.int64,
                                       device=self.device), torch.cuda.Event())
                          for _ in range(self.RING)]
            self._ring_fresh = [True] * self.RING
        i = self._ring_i
        self._ring_i = (i + 1) % self.RING
        host, dev, ev = self._ring[i]
        if not self._ring_fresh[i]:
            ev.synchronize()  # its copy ran RING routes ago: normally long done
        self._ring_fresh[i] = False
        return host, dev, ev

    def _route_host(self, batch: HashedBatch, desc: np.ndarray) -> HashedBatch:
        """The same rows in the same order by explicit index arrays (CPU jobs, dtype
        mismatches); the ring is written after the evicted rows are read."""
        size = self.size
        widx, wsrc = [], []
        order = []  # ("b", idx) / ("r", idx) segments in output order
        for s in range(self.spokes):
            b0, n0, n1, r1, n2, s2, ns, hs, rw, _, c, _ = (int(v) for v in desc[s])
            order.append(("b", b0 + nonheld_row(np.arange(n0), c)))
            order.append(("r", s * size + (r1 + np.arange(n1)) % size))
            order.append(("b", b0 + held_row(s2 + np.arange(n2), c)))
            widx.append(s * size + (rw + np.arange(ns)) % size)
            wsrc.append(b0 + held_row(hs + np.arange(ns), c))
        parts = []
        for kind, idx in order:
            if idx.size == 0:
                continue
            if kind == "b":
                parts.append(batch.select(idx).without_raw())
            else:
                r = self.ring.select(idx).to(batch.y.device)
                parts.append(HashedBatch(r.num.to(batch.num.dtype), r.cat, r.y, None,
                                         batch.cat_span))
        out = HashedBatch.cat_batches(parts) if parts else batch.slice(0, 0).without_raw()
        w = np.concatenate(widx) if widx else np.zeros(0, dtype=np.int64)
        if w.size:
            self._scatter(w, batch.select(np.concatenate(wsrc)))
        return out

    def route(self, batch: HashedBatch) -> HashedBatch:
        """The rows to train on this round (holdout-evicted rows included), spoke-major,
        with ``shards`` = the per-spoke row counts."""
        B = batch.B
        if B == 0 or self.size == 0:
            if B:
                batch.shards = tuple(b - a for a, b in self.shard_bounds(B))
            return batch
        desc = self._plan(B)
        if (self.device.type == "cuda" and batch.y.device == self.device
                and batch.num.dtype == self.ring.num.dtype and batch.cat.dtype == self.ring.cat.dtype
                and all(t.is_contiguous() for t in (batch.num, batch.cat, batch.y))):
            out = self._route_device(batch, desc)
        else:
            out = self._route_host(batch, desc)
        out.shards = tuple(int(v) for v in desc[:, 1] + desc[:, 2] + desc[:, 4])
        return out

    def _scatter(self, pos, rows: HashedBatch):
        p = index_tensor(pos, self.device)
        self.ring.num[p] = rows.num.to(self.device, self.ring.num.dtype)
        self.ring.cat[p] = rows.cat.to(self.device)
        self.ring.y[p] = rows.y.to(self.device)

    # ------------------------------------------------------------------ test sets
    def _spoke_order(self, s: int) -> np.ndarray:
        f = int(self.filled[s])
        return s * self.size + (np.arange(f) + int(self.head[s]) - f) % max(1, self.size)

    def test_sets(self) -> list[HashedBatch]:
        """Each spoke's test set, oldest row first."""
        return [self.ring.select(self._spoke_order(s)) for s in range(self.spokes)]

    def test_set(self) -> HashedBatch:
        """Every spoke's test rows, spoke-major (``shards``: rows per spoke)."""
        idx = [self._spoke_order(s) for s in range(self.spokes)]
        out = self.ring.select(np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64))
        out.shards = tuple(int(i.size) for i in idx)
        return out

    @property
    def n_test(self) -> int:
        return int(self.filled.sum())

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        return {"num": self.ring.num.cpu(), "cat": self.ring.cat.cpu(), "y": self.ring.y.cpu(),
                "count": self.count.tolist(), "head": self.head.tolist(),
                "filled": self.filled.tolist(), "spokes": self.spokes, "size": self.size}

    @staticmethod
    def _spoke_rows(sd: dict) -> list[tuple[torch.Tensor, ...]]:
        """Each saved spoke's rows, oldest first (a pre-spoke checkpoint is one spoke)."""
        cnt = sd["count"]
        S = int(sd.get("spokes", 1 if np.isscalar(cnt) else len(cnt)))
        size = int(sd.get("size", sd["num"].shape[0] // max(1, S)))
        heads = np.atleast_1d(np.asarray(sd["head"], dtype=np.int64))
        fills = np.atleast_1d(np.asarray(sd["filled"], dtype=np.int64))
        out = []
        for s in range(S):
            f = int(fills[s])
            idx = torch.from_numpy(s * size + (np.arange(f) + int(heads[s]) - f) % max(1, size))
            out.append((sd["num"][idx], sd["cat"][idx], sd["y"][idx]))
        return out

    def load_merged(self, sds: list[dict]) -> HashedBatch | None:
        """Re-scaled restore: the spoke rings of the old ranks this rank takes over, dealt
        to this rank's spokes (old spoke i → new spoke i mod S, oldest rows first). Rows
        beyond a ring's ``size`` are returned to be trained on (reference restore: the
        merged test set is popped down to its maximum size and the popped points are fed
        to every pipeline, FlinkSpoke.scala:307-317)."""
        S = self.spokes
        self.count[:], self.head[:], self.filled[:] = 0, 0, 0
        if not sds:
            return None
        old = [r for sd in sds for r in self._spoke_rows(sd)]
        counts = [c for sd in sds for c in np.atleast_1d(np.asarray(sd["count"]))]
        spill = []
        for s in range(S):
            mine = old[s::S]
            if not mine:
                continue
            num = torch.cat([m[0] for m in mine])
            cat = torch.cat([m[1] for m in mine])
            y = torch.cat([m[2] for m in mine])
            n = num.shape[0]
            keep = min(n, self.size)
            sp = n - keep
            if keep:
                a = s * self.size
                self.ring.num[a:a + keep] = num[sp:].to(self.device, self.ring.num.dtype)
                self.ring.cat[a:a + keep] = cat[sp:].to(self.device)
                self.ring.y[a:a + keep] = y[sp:].to(self.device)
            self.filled[s], self.head[s] = keep, keep % max(1, self.size)
            self.count[s] = int(counts[s % len(counts)]) if counts else 0
            if sp:
                spill.append(HashedBatch(num[:sp].to(self.ring.num.dtype), cat[:sp], y[:sp],
                                         cat_span=self.ring.cat_span))
        return HashedBatch.cat_batches(spill) if spill else None

    def load_state_dict(self, sd: dict) -> HashedBatch | None:
        """Same-rank restore. A checkpoint of a different spoke count (or the pre-spoke
        single ring) is dealt like a re-scaled restore; its overflow is returned."""
        cnt = sd["count"]
        S_old = int(sd.get("spokes", 1 if np.isscalar(cnt) else len(cnt)))
        if S_old != self.spokes or int(sd.get("size", self.size)) != self.size:
            return self.load_merged([sd])
        n = min(self.ring.num.shape[0], sd["num"].shape[0])
        self.ring.num[:n] = sd["num"][:n].to(self.device)
        self.ring.cat[:n] = sd["cat"][:n].to(self.device)
        self.ring.y[:n] = sd["y"][:n].to(self.device)
        self.count[:] = np.asarray(sd["count"], dtype=np.int64)
        self.head[:] = np.asarray(sd["head"], dtype=np.int64) % max(1, self.size)
        self.filled[:] = np.minimum(self.size, np.asarray(sd["filled"], dtype=np.int64))
        return None
