"""Holdout test set of a spoke (per rank), kept on the device.

Reference (omldm/operators/spoke/FlinkSpoke.scala:95-104): a counter runs 0..9 over the
training points; points 8 and 9 of every 10 are appended to a FIFO test set of
``testSetSize``; when the FIFO is full the evicted (oldest) point is trained on instead.
The test set scores queries (:160-163) and the final statistics (:136-138).

Micro-batch form: the positions of one batch are classified by the running counter;
holdout rows enter the ring in order; rows they evict (and, once the ring is full, the
earliest rows of the same batch) join the training rows of this round.
"""
from __future__ import annotations

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch, index_tensor


class HoldoutSet:
    def __init__(self, space: FeatureSpace, size: int, device, num_dtype=torch.float32):
        self.size = int(size)
        self.device = torch.device(device)
        self.ring = HashedBatch.empty(space, self.size, device=self.device, num_dtype=num_dtype)
        self.count = 0   # reference counter (mod 10)
        self.head = 0    # next write position
        self.filled = 0

    @staticmethod
    def _held_before(x: int) -> int:
        """Held positions among counter values [0, x): 8 and 9 of every ten."""
        return (x // 10) * 2 + max(0, x % 10 - 8)

    def _route_device(self, batch: HashedBatch) -> HashedBatch:
        """GPU form of ``route``: the same rows in the same order, moved by two kernels
        (csrc/kernels/holdout.hip) from scalar segment descriptors — no index arrays,
        no host synchronisation."""
        from omldm_amd.ops import native

        B, c, size = batch.B, self.count, self.size
        n_hold = self._held_before(c + B) - self._held_before(c)
        n_train = B - n_hold
        self.count = (c + B) % 10
        if n_hold >= size:
            n1, r1 = self.filled, (self.head - self.filled) % size
            n2, s2 = n_hold - size, 0
            ns, hs, rw = size, n_hold - size, 0
            self.head, self.filled = 0, size
        else:
            n1 = max(0, self.filled + n_hold - size)
            r1 = (self.head - self.filled) % size
            n2, s2 = 0, 0
            ns, hs, rw = n_hold, 0, self.head
            self.head = (self.head + n_hold) % size
            self.filled = min(size, self.filled + n_hold)
        n_out = n_train + n1 + n2
        out = HashedBatch(torch.empty((n_out, batch.dn), dtype=batch.num.dtype, device=self.device),
                          torch.empty((n_out, batch.dc), dtype=batch.cat.dtype, device=self.device),
                          torch.empty(n_out, dtype=torch.float32, device=self.device),
                          cat_span=batch.cat_span)
        p = native.ptr
        rc = native.hip().omldm_holdout_route(
            p(batch.num), p(batch.cat), p(batch.y), B, p(self.ring.num), p(self.ring.cat),
            p(self.ring.y), size, p(out.num), p(out.cat), p(out.y), c, n_train, n1, r1, n2, s2,
            ns, hs, rw, batch.dn, batch.dc, batch.num.element_size(), batch.cat.element_size(),
            torch.cuda.current_stream(self.device).cuda_stream)
        native.check(rc, "omldm_holdout_route")
        return out

    def route(self, batch: HashedBatch) -> HashedBatch:
        """Returns the rows to train on this round (holdout-evicted rows included).
        Which rows are held out depends only on the running counter, so every index
        is computed on the host (numpy) and reaches the device as one non-blocking
        copy — no stream synchronisation on the tick's critical path."""
        B = batch.B
        if B == 0 or self.size == 0:
            return batch
        if (self.device.type == "cuda" and batch.y.device == self.device
                and batch.num.dtype == self.ring.num.dtype and batch.cat.dtype == self.ring.cat.dtype
                and all(t.is_contiguous() for t in (batch.num, batch.cat, batch.y))):
            return self._route_device(batch)
        pos = (np.arange(B, dtype=np.int64) + self.count) % 10
        self.count = (self.count + B) % 10
        hold = pos >= 8
        idx_hold = np.flatnonzero(hold)
        n_hold = int(idx_hold.size)
        if n_hold == 0:
            return batch
        idx_train = np.flatnonzero(~hold)
        out = [batch.select(idx_train)]
        if n_hold >= self.size:
            # earlier holdout rows of this batch are evicted by later ones: train on them
            if self.filled:
                out.append(self._ring_in_order())
            spill = idx_hold[: n_hold - self.size]
            if spill.size:
                out.append(batch.select(spill))
            keep = batch.select(idx_hold[n_hold - self.size:])
            self._write(0, keep)
            self.head = 0
            self.filled = self.size
        else:
            new = batch.select(idx_hold)
            n_evict = max(0, self.filled + n_hold - self.size)
            if n_evict:
                oldest = (self.head - self.filled) % self.size
                ev = (np.arange(n_evict) + oldest) % self.size
                out.append(self.ring.select(ev).to(batch.y.device))
            pos_w = (np.arange(n_hold) + self.head) % self.size
            self._scatter(pos_w, new)
            self.head = (self.head + n_hold) % self.size
            self.filled = min(self.size, self.filled + n_hold)
        return HashedBatch.cat_batches(out)

    def _write(self, at: int, rows: HashedBatch):
        n = rows.B
        self.ring.num[at:at + n] = rows.num.to(self.device, self.ring.num.dtype)
        self.ring.cat[at:at + n] = rows.cat.to(self.device)
        self.ring.y[at:at + n] = rows.y.to(self.device)

    def _scatter(self, pos, rows: HashedBatch):
        p = index_tensor(pos, self.device)
        self.ring.num[p] = rows.num.to(self.device, self.ring.num.dtype)
        self.ring.cat[p] = rows.cat.to(self.device)
        self.ring.y[p] = rows.y.to(self.device)

    def _ring_in_order(self) -> HashedBatch:
        oldest = (self.head - self.filled) % self.size
        idx = (np.arange(self.filled) + oldest) % self.size
        return self.ring.select(idx)

    def test_set(self) -> HashedBatch:
        return self._ring_in_order()

    def state_dict(self) -> dict:
        return {"num": self.ring.num.cpu(), "cat": self.ring.cat.cpu(), "y": self.ring.y.cpu(),
                "count": self.count, "head": self.head, "filled": self.filled}

    @staticmethod
    def _rows_in_order(sd: dict) -> tuple[torch.Tensor, ...]:
        size, filled = sd["num"].shape[0], int(sd["filled"])
        idx = (torch.arange(filled) + (int(sd["head"]) - filled)) % max(1, size)
        return sd["num"][idx], sd["cat"][idx], sd["y"][idx]

    def load_merged(self, sds: list[dict]) -> HashedBatch | None:
        """Re-scaled restore: the rings of several old ranks merged into this one, oldest
        rows first (old-rank order). Rows beyond ``size`` are returned to be trained on
        (reference restore: the merged test set is popped down to its maximum size and
        the popped points are fed to every pipeline, FlinkSpoke.scala:307-317)."""
        self.count, self.head, self.filled = 0, 0, 0
        if not sds:
            return None
        parts = [self._rows_in_order(sd) for sd in sds]
        num = torch.cat([p[0] for p in parts])
        cat = torch.cat([p[1] for p in parts])
        y = torch.cat([p[2] for p in parts])
        n = num.shape[0]
        keep = min(n, self.size)
        spill = n - keep
        if keep:
            self.ring.num[:keep] = num[spill:].to(self.device, self.ring.num.dtype)
            self.ring.cat[:keep] = cat[spill:].to(self.device)
            self.ring.y[:keep] = y[spill:].to(self.device)
        self.filled, self.head = keep, keep % max(1, self.size)
        self.count = int(sds[0]["count"])
        if spill == 0:
            return None
        return HashedBatch(num[:spill].to(self.ring.num.dtype), cat[:spill], y[:spill],
                           cat_span=self.ring.cat_span)

    def load_state_dict(self, sd: dict) -> None:
        n = min(self.size, sd["num"].shape[0])
        self.ring.num[:n] = sd["num"][:n].to(self.device)
        self.ring.cat[:n] = sd["cat"][:n].to(self.device)
        self.ring.y[:n] = sd["y"][:n].to(self.device)
        self.count, self.head = int(sd["count"]), int(sd["head"]) % max(1, self.size)
        self.filled = min(self.size, int(sd["filled"]))
