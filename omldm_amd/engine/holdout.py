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

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch


class HoldoutSet:
    def __init__(self, space: FeatureSpace, size: int, device, num_dtype=torch.float32):
        self.size = int(size)
        self.device = torch.device(device)
        self.ring = HashedBatch.empty(space, self.size, device=self.device, num_dtype=num_dtype)
        self.count = 0   # reference counter (mod 10)
        self.head = 0    # next write position
        self.filled = 0

    def route(self, batch: HashedBatch) -> HashedBatch:
        """Returns the rows to train on this round (holdout-evicted rows included)."""
        B = batch.B
        if B == 0 or self.size == 0:
            return batch
        pos = (torch.arange(B) + self.count) % 10
        self.count = (self.count + B) % 10
        hold = pos >= 8
        n_hold = int(hold.sum())
        if n_hold == 0:
            return batch
        idx_hold = torch.nonzero(hold).flatten()
        idx_train = torch.nonzero(~hold).flatten()
        out = [batch.select(idx_train.to(batch.y.device))]
        if n_hold >= self.size:
            # earlier holdout rows of this batch are evicted by later ones: train on them
            if self.filled:
                out.append(self._ring_in_order())
            spill = idx_hold[: n_hold - self.size]
            out.append(batch.select(spill.to(batch.y.device)))
            keep = batch.select(idx_hold[n_hold - self.size:].to(batch.y.device))
            self._write(0, keep)
            self.head = 0
            self.filled = self.size
        else:
            new = batch.select(idx_hold.to(batch.y.device))
            n_evict = max(0, self.filled + n_hold - self.size)
            if n_evict:
                oldest = (self.head - self.filled) % self.size
                ev = (torch.arange(n_evict) + oldest) % self.size
                out.append(self.ring.select(ev.to(self.device)).to(batch.y.device))
            pos_w = (torch.arange(n_hold) + self.head) % self.size
            self._scatter(pos_w, new)
            self.head = (self.head + n_hold) % self.size
            self.filled = min(self.size, self.filled + n_hold)
        return HashedBatch.cat_batches(out)

    def _write(self, at: int, rows: HashedBatch):
        n = rows.B
        self.ring.num[at:at + n] = rows.num.to(self.device, self.ring.num.dtype)
        self.ring.cat[at:at + n] = rows.cat.to(self.device)
        self.ring.y[at:at + n] = rows.y.to(self.device)

    def _scatter(self, pos: torch.Tensor, rows: HashedBatch):
        p = pos.to(self.device)
        self.ring.num[p] = rows.num.to(self.device, self.ring.num.dtype)
        self.ring.cat[p] = rows.cat.to(self.device)
        self.ring.y[p] = rows.y.to(self.device)

    def _ring_in_order(self) -> HashedBatch:
        oldest = (self.head - self.filled) % self.size
        idx = (torch.arange(self.filled) + oldest) % self.size
        return self.ring.select(idx.to(self.device))

    def test_set(self) -> HashedBatch:
        return self._ring_in_order()

    def state_dict(self) -> dict:
        return {"num": self.ring.num.cpu(), "cat": self.ring.cat.cpu(), "y": self.ring.y.cpu(),
                "count": self.count, "head": self.head, "filled": self.filled}

    def load_state_dict(self, sd: dict) -> None:
        n = min(self.size, sd["num"].shape[0])
        self.ring.num[:n] = sd["num"][:n].to(self.device)
        self.ring.cat[:n] = sd["cat"][:n].to(self.device)
        self.ring.y[:n] = sd["y"][:n].to(self.device)
        self.count, self.head = int(sd["count"]), int(sd["head"]) % max(1, self.size)
        self.filled = min(self.size, int(sd["filled"]))
