"""HBM model store for multi-pipeline serving (BASELINE config 5).

Reference: M independent pipelines (networkIds) co-reside in every spoke; each point is
fed to every pipeline in a host loop (omldm/operators/spoke/FlinkSpoke.scala:97,101,105)
and each pipeline predicts separately.

Here the weight vectors of every hashed-linear pipeline live as rows of ONE fp32 arena
``W[capacity, dim]`` in HBM (288 GB holds ~68k pipelines of 2^20 features), so a
forecast batch is scored against all of them by ONE launch of the multi-model predict
kernel (csrc/kernels/linear_spoke.hip: linear_predict with M rows and a row stride) —
one read of the point's features, M gathers of weights — instead of M launches. The
arena grows by doubling; learners are re-pointed at their new rows (``attach``).
"""
from __future__ import annotations

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.ops import linear as L


class ModelStore:
    def __init__(self, dim: int, device, capacity: int = 4):
        self.dim = int(dim)
        self.device = torch.device(device)
        self.W = torch.zeros((max(1, capacity), self.dim), dtype=torch.float32,
                             device=self.device)
        self.owner: dict[int, object] = {}   # row -> learner
        self.free_rows = list(range(self.W.shape[0]))[::-1]

    @property
    def capacity(self) -> int:
        return int(self.W.shape[0])

    def bytes(self) -> int:
        return self.W.numel() * 4

    def _grow(self) -> None:
        old = self.W
        new = torch.zeros((2 * old.shape[0], self.dim), dtype=old.dtype, device=self.device)
        new[: old.shape[0]].copy_(old)
        self.W = new
        self.free_rows = list(range(old.shape[0], new.shape[0]))[::-1] + self.free_rows
        for row, learner in self.owner.items():
            learner.attach(self.W[row])

    def add(self, learner) -> int:
        """Move ``learner``'s weights into the arena (it must implement ``attach``)."""
        if not self.free_rows:
            self._grow()
        row = self.free_rows.pop()
        self.W[row].copy_(learner.w)
        learner.attach(self.W[row])
        self.owner[row] = learner
        return row

    def remove(self, row: int) -> None:
        learner = self.owner.pop(row, None)
        if learner is not None:
            learner.detach()
        self.W[row].zero_()
        self.free_rows.append(row)

    def scores(self, batch: HashedBatch, rows: list[int], bias: bool = True) -> torch.Tensor:
        """[B, len(rows)] decision values of the given pipelines in one kernel launch
        (over the contiguous row span covering them)."""
        lo, hi = min(rows), max(rows) + 1
        s = L.linear_predict(self.W[lo:hi], batch, bias=bias)
        if hi - lo == len(rows) and rows == list(range(lo, hi)):
            return s
        return s[:, torch.tensor([r - lo for r in rows], device=s.device)]
