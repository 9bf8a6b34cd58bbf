"""Ops of the dense-feature and multi-class learners.

GPU: csrc/kernels/dense_learners.hip (MFMA Gram / K-means assignment) and
csrc/kernels/multiclass_spoke.hip; CPU: identical math in PyTorch / the C++ mirror.
"""
from __future__ import annotations

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr


def gram_update(x: torch.Tensor, y: torch.Tensor, G: torch.Tensor) -> None:
    """G[:d+2, :d+2] += Σ_rows z zᵀ with z = [x, 1, y] over rows whose y is finite."""
    B, d = x.shape
    if B == 0:
        return
    x = x.float().contiguous()
    y = y.float().contiguous()
    if x.is_cuda:
        check(native.hip().omldm_gram_update(ptr(x), ptr(y), B, d, ptr(G), G.shape[1],
                                             native.stream_of(x)), "omldm_gram_update")
        return
    ok = ~torch.isnan(y)
    z = torch.cat([x[ok], torch.ones((int(ok.sum()), 1)), y[ok].unsqueeze(1)], 1).double()
    G[: d + 2, : d + 2] += (z.T @ z).float()


def kmeans_assign(x: torch.Tensor, y: torch.Tensor | None, cent: torch.Tensor,
                  sums: torch.Tensor | None, counts: torch.Tensor | None,
                  inertia: torch.Tensor | None = None, want_assign: bool = False):
    """Nearest-centroid assignment; optionally accumulates per-cluster sums/counts of
    the training rows (finite y, or all rows when y is None)."""
    B, d = x.shape
    k = cent.shape[0]
    assign = torch.empty(B, dtype=torch.int32, device=x.device) if want_assign else None
    if B == 0:
        return assign
    x = x.float().contiguous()
    if x.is_cuda:
        check(native.hip().omldm_kmeans_assign(ptr(x), ptr(y), B, d, k, ptr(cent), ptr(sums),
                                               ptr(counts), ptr(assign), ptr(inertia),
                                               native.stream_of(x)), "omldm_kmeans_assign")
        return assign
    dist = torch.cdist(x, cent.float()) ** 2
    a = dist.argmin(1)
    if assign is not None:
        assign.copy_(a)
    if sums is not None:
        train = torch.ones(B, dtype=torch.bool) if y is None else ~torch.isnan(y)
        sums.index_add_(0, a[train], x[train])
        counts.index_add_(0, a[train], torch.ones(int(train.sum())))
        if inertia is not None:
            inertia += dist[train, a[train]].sum()
    return assign


def multiclass_round(W: torch.Tensor, batch: HashedBatch, R: int, S: int, nclass: int,
                     variant: int, C: float, bias: bool, dacc: torch.Tensor,
                     stats: torch.Tensor, log2cap: int = 11) -> None:
    """S virtual spokes of MultiClassPA; dacc[K, dim] += Σ_s Δ_s; stats += (loss, n,
    mistakes, active spokes, -, overflow)."""
    K, dim = W.shape
    assert batch.cat_span == 0, "MultiClassPA consumes the int32 categorical format"
    if batch.B == 0:
        return
    num = batch.num.float().contiguous()
    if W.is_cuda:
        check(native.hip().omldm_multiclass_round(
            ptr(W), ptr(num), num.shape[1], ptr(batch.cat), batch.cat.shape[1], ptr(batch.y),
            batch.B, R, S, dim, nclass, variant, C, int(bias), ptr(dacc), ptr(stats), log2cap,
            native.stream_of(W)), "omldm_multiclass_round")
    else:
        native.host().omldm_cpu_multiclass_round(
            ptr(W), ptr(num), num.shape[1], ptr(batch.cat), batch.cat.shape[1], ptr(batch.y),
            batch.B, R, S, dim, nclass, variant, C, int(bias), ptr(dacc), ptr(stats))


def multiclass_apply(W: torch.Tensor, dacc: torch.Tensor, nact: torch.Tensor) -> None:
    if W.is_cuda:
        check(native.hip().omldm_multiclass_apply(ptr(W), ptr(dacc), W.numel(), ptr(nact),
                                                  native.stream_of(W)), "omldm_multiclass_apply")
    else:
        n = float(nact.item())
        if n > 0:
            W.add_(dacc / n)
        dacc.zero_()
