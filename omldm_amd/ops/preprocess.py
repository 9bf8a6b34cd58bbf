"""Preprocessor ops (csrc/kernels/preprocess.hip on GPU; identical math in torch on CPU)."""
from __future__ import annotations

import torch

from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr

ROWS_PER_BLOCK = 1024
_PART: dict = {}


def _partial(device, n: int) -> torch.Tensor:
    t = _PART.get(device)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1 << 14), dtype=torch.float32, device=device)
        _PART[device] = t
    return t


def _colstats(x: torch.Tensor, count: float, mean, m2, lo, hi, mode: int) -> None:
    B, d = x.shape
    nblk = -(-B // ROWS_PER_BLOCK)
    part = _partial(x.device, nblk * d * 4)
    rc = native.hip().omldm_colstats_update(ptr(x), B, d, float(count), ptr(mean), ptr(m2),
                                            ptr(lo), ptr(hi), mode, ptr(part), ROWS_PER_BLOCK,
                                            native.stream_of(x))
    check(rc, "omldm_colstats_update")


def welford_update(x: torch.Tensor, count: float, mean: torch.Tensor, m2: torch.Tensor) -> float:
    """Chan merge of the batch moments into (count, mean, m2) [f64]. Returns new count."""
    B = x.shape[0]
    if B == 0:
        return count
    if x.is_cuda:
        _colstats(x, count, mean, m2, None, None, 1)
    else:
        xd = x.double()
        mb = xd.mean(0)
        m2b = ((xd - mb) ** 2).sum(0)
        tot = count + B
        delta = mb - mean
        mean.add_(delta * (B / tot))
        m2.add_(m2b + delta * delta * (count * B / tot))
    return count + B


def standardize(x: torch.Tensor, mean, m2, count: float) -> torch.Tensor:
    if x.is_cuda:
        y = torch.empty_like(x)
        check(native.hip().omldm_scale(ptr(x), ptr(y), x.shape[0], x.shape[1], 0, ptr(mean),
                                       ptr(m2), float(count), None, None, native.stream_of(x)),
              "omldm_scale")
        return y
    var = m2 / count if count > 0 else torch.zeros_like(m2)
    sd = torch.where(var > 0, var.sqrt(), torch.ones_like(var)).float()
    return (x - mean.float()) / sd


def minmax_update(x: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor) -> None:
    if x.shape[0] == 0:
        return
    if x.is_cuda:
        _colstats(x, 0.0, None, None, lo, hi, 2)
    else:
        torch.minimum(lo, x.min(0).values, out=lo)
        torch.maximum(hi, x.max(0).values, out=hi)


def minmax_scale(x: torch.Tensor, lo, hi) -> torch.Tensor:
    if x.is_cuda:
        y = torch.empty_like(x)
        check(native.hip().omldm_scale(ptr(x), ptr(y), x.shape[0], x.shape[1], 1, None, None, 0.0,
                                       ptr(lo), ptr(hi), native.stream_of(x)), "omldm_scale")
        return y
    rg = hi - lo
    return torch.where(rg > 0, (x - lo) / torch.where(rg > 0, rg, torch.ones_like(rg)),
                       torch.zeros_like(x))


def poly_expand(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    B, d = x.shape
    ncomb, deg = idx.shape
    if x.is_cuda:
        out = torch.empty((B, d + ncomb), dtype=torch.float32, device=x.device)
        check(native.hip().omldm_poly(ptr(x), B, d, ptr(idx), ncomb, deg, ptr(out),
                                      native.stream_of(x)), "omldm_poly")
        return out
    cols = [x]
    if ncomb:
        il = idx.long()
        prod = torch.ones((B, ncomb), dtype=x.dtype)
        for k in range(deg):
            sel = il[:, k]
            f = torch.where(sel >= 0, x[:, sel.clamp(min=0)], torch.ones_like(prod))
            prod = prod * f
        cols.append(prod)
    return torch.cat(cols, 1)
