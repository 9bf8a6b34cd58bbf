"""Fused hub-merge ops of the protocols (csrc/kernels/merge.hip on GPU; the same math in
PyTorch on CPU). Each is one pass over the flat parameter vector."""
from __future__ import annotations

import torch

from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr


def _gpu(t: torch.Tensor) -> bool:
    """The fused HIP kernels take fp32 vectors; other dtypes (ORR's fp64 sufficient
    statistics) use the same math in PyTorch (small vectors, off the hot path)."""
    return t.is_cuda and t.dtype == torch.float32


def drift_norms(x: torch.Tensor, E: torch.Tensor, scale: float,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """[Σ((x − E)·scale)², ΣE²] as a 2-float device tensor (no host sync)."""
    if out is None:
        out = torch.empty(2, dtype=torch.float32, device=x.device)
    if _gpu(x):
        check(native.hip().omldm_drift_norms(ptr(x), ptr(E), x.numel(), float(scale), ptr(out),
                                             native.stream_of(x)), "omldm_drift_norms")
    else:
        out[0] = ((x - E) * scale).pow(2).sum().to(out.dtype)
        out[1] = E.pow(2).sum().to(out.dtype)
    return out


def fold_reload(E: torch.Tensor, d: torch.Tensor, alpha: float, x: torch.Tensor) -> None:
    """E += α·d; x = E."""
    if _gpu(E):
        check(native.hip().omldm_fold_reload(ptr(E), ptr(d), float(alpha), ptr(x), E.numel(),
                                             native.stream_of(E)), "omldm_fold_reload")
    else:
        E.add_(d, alpha=alpha)
        x.copy_(E)


def elastic_pre(x, c, diff, s) -> None:
    if _gpu(x):
        check(native.hip().omldm_elastic_pre(ptr(x), ptr(c), ptr(diff), ptr(s), x.numel(),
                                             native.stream_of(x)), "omldm_elastic_pre")
    else:
        torch.sub(x, c, out=diff)
        s.copy_(diff)


def elastic_post(x, c, diff, s, alpha: float) -> None:
    if _gpu(x):
        check(native.hip().omldm_elastic_post(ptr(x), ptr(c), ptr(diff), ptr(s), float(alpha),
                                              x.numel(), native.stream_of(x)),
              "omldm_elastic_post")
    else:
        x.sub_(diff, alpha=alpha)
        c.add_(s, alpha=alpha)


def async_push(x, E, shipped, sent, buf) -> None:
    """sent = x − E − shipped; buf = sent; shipped += sent."""
    if _gpu(x):
        check(native.hip().omldm_async_push(ptr(x), ptr(E), ptr(shipped), ptr(sent), ptr(buf),
                                            x.numel(), native.stream_of(x)), "omldm_async_push")
    else:
        torch.sub(x - E, shipped, out=sent)
        buf.copy_(sent)
        shipped.add_(sent)


def async_pull(x, E, shipped, sent, merged, scale: float) -> None:
    """x += merged·scale − sent; shipped −= sent; E += merged·scale."""
    if _gpu(x):
        check(native.hip().omldm_async_pull(ptr(x), ptr(E), ptr(shipped), ptr(sent), ptr(merged),
                                            float(scale), x.numel(), native.stream_of(x)),
              "omldm_async_pull")
    else:
        m = merged * scale
        x.add_(m - sent)
        shipped.sub_(sent)
        E.add_(m)
