"""Fused hub-merge ops of the protocols (csrc/kernels/merge.hip on GPU; the same math in
PyTorch on CPU). Each is one pass over the flat parameter vector."""
from __future__ import annotations

import math

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


# ------------------------------------------------- GM / FGM monitoring (one device lane)
# FGM state (fp64[8]): c_prev, csum, theta, phi0, phi, decision latch, subrounds, spare.
FGM_BIG = 1e12


def _fgm_counter(phi: float, phi0: float, theta: float) -> float:
    num = phi - phi0
    if theta <= 0.0:
        return FGM_BIG if num > 0.0 else 0.0
    return min(FGM_BIG, max(0.0, math.floor(num / theta)))


def gm_local(nrm: torch.Tensor, thr: float, msg: torch.Tensor) -> None:
    """msg[0] = 1 if ‖X_i‖² > θ·max(‖E‖², 1) else 0."""
    if nrm.is_cuda:
        check(native.hip().omldm_gm_local(ptr(nrm), float(thr), ptr(msg), native.stream_of(nrm)),
              "omldm_gm_local")
    else:
        x2, e2 = (float(v) for v in nrm.tolist())
        msg[0] = 1.0 if x2 > float(torch.tensor(thr, dtype=torch.float32)) * max(e2, 1.0) else 0.0


def fgm_local(nrm: torch.Tensor, st: torch.Tensor, eps: float, msg: torch.Tensor) -> None:
    """φ = ‖X_i‖² − ε‖E‖²; msg = (counter increment, φ); state counter/φ updated."""
    if nrm.is_cuda:
        check(native.hip().omldm_fgm_local(ptr(nrm), ptr(st), float(eps), ptr(msg),
                                           native.stream_of(nrm)), "omldm_fgm_local")
        return
    x2, e2 = (float(v) for v in nrm.tolist())
    s = st.tolist()
    phi = x2 - eps * e2
    c = _fgm_counter(phi, s[3], s[2])
    msg[0], msg[1] = c - s[0], phi
    st[0], st[4] = c, phi


def fgm_hub(st: torch.Tensor, msg: torch.Tensor, eps_psi: float, G: int,
            flag: torch.Tensor) -> None:
    """Replicated hub step on the reduced (Σ increments, ψ); flag[0] = full sync due."""
    if st.is_cuda:
        check(native.hip().omldm_fgm_hub(ptr(st), ptr(msg), float(eps_psi), int(G), ptr(flag),
                                         native.stream_of(st)), "omldm_fgm_hub")
        return
    s = st.tolist()
    inc, psi = (float(v) for v in msg.tolist())
    if s[5] == 0.0:
        s[1] += inc
        if s[1] > G:
            s[6] += 1.0
            if psi >= eps_psi * G * s[3]:
                s[5] = 1.0
            else:
                s[2] = -psi / (2.0 * G)
                s[1] = 0.0
                s[0] = _fgm_counter(s[4], s[3], s[2])
    st.copy_(torch.tensor(s, dtype=st.dtype))
    flag[0] = s[5]


def fgm_begin(nrm: torch.Tensor, st: torch.Tensor, eps: float) -> None:
    """Round start after a full sync: φ(0) = −ε‖E‖², θ = −φ(0)/2, counters cleared."""
    if nrm.is_cuda:
        check(native.hip().omldm_fgm_begin(ptr(nrm), ptr(st), float(eps), native.stream_of(nrm)),
              "omldm_fgm_begin")
        return
    phi0 = -eps * float(nrm[1])
    st[0] = st[1] = st[4] = st[5] = 0.0
    st[2] = -phi0 / 2.0 if phi0 < 0.0 else 0.0
    st[3] = phi0


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
