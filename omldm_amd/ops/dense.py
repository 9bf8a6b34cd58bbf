"""Ops of the dense-feature and multi-class learners.

GPU: csrc/kernels/dense_learners.hip (MFMA Gram / K-means assignment) and
csrc/kernels/multiclass_spoke.hip; CPU: identical math in PyTorch / the C++ mirror.
"""
from __future__ import annotations

import os

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr


def _gram_part(device) -> torch.Tensor:
    """Scratch of the Gram kernel's per-block tile sums: ≤ 256 blocks × 10 tiles × 1024
    (csrc/kernels/dense_learners.hip gram_colsum_kernel adds them into G)."""
    from omldm_amd.ops.linear import _workspace

    return _workspace(device, 256 * 10 * 1024, key="gram_part")


def gram_update(x: torch.Tensor, y: torch.Tensor, G: torch.Tensor,
                cnt: torch.Tensor | None = None, pairs: torch.Tensor | None = None) -> None:
    """G[:d+2, :d+2] += Σ_rows z zᵀ with z = [x, 1, y] over rows whose y is finite;
    ``cnt`` (one fp64 element: a running total) += the number of those rows, read off
    the Gram's (d, d) entry inside the same kernel. ``pairs`` (int32 [np, 2]): x holds the
    raw features of a PolynomialFeatures(2) map and z = [x, x_a·x_b per pair, 1, y] — the
    GPU kernel forms the products in its operand fetch (csrc/kernels/dense_learners.hip
    gram_map_kernel), so the expansion never reaches HBM."""
    B, d0 = x.shape
    if B == 0:
        return
    x = x.float().contiguous()
    y = y.float().contiguous()
    assert cnt is None or (cnt.dtype == torch.float64 and cnt.numel() == 1)
    if pairs is not None:
        pairs = pairs.to(device=x.device, dtype=torch.int32).contiguous()
        assert pairs.dim() == 2 and pairs.shape[1] == 2
        if x.is_cuda and d0 + pairs.shape[0] + 2 <= 128:
            check(native.hip().omldm_gram_update_poly2(
                ptr(x), ptr(y), B, d0, ptr(pairs), pairs.shape[0], ptr(G), G.shape[1], ptr(cnt),
                ptr(_gram_part(x.device)), native.stream_of(x)), "omldm_gram_update_poly2")
            return
        from omldm_amd.ops.preprocess import poly_expand

        x = poly_expand(x, pairs)
    B, d = x.shape
    if x.is_cuda:
        check(native.hip().omldm_gram_update(ptr(x), ptr(y), B, d, ptr(G), G.shape[1], ptr(cnt),
                                             ptr(_gram_part(x.device)), native.stream_of(x)),
              "omldm_gram_update")
        return
    ok = ~torch.isnan(y)
    if cnt is not None:
        cnt += ok.sum()
    z = torch.cat([x[ok], torch.ones((int(ok.sum()), 1)), y[ok].unsqueeze(1)], 1).double()
    G[: d + 2, : d + 2] += (z.T @ z).float()


KMEANS_MAX_BLOCKS = 512  # csrc/kernels/dense_learners.hip kKmeansMaxBlocks


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
        from omldm_amd.ops.linear import _workspace

        # per-block partials, summed per column by a second launch (csrc: kmeans_flush)
        part = _workspace(x.device, KMEANS_MAX_BLOCKS * (k * d + k + 1), key="km_part") \
            if sums is not None else None
        check(native.hip().omldm_kmeans_assign(ptr(x), ptr(y), B, d, k, ptr(cent), ptr(sums),
                                               ptr(counts), ptr(assign), ptr(inertia), ptr(part),
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


def class_pad(nclass: int) -> int:
    """Row stride of the key-major prototype shadow: a power of two ≥ nclass up to 16
    (the K of the v3 multiclass scan), a multiple of 4 above."""
    if nclass <= 16:
        return 2 if nclass <= 2 else 4 if nclass <= 4 else 8 if nclass <= 8 else 16
    return (nclass + 3) // 4 * 4


def proto_shadow(W: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """Key-major copy Wt[dim][kp] of the prototypes W[K][dim] (zero-padded classes) —
    what the GPU round gathers: one cache line per key instead of K."""
    K, dim = W.shape
    Wt = torch.zeros((dim, class_pad(K)), dtype=dtype, device=W.device)
    Wt[:, :K].copy_(W.t())
    return Wt


def multiclass_round(W: torch.Tensor, batch: HashedBatch, R: int, S: int, nclass: int,
                     variant: int, C: float, bias: bool, dacc: torch.Tensor,
                     stats: torch.Tensor, log2cap: int = 0,
                     Wt: torch.Tensor | None = None) -> None:
    """S virtual spokes of MultiClassPA; dacc[K, dim] += Σ_s Δ_s; stats += (loss, n,
    mistakes, active spokes, -, overflow).

    GPU: the compact or wide categorical wire, bf16 or fp32 numerical features and fp32
    or int8 labels are read as they are; ``log2cap`` 0 sizes the LDS delta table (one
    slot of K floats per hashed key) from the spoke's rows. CPU: the C++ mirror on the
    wide int32 format."""
    from omldm_amd.ops.linear import _workspace

    K, dim = W.shape
    if batch.B == 0:
        return
    if W.is_cuda:
        num, cat, y = batch.num, batch.cat, batch.y
        assert num.dtype in (torch.float32, torch.bfloat16) and y.dtype in (torch.float32, torch.int8)
        assert all(t.is_contiguous() for t in (num, cat, y))
        dn, dc = int(num.shape[1]), int(cat.shape[1])
        if log2cap <= 0:  # ≤ 1/2 load for the spoke's hashed keys (K floats per slot)
            from omldm_amd.ops.linear import min_log2cap

            want = max(1, 2 * R * max(1, dc) - 1).bit_length()
            kp = 2 if nclass <= 2 else 4 if nclass <= 4 else 8 if nclass <= 8 else 16
            log2cap = max(min_log2cap(dim), min(12, want))
            while log2cap > min_log2cap(dim) and ((1 << log2cap) + 64) * (4 + 4 * kp) > 64 << 10:
                log2cap -= 1  # ≤ 64 KiB of LDS per spoke wave
        wsw = 8 + nclass * (dn + 1)
        ws = _workspace(W.device, S * wsw, key="mc_ws")
        tables = _workspace(W.device, nclass * S * (1 << log2cap) * 2, key="mc_tables")
        if Wt is None:
            Wt = proto_shadow(W)
        assert Wt.shape == (dim, class_pad(nclass)) and Wt.is_contiguous()
        from omldm_amd.ops.linear import spill_log2cap, spill_workspace

        lg = spill_log2cap(R, dn + dc + 1, S, class_pad(nclass))
        spill = spill_workspace(W.device, S, lg, class_pad(nclass))
        check(native.hip().omldm_multiclass_round(
            ptr(Wt), int(Wt.dtype == torch.bfloat16), ptr(num), int(num.dtype == torch.bfloat16),
            dn, ptr(cat), dc, batch.cat_span,
            ptr(y), int(y.dtype == torch.int8), batch.B, R, S, dim, nclass, variant, C, int(bias),
            ptr(dacc), ptr(stats), log2cap, ptr(ws), ptr(tables), ptr(spill), lg,
            native.stream_of(W)),
            "omldm_multiclass_round")
    else:
        batch = batch.to_wide()
        num = batch.num.float().contiguous()
        native.host().omldm_cpu_multiclass_round(
            ptr(W), ptr(num), num.shape[1], ptr(batch.cat), batch.cat.shape[1],
            ptr(batch.y.float().contiguous()), batch.B, R, S, dim, nclass, variant, C, int(bias),
            ptr(dacc), ptr(stats))


def kmeans_seq(x: torch.Tensor, y: torch.Tensor | None, cent: torch.Tensor, n: torch.Tensor,
               cum: torch.Tensor | None) -> None:
    """Exact sequential (MacQueen) k-means over the rows of x, in order (GPU:
    csrc/kernels/kmeans_seq.hip, one wave holding the model in registers; CPU:
    csrc/host/dense_cpu.cpp). Rows with a NaN ``y`` are skipped."""
    k, d = cent.shape
    x = x.float().contiguous()
    assert x.shape[1] >= d and cent.is_contiguous() and n.is_contiguous()
    assert cum is None or cum.dtype == torch.float64
    yv = None if y is None else y.float().contiguous()
    if x.is_cuda:
        check(native.hip().omldm_kmeans_seq(ptr(x), x.shape[1], ptr(yv), x.shape[0], d, k,
                                            ptr(cent), ptr(n), ptr(cum), native.stream_of(x)),
              "omldm_kmeans_seq")
    else:
        check(native.host().omldm_cpu_kmeans_seq(ptr(x), x.shape[1], ptr(yv), x.shape[0], d, k,
                                                 ptr(cent), ptr(n), ptr(cum)),
              "omldm_cpu_kmeans_seq")


def kmeans_seq_form(form: int = -1) -> int:
    """GPU form of the exact sequential k-means: 1 = the fast one-wave kernel (every lane on
    the per-point chain: G lanes per centroid or CPL centroids per lane, packed fp32, LDS
    broadcast points; k ≤ 512, d ≤ 64), 0 = the earlier one-wave / workgroup kernels.
    ``form`` < 0 only reads the current setting (default 1; env OMLDM_KMEANS_FAST=0)."""
    return int(native.hip().omldm_kmeans_seq_form(int(form)))


def kmeans_seq_fits(d: int, k: int) -> bool:
    """The exact sequential kernels take every (d, k) with d ≤ 8192
    (csrc/kernels/kmeans_seq.hip): one wave for k ≤ 64 (G lanes per centroid), four waves
    for k ≤ 1024 (d ≤ 64), the LDS workgroup form up to k·(d + 1) floats in 160 KiB, and
    the HBM-resident form past that."""
    return 1 <= d <= 8192 and k >= 1


def kmeans_apply(cent: torch.Tensor, n: torch.Tensor, sums: torch.Tensor, counts: torch.Tensor,
                 inertia: torch.Tensor, cum: torch.Tensor | None) -> None:
    """GPU: one launch — c ← (n·c + Σx)/(n + cnt) where n + cnt > 0, n += cnt, Σx = cnt = 0,
    cum[0] += inertia, cum[1] += Σcnt, inertia = 0."""
    k, d = cent.shape
    assert cum is None or cum.dtype == torch.float64
    check(native.hip().omldm_kmeans_apply(ptr(cent), ptr(n), k, d, ptr(sums), ptr(counts),
                                          ptr(inertia), ptr(cum), native.stream_of(cent)),
          "omldm_kmeans_apply")


MLP_MB = 32          # mini-batch rows of the fused MLP kernel
MLP_MAX_LAYERS = 4


def _widths_arr(widths):
    import ctypes

    return (ctypes.c_int * len(widths))(*[int(v) for v in widths])


def mlp_lds_bytes(widths: list[int]) -> int:
    return int(native.hip().omldm_mlp_lds_bytes(len(widths) - 1, _widths_arr(widths)))


def _mlp_unflatten(w: torch.Tensor, widths):
    out, o = [], 0
    for a, b in zip(widths[:-1], widths[1:]):
        out.append((w[o:o + a * b].view(b, a), w[o + a * b:o + a * b + b]))
        o += a * b + b
    return out


MLP_ACTS = {"relu": 0, "tanh": 1, "sigmoid": 2, "identity": 3}
MLP_BF16 = 0x100  # flag OR-ed into `act`: bf16 GEMM operands (v_mfma_f32_32x32x16_bf16)
_ACT_FN_BASE = {0: torch.relu, 1: torch.tanh, 2: torch.sigmoid, 3: lambda t: t}


class _ActFns(dict):
    """Activation lookup that ignores the precision flag (the CPU mirror is fp32)."""

    def __getitem__(self, k):
        return super().__getitem__(k & 0xFF)


_ACT_FN = _ActFns(_ACT_FN_BASE)


def mlp_forward_reference(w: torch.Tensor, x: torch.Tensor, widths, act: int = 0
                          ) -> torch.Tensor:
    h = x
    layers = _mlp_unflatten(w, widths)
    for i, (W, b) in enumerate(layers):
        h = torch.nn.functional.linear(h, W, b)
        if i + 1 < len(layers):
            h = _ACT_FN[act](h)
    return h


def _mlp_grad_out(o: torch.Tensor, y: torch.Tensor, task: int, K: int):
    """dLoss/dlogits (sum over rows) + (loss, correct) — same rules as the kernel."""
    if task == 0:
        e = o[:, 0] - y
        g = torch.zeros_like(o)
        g[:, 0] = 2 * e
        return g, (e * e).sum(), torch.zeros((), device=o.device)
    if task == 1:
        t = (y > 0).float()
        z = o[:, 0]
        g = torch.zeros_like(o)
        g[:, 0] = torch.sigmoid(z) - t
        loss = (torch.clamp(z, min=0) - z * t + torch.log1p(torch.exp(-z.abs()))).sum()
        return g, loss, ((z >= 0).float() == t).float().sum()
    yi = y.long().clamp(0, K - 1)
    p = torch.softmax(o, 1)
    g = p - torch.nn.functional.one_hot(yi, K).float()
    loss = -torch.log_softmax(o, 1).gather(1, yi.unsqueeze(1)).sum()
    return g, loss, (o.argmax(1) == yi).float().sum()


def mlp_round_reference(w, x, y, R, S, widths, task, lr, dacc, stats, act: int = 0,
                        nact=None) -> None:
    """CPU mirror of mlp_round_kernel: spoke s runs 32-row mini-batch SGD over rows
    [sR, sR+R) from the round-start model; dacc += Σ Δ_s; stats += (loss, n, correct,
    active spokes)."""
    B = x.shape[0]
    K = widths[-1]
    for s in range(S):
        r0, r1 = s * R, min(B, s * R + R)
        if r0 >= B:
            break
        ws = w.detach().clone()
        loss_s, n_s, c_s = 0.0, 0, 0.0
        for m0 in range(r0, r1, MLP_MB):
            xb, yb = x[m0:min(r1, m0 + MLP_MB)], y[m0:min(r1, m0 + MLP_MB)]
            ok = ~torch.isnan(yb)
            cnt = int(ok.sum())
            if cnt == 0:
                continue
            wv = ws.clone().requires_grad_(True)
            o = mlp_forward_reference(wv, xb[ok], widths, act)
            g, ls, cs = _mlp_grad_out(o.detach(), yb[ok], task, K)
            gw, = torch.autograd.grad(o, wv, grad_outputs=g)
            ws -= (lr / cnt) * gw
            loss_s += float(ls)
            c_s += float(cs)
            n_s += cnt
        dacc += ws - w
        if n_s:
            stats[0] += loss_s
            stats[1] += n_s
            stats[2] += c_s
            stats[3] += 1
            if nact is not None:
                nact += 1


def mlp_round(w: torch.Tensor, x: torch.Tensor, y: torch.Tensor, R: int, S: int,
              widths: list[int], task: int, lr: float, dacc: torch.Tensor,
              stats: torch.Tensor, act: int = 0, nact: torch.Tensor | None = None) -> None:
    """``nact`` (optional, one fp32 element, zero on entry): += the number of spokes with at
    least one labelled row — the divisor of the following apply."""
    B = x.shape[0]
    if B == 0:
        return
    x = x.float().contiguous()
    y = y.float().contiguous()
    if len(widths) - 1 > MLP_MAX_LAYERS:
        raise ValueError(f"NN: at most {MLP_MAX_LAYERS} layers on the fused kernel")
    if x.is_cuda:
        from omldm_amd.ops.linear import _workspace

        # spoke deltas as plain rows + slab column sums (no per-spoke same-address atomics)
        ws = _workspace(x.device, S * w.numel(), key="mlp_ws")
        check(native.hip().omldm_mlp_round(ptr(w), ptr(x), ptr(y), B, R, S, len(widths) - 1,
                                           _widths_arr(widths), task, act, lr, ptr(dacc),
                                           ptr(stats), ptr(nact), ptr(ws), native.stream_of(x)),
              "omldm_mlp_round")
    else:
        mlp_round_reference(w, x, y, R, S, widths, task, lr, dacc, stats, act, nact)


def mlp_forward(w: torch.Tensor, x: torch.Tensor, widths: list[int], act: int = 0
                ) -> torch.Tensor:
    B = x.shape[0]
    out = torch.empty((B, widths[-1]), dtype=torch.float32, device=x.device)
    if B == 0:
        return out
    x = x.float().contiguous()
    if x.is_cuda:
        check(native.hip().omldm_mlp_forward(ptr(w), ptr(x), B, len(widths) - 1,
                                             _widths_arr(widths), act, ptr(out),
                                             native.stream_of(x)), "omldm_mlp_forward")
        return out
    return mlp_forward_reference(w, x, widths, act)


# classes the v3 multiclass scan takes (K templates 2 / 4 / 8 / 16; OMLDM_MC_SCAN_KMAX caps it)
_MC_SCAN_KMAX = int(os.environ.get("OMLDM_MC_SCAN_KMAX", "16"))


def multiclass_scan3_fits(batch, R: int, nclass: int, bias: bool, Wt) -> bool:
    """The MultiClassPA round on the v3 table scan (csrc/kernels/linear_scan3.hip,
    s3mc_scan_kernel) takes this batch: the engine's field-aware wire on a GPU, K ≤ 16 classes,
    fp32 key-major prototypes, a shape the v3 prep takes."""
    from omldm_amd.ops import linear as L

    return (Wt is not None and Wt.is_cuda and Wt.dtype == torch.float32 and nclass <= _MC_SCAN_KMAX
            and getattr(batch, "cat_span", 0) > 0 and batch.B > 0 and 0 < batch.dc
            and L.SEQ_KERNEL == "scan3" and batch.y.is_cuda
            and batch.dn + batch.dc * batch.cat_span <= int(Wt.shape[0]) - 1
            and L.scan3_fits(batch.dn, batch.dc, R, bias))


def multiclass_scan3_round(Wt: torch.Tensor, batch, R: int, S: int, nclass: int, variant: int,
                           C: float, bias: bool, dacc: torch.Tensor, stats: torch.Tensor) -> None:
    """S exact sequential MultiClassPA spokes of R rows on the v3 table scan: the binary
    scan's prep (slots, occurrence flags, chunk Grams; a_t = 1/(2‖x‖² + kadd)), one 12-wave
    workgroup per spoke carrying the K scores of each row through the chunk recurrence, then
    one scatter of the rows' ±τ into dacc [K, dim]. stats[0..3] += (loss, rows, mistakes,
    active spokes), like ``multiclass_round``."""
    from omldm_amd.api.batch import RawBatch
    from omldm_amd.ops import linear as L
    from omldm_amd.ops.linear import _workspace

    dim, kp = int(Wt.shape[0]), int(Wt.shape[1])
    K = class_pad(nclass)  # the scan's class template: 2, 4, 8 or 16
    kt = int(os.environ.get("OMLDM_MC_KT", "0") or 0)  # diagnostics: a wider template
    if kt in (4, 8, 16) and kt > K and kt <= int(Wt.shape[1]):
        K = kt
    num = batch.num.float().contiguous()
    y = batch.y.float().contiguous() if batch.y.dtype != torch.int8 else batch.y.contiguous()
    rb = RawBatch(num, batch.cat.contiguous(), y, span=batch.cat_span, cbase=batch.dn)
    rule = L.LinearRule(rule=L.RULE_MULTI, variant=variant, C=C, bias=bias)
    key = L._s3_key(rb, R, S, dim, bias, rule)
    sp = getattr(batch, "prep", None)
    if not (isinstance(sp, L.Scan3Prep) and sp.key == key):
        sp = L.linear_scan3_prepare(rb, R, S, dim, bias, rule, hashed=True,
                                    slot=L._s3_slot_for(key, Wt.device))
        batch.prep = sp
    elif sp.event is not None:
        torch.cuda.current_stream(Wt.device).wait_event(sp.event)
    L.SCAN3_ROUNDS += 1
    h = native.hip()
    dev = Wt.device
    ws = _workspace(dev, S * 8, key="mc3_ws")
    wsd = _workspace(dev, S * K * 32, key="mc3_wsd")
    ag = _workspace(dev, S * int(h.omldm_scan3mc_spill_floats(R, batch.dc, K)), key="mc3_ag")
    tau = _workspace(dev, batch.B, key="mc3_tau")
    rr = _workspace(dev, batch.B, key="mc3_rr")  # int32 view of an fp32 scratch
    check(h.omldm_scan3mc_run(ptr(Wt), kp, K, nclass, batch.dn, batch.dc, ptr(y),
                              int(y.dtype == torch.int8), batch.B, R, S, ptr(dacc), dim, ptr(stats),
                              int(variant), float(C), int(bias), sp.ptrs, ptr(ws), ptr(wsd),
                              ptr(ag), ptr(tau), ptr(rr), native.stream_of(Wt)),
          "omldm_scan3mc_run")
    L._s3_mark_read(sp)


def multiclass_apply(W: torch.Tensor, dacc: torch.Tensor, nact: torch.Tensor,
                     Wt: torch.Tensor | None = None, st: torch.Tensor | None = None,
                     cum: torch.Tensor | None = None, fold: int = 0,
                     nact_next: torch.Tensor | None = None) -> None:
    """W += dacc / n_active; dacc = 0; refresh the key-major shadow ``Wt`` if given.
    ``fold`` > 0 also folds the round statistics ``st`` into the running totals ``cum``
    and clears st[0..3] in the same launch (1: cum[:3] += st[:3]; 2: cum[:2] += st[:2];
    3: as 2 plus cum[2] += st[1] − st[2]). ``nact`` must then be its own buffer.
    ``nact_next`` (optional, another buffer) is zeroed in the same launch: the divisor the
    next round counts into."""
    assert nact_next is None or nact_next.data_ptr() != nact.data_ptr()
    if fold:
        assert st is not None and cum is not None and nact.data_ptr() != st.data_ptr()
        assert cum.dtype == torch.float64  # running totals (kernel adds in fp64)
    if W.is_cuda:
        K, dim = (1, W.numel()) if W.dim() == 1 else W.shape  # 1-D: a flat parameter vector
        assert Wt is None or W.dim() == 2
        check(native.hip().omldm_multiclass_apply(
            ptr(W), ptr(dacc), dim, K, ptr(Wt), int(Wt is not None and Wt.dtype == torch.bfloat16),
            int(Wt.shape[1]) if Wt is not None else class_pad(K), ptr(nact), ptr(st), ptr(cum),
            int(fold), ptr(nact_next),
            native.stream_of(W)),
            "omldm_multiclass_apply")
    else:
        n = float(nact.item())
        if n > 0:
            W.add_(dacc / n)
        dacc.zero_()
        if fold:
            cum[:2] += st[:2]
            if fold == 1:
                cum[2] += st[2]
            elif fold == 3:
                cum[2] += st[1] - st[2]
            st[:4] = 0.0
        if nact_next is not None:
            nact_next.zero_()


def _tree_ptrs(tree: list[torch.Tensor]):
    import ctypes

    return (ctypes.c_void_p * len(tree))(*[t.data_ptr() for t in tree])


_HT_WS: dict = {}


def ht_update(x: torch.Tensor, y: torch.Tensor, C: int, depth: int, tree: list[torch.Tensor],
              nfit: torch.Tensor, N: int = 0, sort: bool = True) -> None:
    """Route rows to leaves and add their Gaussian statistics (device only).
    sort (default, needs the node capacity N): rows counting-sorted by (leaf, class) and
    one reducer block per pair — no atomics on the statistics; otherwise the
    wave-aggregated atomic kernel."""
    B, d = x.shape
    x = x.float().contiguous()
    y = y.float().contiguous()
    assert nfit is None or nfit.dtype == torch.float64
    ws = None
    if sort and N > 0 and N * C * 4 <= 64 << 10:
        n = int(native.hip().omldm_ht_update_ws_ints(B, N, C))
        ws = _HT_WS.get(x.device)
        if ws is None or ws.numel() < n:
            ws = torch.empty(max(n, 1 << 16), dtype=torch.int32, device=x.device)
            _HT_WS[x.device] = ws
    check(native.hip().omldm_ht_update(ptr(x), ptr(y), B, d, C, depth, int(N), _tree_ptrs(tree),
                                       ptr(nfit), ptr(ws), native.stream_of(x)),
          "omldm_ht_update")


def ht_split(N: int, d: int, C: int, nb: int, grace: float, delta: float, tau: float,
             tree: list[torch.Tensor]) -> None:
    check(native.hip().omldm_ht_split(N, d, C, nb, grace, delta, tau, _tree_ptrs(tree),
                                      native.stream_of(tree[0])), "omldm_ht_split")


def ht_exact(x: torch.Tensor, y: torch.Tensor, C: int, depth: int, N: int, nb: int,
             grace: float, delta: float, tau: float, tree: list[torch.Tensor],
             nfit: torch.Tensor | None, dbg: torch.Tensor | None = None) -> bool:
    """The per-point VFDT over a whole tick in one persistent launch
    (csrc/kernels/hoeffding.hip: ht_exact_kernel): each leaf is checked at the very row
    where it reaches the grace period, no host round trip. False when the tree's LDS
    layout does not fit (the caller keeps the host-driven segment loop). ``dbg``: an int64
    [8] device tensor that accumulates chunks, segments, splits and the cycles of the
    kernel's phases (diagnostics)."""
    B, d = x.shape
    if B == 0:
        return True
    x = x.float().contiguous()
    y = y.float().contiguous()
    assert nfit is None or nfit.dtype == torch.float64
    rc = int(native.hip().omldm_ht_exact(ptr(x), ptr(y), B, d, C, depth, N, nb, float(grace),
                                         float(delta), float(tau), _tree_ptrs(tree), ptr(nfit),
                                         ptr(dbg), native.stream_of(x)))
    if rc == -2:
        return False
    check(rc, "omldm_ht_exact")
    return True


def ht_route(x: torch.Tensor, depth: int, tree: list[torch.Tensor]) -> torch.Tensor:
    """The leaf node of every row (int32, device)."""
    B, d = x.shape
    out = torch.empty(B, dtype=torch.int32, device=x.device)
    if B:
        x = x.float().contiguous()
        check(native.hip().omldm_ht_route(ptr(x), B, d, depth, _tree_ptrs(tree), ptr(out),
                                          native.stream_of(x)), "omldm_ht_route")
    return out


def ht_predict(x: torch.Tensor, C: int, depth: int, tree: list[torch.Tensor]) -> torch.Tensor:
    B, d = x.shape
    out = torch.empty(B, dtype=torch.float32, device=x.device)
    if B:
        x = x.float().contiguous()
        check(native.hip().omldm_ht_predict(ptr(x), B, d, C, depth, _tree_ptrs(tree), ptr(out),
                                            native.stream_of(x)), "omldm_ht_predict")
    return out
