"""Linear-family ops: virtual-spoke training round, batched predict, round apply.

GPU tensors → hand-written HIP kernels (csrc/kernels/linear_spoke.hip).
CPU tensors → the C++ reference implementation (csrc/host/linear_cpu.cpp) with the
identical semantics (golden oracle + CPU engine path).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass

import torch

from omldm_amd.api.batch import HashedBatch, RawBatch
from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr

log = logging.getLogger(__name__)

STAT_W = 6  # loss_sum, n, mistakes, sq_err, sigma, overflow

RULE_HINGE, RULE_EPS, RULE_LOGISTIC, RULE_PEGASOS = 0, 1, 2, 3
RULE_MULTI = 4  # the MultiClassPA scan's prep (ops.dense.multiclass_scan3_round)
PA, PA1, PA2 = 0, 1, 2


@dataclass
class LinearRule:
    rule: int = RULE_HINGE
    variant: int = PA1
    C: float = 1.0
    eps: float = 0.1
    lr: float = 0.1
    lam: float = 0.0
    bias: bool = True
    # RULE_PEGASOS: step index T of each spoke's first row this round (row e: T + e; ≥ 2)
    tbase: float = 2.0


WS_STAT = 8  # per-spoke workspace stat columns (see linear_spoke.hip kWsStat)
_WS: dict = {}


def _workspace(device, n: int, key: str = "ws", per_stream: bool = True) -> torch.Tensor:
    """Scratch (per-spoke rows, spoke delta tables), one buffer per (device, key, current
    stream): every round kernel fully rewrites what its reduce/finish kernels read, so reuse
    is safe in stream order — and pipelines that train side by side on different streams
    (engine/job.py: pipelineStreams) get buffers of their own. ``per_stream=False``: one
    buffer per device whose caller orders the streams itself (the v3 prep ring, the v3
    run-time buffers keyed by stream in ``key``)."""
    dev = torch.device(device)
    sid = torch.cuda.current_stream(dev).cuda_stream if (per_stream and dev.type == "cuda") else 0
    k = (device, key, sid)
    t = _WS.get(k)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=device)
        _WS[k] = t
    return t


_SPILL: dict = {}


# HBM budget of one spill workspace (OMLDM_SPILL_BUDGET_MB, default 2 GiB of the 288 GB):
# a MultiClassPA spill at R = 8192 with 16-float entries would otherwise take ~1.2 GB per
# stream and up to 16 of them stay cached
_SPILL_BUDGET = int(os.environ.get("OMLDM_SPILL_BUDGET_MB", "2048")) << 20


def spill_log2cap(R: int, keys_per_row: int, S: int = 1, vk: int = 1) -> int:
    """HBM spill entries per spoke (log2): ≥ 2 × the spoke's key occurrences, so a spoke
    whose every key missed its LDS table still finds room (load ≤ 1/2), capped so the S
    spokes' spill (entries of ``vk`` values) stays within the spill budget (keys past a
    full spill are counted as overflow, which the engine's health check fails on)."""
    lg = max(6, min(24, (2 * max(1, R) * max(1, keys_per_row) - 1).bit_length()))
    words = native.hip().omldm_spill_words
    while lg > 6 and int(words(int(S), lg, int(vk))) * 4 > _SPILL_BUDGET:
        lg -= 1
    return lg


def spill_workspace(device, S: int, log2gcap: int, vk: int) -> torch.Tensor:
    """The spokes' HBM spill (csrc/kernels/spoke_table.h: Spill) for the current stream:
    keys −1, values and counters 0 when allocated; every round restores what it used, so
    the buffer stays clean across rounds without a memset."""
    dev = torch.device(device)
    sid = torch.cuda.current_stream(dev).cuda_stream
    key = (str(dev), sid, int(S), int(log2gcap), int(vk))
    t = _SPILL.get(key)
    if t is None:
        words = int(native.hip().omldm_spill_words(int(S), int(log2gcap), int(vk)))
        t = torch.zeros(words, dtype=torch.int32, device=dev)
        t[: int(S) << int(log2gcap)].fill_(-1)
        if len(_SPILL) > 16:
            _SPILL.clear()
        _SPILL[key] = t
    return t


def min_log2cap(dim: int) -> int:
    """Smallest LDS table (log2 entries) with ≥ 4 slots per key bucket for this dim."""
    ld = max(0, (dim - 1).bit_length())
    return max(4, ld - min(ld, 12) + 2)


def auto_log2cap(dim: int, rows: int, keys_per_row: int) -> int:
    """LDS delta-table size (log2 entries) for a spoke that sees ``rows`` examples with
    ``keys_per_row`` hashed keys each: load factor ≤ 1/2 for distinct keys, clamped so
    a wave's table stays ≤ 64 KiB (occupancy: 8 KiB tables allow 20 waves per CU,
    64 KiB only 2 — profiles/round1_ablation.md "Occupancy"). Keys beyond the table
    go to the spoke's HBM spill (spoke_table.h), so the size only affects speed, never
    the result: no update is dropped."""
    want = max(1, 2 * rows * max(1, keys_per_row) - 1).bit_length()
    return min(13, max(min_log2cap(dim), want))


def _cpu_threads() -> int:
    return int(os.environ.get("OMLDM_CPU_THREADS", min(8, os.cpu_count() or 1)))


def linear_round(w: torch.Tensor, batch: HashedBatch, R: int, S: int, dacc: torch.Tensor,
                 stats: torch.Tensor | None, rule: LinearRule, inv_p: float, log2cap: int = 0,
                 cum: torch.Tensor | None = None, ablate: int = 0, chunk: int = 8,
                 parts: int = 1, on_part=None) -> None:
    """One protocol round of S virtual spokes, R examples each (spoke s gets rows
    [s·R, (s+1)·R)). Every spoke with ≥1 row accumulates σ·Δ·inv_p into ``dacc[:dim]``,
    σ·inv_p into ``dacc[dim]`` and inv_p into ``dacc[dim+1]`` (so ``dacc`` is [dim+2]);
    writes per-spoke stats [S, 6] (optional) and adds the round totals into ``cum[:6]``
    (optional, device-side running counters). ``linear_apply`` then averages over the
    active workers: w = (dacc[dim]·w + dacc[:dim]) / dacc[dim+1].

    ``parts`` > 1 (GPU): the reduce of the spoke tables into ``dacc`` is issued as that
    many launches over disjoint key ranges, and ``on_part(k, lo, hi)`` runs after part k
    is enqueued with the slice ``dacc[lo:hi]`` it completes (``part_bounds``), so the
    caller can start that slice's collective while the next part reduces. The CPU path
    computes everything first and reports the same slices."""
    dim = int(dacc.shape[0]) - 2
    assert w.shape[0] == dim and (stats is None or stats.shape == (S, STAT_W))
    assert dacc.dtype == torch.float32
    assert cum is None or cum.dtype == torch.float64  # running totals, added in fp64
    num, cat, y = batch.num, batch.cat, batch.y
    assert cat.dtype == (torch.int16 if batch.cat_span else torch.int32)
    # labels: fp32, or int8 on the compact classification wire (GPU kernel reads either)
    assert y.dtype == torch.float32 or (y.dtype == torch.int8 and rule.rule != RULE_EPS)
    assert rule.rule != RULE_PEGASOS or (rule.lam > 0 and rule.tbase >= 2), "Pegasos: λ > 0, T ≥ 2"
    assert num.is_contiguous() and cat.is_contiguous() and y.is_contiguous()
    if S <= 0:
        return
    if w.is_cuda:
        # batch rows may be device tensors or pinned host memory (zero-copy ingest)
        assert all(t.is_cuda or t.is_pinned() for t in (num, cat, y)) and dacc.is_cuda
        assert stats is None or stats.is_cuda
        assert num.dtype in (torch.float32, torch.bfloat16)
        assert num.shape[1] + cat.shape[1] + int(rule.bias) <= 256, "≤ 256 features per example"
        if log2cap <= 0:  # auto: sized from rows per spoke × keys per row
            log2cap = auto_log2cap(dim, R, cat.shape[1])
        log2cap = max(log2cap, min_log2cap(dim))
        assert 4 <= log2cap <= 14
        wsw = WS_STAT + num.shape[1] + 1
        ws = _workspace(w.device, S * wsw)
        tables = _workspace(w.device, S * ((1 << log2cap) + 64) * 2, key="tables")
        lg = spill_log2cap(R, num.shape[1] + cat.shape[1] + 1, S, 1)
        spill = spill_workspace(w.device, S, lg, 1)
        dp = native.dptr
        rc = native.hip().omldm_linear_round(
            ptr(w), int(w.dtype == torch.bfloat16), dp(num), int(num.dtype == torch.bfloat16),
            num.shape[1], dp(cat), cat.shape[1], dp(y), int(y.dtype == torch.int8), batch.B, R, S,
            ptr(dacc), dim,
            ptr(ws), ptr(tables), ptr(cum), rule.rule, rule.variant, rule.C, rule.eps, rule.lr,
            rule.lam, inv_p, int(rule.bias), batch.cat_span, log2cap, int(chunk), int(ablate),
            int(parts), float(rule.tbase), ptr(spill), lg, native.stream_of(w))
        check(rc, "omldm_linear_round")
        if on_part is not None:
            on_part(0, *part_bounds(dim, 0, parts, cuda=True))
        for k in range(1, parts):
            rc = native.hip().omldm_linear_reduce_part(
                ptr(tables), ptr(ws), ptr(cum), ptr(dacc), dim, num.shape[1], cat.shape[1],
                batch.cat_span, batch.B, R, S, log2cap, k, parts, int(ablate), native.stream_of(w))
            check(rc, "omldm_linear_reduce_part")
            if on_part is not None:
                on_part(k, *part_bounds(dim, k, parts, cuda=True))
        if stats is not None:
            stats.copy_(ws[: S * wsw].view(S, wsw)[:, :STAT_W])
    else:
        num32 = num.float().contiguous()
        y = y.float().contiguous()
        st = stats if stats is not None else torch.zeros((S, STAT_W), dtype=torch.float32)
        native.host().omldm_cpu_linear_round(
            ptr(w), int(w.dtype == torch.bfloat16), ptr(num32), num32.shape[1], ptr(cat),
            cat.shape[1], ptr(y), batch.B, R, S, ptr(dacc), dim, ptr(st), rule.rule,
            rule.variant, rule.C, rule.eps, rule.lr, rule.lam, inv_p, int(rule.bias), batch.cat_span,
            float(rule.tbase), _cpu_threads())
        if cum is not None:
            cum[:STAT_W] += st.sum(0)
            cum[4] -= st[:, 4].sum()  # sigma is not a running total
        if on_part is not None:
            for k in range(parts):
                on_part(k, *part_bounds(dim, k, parts, cuda=False))


def part_bounds(dim: int, part: int, parts: int, cuda: bool = True) -> tuple[int, int]:
    """Slice [lo, hi) of a [dim + 2] round accumulator completed by reduce part ``part``
    of ``parts`` — a function of dim only, so every rank issues identical collectives
    (GPU: the kernel library's own key-group split; CPU: the same formula with the
    default geometry, 4096-key groups)."""
    if cuda:
        import ctypes

        lh = (ctypes.c_longlong * 2)()
        check(native.hip().omldm_linear_part_bounds(dim, part, parts, lh),
              "omldm_linear_part_bounds")
        return int(lh[0]), int(lh[1])
    ld = max(0, (dim - 1).bit_length())
    g = min(ld, 12)
    ng = (dim + (1 << g) - 1) >> g
    lo = 0 if part == 0 else (ng * part // parts) << g
    hi = dim + 2 if part == parts - 1 else min(dim + 2, (ng * (part + 1) // parts) << g)
    return lo, hi


def linear_apply(w32: torch.Tensor, w16: torch.Tensor | None, dacc: torch.Tensor) -> None:
    """w = dacc[dim]·w + dacc[:dim]; dacc = 0; refresh the bf16 shadow if given."""
    dim = int(w32.shape[0])
    if w32.is_cuda:
        check(native.hip().omldm_linear_apply(ptr(w32), ptr(w16), ptr(dacc), dim,
                                              native.stream_of(w32)), "omldm_linear_apply")
    else:
        native.host().omldm_cpu_linear_apply(ptr(w32), ptr(w16), ptr(dacc), dim)


def linear_apply_multi(w32s: list, w16s: list, daccs: list) -> None:
    """``linear_apply`` of M equal-size models in one launch (GPU; M ≤ 16 per launch)."""
    import ctypes

    dim = int(w32s[0].shape[0])
    if not w32s[0].is_cuda:
        for w, w16, d in zip(w32s, w16s, daccs):
            linear_apply(w, w16, d)
        return
    for i in range(0, len(w32s), 16):
        ws, hs, ds = w32s[i:i + 16], w16s[i:i + 16], daccs[i:i + 16]
        M = len(ws)
        P = lambda ts: (ctypes.c_void_p * M)(*[ptr(t) for t in ts])  # noqa: E731
        check(native.hip().omldm_linear_apply_multi(M, P(ws), P(hs), P(ds), dim,
                                                    native.stream_of(ws[0])),
              "omldm_linear_apply_multi")


def linear_predict(w: torch.Tensor, batch: HashedBatch, wscale: torch.Tensor | None = None,
                   out: torch.Tensor | None = None, bias: bool = True) -> torch.Tensor:
    """Scores for every (point, model): w is [dim] or [M, dim]; returns [B] or [B, M]."""
    single = w.dim() == 1
    W = w.unsqueeze(0) if single else w
    M, dim = int(W.shape[0]), int(W.shape[1])
    B = batch.B
    if out is None:
        out = torch.empty((B, M), dtype=torch.float32, device=w.device)
    if B == 0:
        return out.view(B) if single else out
    if w.is_cuda:
        num = batch.num
        dp = native.dptr  # inputs/outputs may be pinned host memory (zero-copy predict)
        rc = native.hip().omldm_linear_predict(
            ptr(W), int(W.dtype == torch.bfloat16), W.stride(0), M, dp(num),
            int(num.dtype == torch.bfloat16), num.shape[1], dp(batch.cat), batch.cat.shape[1], B,
            dim, int(bias), batch.cat_span, ptr(wscale), dp(out), native.stream_of(w))
        check(rc, "omldm_linear_predict")
    else:
        W32 = W.float().contiguous()
        num = batch.num.float().contiguous()
        native.host().omldm_cpu_linear_predict(ptr(W32), W32.stride(0), M, ptr(num), num.shape[1],
                                               ptr(batch.cat), batch.cat.shape[1], B, dim,
                                               int(bias), batch.cat_span, ptr(wscale), ptr(out))
    return out.view(B) if single else out


# ------------------------------------------------------------------ raw-wire sequential round
SEQ_RULES = (RULE_HINGE, RULE_EPS, RULE_LOGISTIC)  # v1 (linear_seq.hip) and the CPU oracle
# the v3 table scan also takes the rules whose model shrinks every step (w = σ·v: the L2
# shrink of SVM / RegressorPA / logistic with λ > 0, Pegasos): s3_sigma_kernel
V3_RULES = SEQ_RULES + (RULE_PEGASOS,)


def shrinks(rule: "LinearRule") -> bool:
    return rule.rule == RULE_PEGASOS or rule.lam > 0.0


def _s3_shrink(rule: "LinearRule") -> tuple[int, float, float]:
    """(shr, r, tbase) of the v3 round: 0 no shrink; 1 σ ×= r per row (r = 1 − λ, logistic
    1 − lr·λ; linear_cpu.cpp's shrink); 2 Pegasos σ ×= (T − 1)/T, T = tbase + row index."""
    if rule.rule == RULE_PEGASOS:
        return 2, 1.0, float(rule.tbase)
    if rule.lam > 0.0:
        r = 1.0 - (rule.lr * rule.lam if rule.rule == RULE_LOGISTIC else rule.lam)
        return 1, float(r), 0.0
    return 0, 1.0, 0.0


# GPU kernel of the exact sequential round: "scan3" (linear_scan3.hip, default: LDS slot
# table per spoke, whole-GPU combine) or "seq" (linear_seq.hip: every spoke builds its own
# chunk Grams on dense replicas) — an A/B knob; v3 falls back to v1 (logged once) for raw
# batches of a shape it does not take (> 8192 rows per spoke, > 32 fields)
SEQ_KERNEL = os.environ.get("OMLDM_SEQ_KERNEL", "scan3")
_V1_LOGGED: set = set()


def _log_v1_fallback(batch: RawBatch, R: int) -> None:
    key = (batch.dn, batch.dc, R)
    if SEQ_KERNEL == "scan3" and key not in _V1_LOGGED:
        _V1_LOGGED.add(key)
        log.warning("exact sequential round: shape dn=%d dc=%d R=%d is outside the v3 table "
                    "scan (linear_scan3.hip); running the v1 kernel (linear_seq.hip)", *key)


# ------------------------------------------------------------------ v3: the table scan
S3_BUFS = ("slotsT", "meta", "lidcount", "prep", "cout", "ws", "wsd", "aglob")
_S3_SHARED = (4, 5, 6, 7)  # run-time buffers (scan → combine, same stream): one set per device


@dataclass
class Scan3Prep:
    """Passes 1-3 of a v3 round (field-major slots, per-(spoke, field) occurrence flags and
    table ids, scaled chunk Grams) — model-independent, made ahead on another stream while
    the previous round scans. ``ptrs`` = the 8 workspaces."""

    bufs: list
    ptrs: object
    key: tuple          # (B, R, S, dim, bias, rule, variant, C, dn, dc) it was made for
    event: object = None
    slot: object = None  # workspace set (ring slot "k<i>" for inline preps)
    ready: object = None  # (ready word address, epoch): set at the prep's end on its stream


# The preps' ready words, one per (device, workspace slot), each counting its preps. A prep
# made on a stream of its own ends with omldm_scan3_signal, and the round's launch waits for
# the word in its workgroups (omldm_scan3_wait_next) instead of a cross-stream wait on the
# prep's event: that barrier packet released the scan ~11 µs after the previous round's
# apply (profiles/round5/devgap/: 0.311 → 0.292 ms per device-ingest round).
# OMLDM_S3_READY=0: the event wait (A/B).
_S3_READY_WAIT = os.environ.get("OMLDM_S3_READY", "1") != "0"
_S3_READY: dict = {}


def _s3_ready_word(dev, slot):
    rec = _S3_READY.get(str(dev))
    if rec is None:
        rec = _S3_READY[str(dev)] = (torch.zeros(256, dtype=torch.int64, device=dev), {}, {})
        torch.cuda.synchronize(dev)  # zero before a prep stream's first signal lands
    words, index, epochs = rec
    i = index.get(slot)
    if i is None:
        if len(index) >= words.numel():
            return None
        i = index[slot] = len(index)
    epochs[slot] = epochs.get(slot, 0) + 1
    return words.data_ptr() + 8 * i, epochs[slot]


def _s3_wait_prep(sp, dev) -> None:
    """Order the next v3 launch on the current stream after the prep ``sp``."""
    if _S3_READY_WAIT and sp.ready is not None:
        _s3_lib().omldm_scan3_wait_next(sp.ready[0], sp.ready[1])
    elif sp.event is not None:
        torch.cuda.current_stream(dev).wait_event(sp.event)


# v3 table-scan kernel generation: 4 = the split spoke (a scanner and a table workgroup per
# spoke, csrc/kernels/linear_scan3.hip: s4_scan_kernel), 3 = one workgroup per spoke with
# in-launch combiners (the A/B reference). Fixed per process before the first prepare.
S3_MODE = int(os.environ.get("OMLDM_S3_MODE", "4"))
_S3_MODE_SET = {"done": False}


def _s3_lib():
    h = native.hip()
    if not _S3_MODE_SET["done"]:
        h.omldm_scan3_set_mode(S3_MODE)
        # A/B: the launch form (0 auto, 1 latency form always, 2 throughput form always)
        h.omldm_scan3_set_form(int(os.environ.get("OMLDM_S3_FORM", "0")))
        h.omldm_scan3_set_cns(int(os.environ.get("OMLDM_S3_CNS", "0")))
        # A/B: 0 = the combiner workgroups (the round-5 form) instead of the in-scan combine
        h.omldm_scan3_set_inscan(int(os.environ.get("OMLDM_S3_INSCAN", "1")))
        _S3_MODE_SET["done"] = True
    return h


def set_scan3_mode(mode: int) -> int:
    """Switch the v3/v4 round generation (tests, A/B); returns the previous one. The
    device must be idle: preps made for the other layout are dropped with the caches."""
    global S3_MODE
    old = S3_MODE
    S3_MODE = 3 if int(mode) == 3 else 4
    native.hip().omldm_scan3_set_mode(S3_MODE)
    _S3_MODE_SET["done"] = True
    _S3_WS_CACHE.clear()
    _S3_RUN_CACHE.clear()
    return old


def scan3_fits(dn: int, dc: int, R: int, bias: bool) -> bool:
    return bool(_s3_lib().omldm_scan3_fits(int(dn), int(dc), int(R), int(bias)))


def scan3_eligible(batch: RawBatch, R: int, bias: bool) -> bool:
    return (SEQ_KERNEL == "scan3" and batch.y.is_cuda and 0 < batch.dc
            and scan3_fits(batch.dn, batch.dc, R, bias))


def _s3_span(batch: RawBatch, dim: int) -> int:
    """Slots per field: the compact wire's cat_span, else the token hashing's."""
    return int(batch.span) if batch.span > 0 else (dim - batch.dn - 1) // batch.dc


def scan3_eligible_compact(batch: RawBatch, R: int, bias: bool, dim: int) -> bool:
    """v3 on compact slots: the field ranges [cbase + f·span, …) must fit the model."""
    return (scan3_eligible(batch, R, bias)
            and batch.cbase + batch.dc * batch.span <= dim - 1)


def _s3_mode(batch: RawBatch, hashed: bool) -> int:
    """s3_slots_kernel input: 0 tokens, 1 int32 signed slots, 2 compact int16 slots."""
    if batch.span > 0:
        assert batch.tok.dtype == torch.int16, batch.tok.dtype
        return 2
    assert batch.tok.dtype == torch.int32, batch.tok.dtype
    return 1 if hashed else 0


def _s3_key(batch, R, S, dim, bias, rule: "LinearRule") -> tuple:
    """What a v3 prep depends on: the batch, the geometry, the rule's row scale (C only
    through PA-II's 1/(2C)) — pipelines that differ in C share one prep."""
    c = float(rule.C) if rule.variant == PA2 else None
    # the row scaling depends on the rule family (a = −1/(‖x‖²+kadd), 1 or y) and the shrink
    fam = {RULE_PEGASOS: 2, RULE_LOGISTIC: 1, RULE_MULTI: 3}.get(rule.rule, 0)
    # logistic without shrink: lr·y in the Grams' columns (linear_scan3.hip s3_gram_colscale)
    lr = float(rule.lr) if fam == 1 and _s3_shrink(rule)[0] == 0 else None
    return (batch.B, R, S, dim, bool(bias), fam, rule.variant == PA2, c, _s3_shrink(rule), lr,
            batch.dn, batch.dc, int(batch.span), batch.y.data_ptr(), batch.tok.data_ptr(), S3_MODE)


_S3_WS_CACHE: dict = {}


def _s3_workspaces(dev, B, R, S, dn, dc, span, bias, slot):
    """The 8 workspaces of a v3 round and their pointer array, cached per geometry (the
    lookup + ctypes array were a per-tick host cost); refreshed if a workspace moved."""
    import ctypes

    h = _s3_lib()
    key = (str(dev), B, R, S, dn, dc, span, bias, slot, S3_MODE)
    hit = _S3_WS_CACHE.get(key)
    bufs = []
    for i, name in enumerate(S3_BUFS):
        n = int(h.omldm_scan3_ws_words(i, B, R, S, dn, dc, span, int(bias))) if hit is None \
            else hit[2][i]
        wkey = f"s3_{name}" if i in _S3_SHARED else f"s3_{name}{slot}"
        bufs.append(_workspace(dev, n, key=wkey, per_stream=False))
    if hit is not None and all(a.data_ptr() == b.data_ptr() for a, b in zip(bufs, hit[0])):
        return hit[0], hit[1]
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
    sizes = [int(h.omldm_scan3_ws_words(i, B, R, S, dn, dc, span, int(bias)))
             for i in range(len(S3_BUFS))]
    if len(_S3_WS_CACHE) > 64:
        _S3_WS_CACHE.clear()
    _S3_WS_CACHE[key] = (bufs, ptrs, sizes)
    return bufs, ptrs


_S3_RUN_CACHE: dict = {}
_S3_SLOTS = {"next": 0}
S3_SLOT_RING = 16


_S3_SLOT_LAST: dict = {}  # ring slot → event after the last scan that read its prep


def _s3_slot_for(key, device=None) -> str:
    """Workspace set of an inline prep: a ring of 16, one per distinct prep key in turn.
    Pipelines of one tick may scan on different streams, so two preps alive at once must
    not share buffers; a slot that comes round again while a scan on another stream may
    still read it is reused only after that scan (the current stream — the one the new
    prep is made on — waits on the event the last scan of the slot recorded)."""
    i = _S3_SLOTS["next"]
    _S3_SLOTS["next"] = (i + 1) % S3_SLOT_RING
    slot = f"k{i}"
    ev = _S3_SLOT_LAST.pop(slot, None)
    if ev is not None:
        torch.cuda.current_stream(device).wait_event(ev)
    return slot


def _s3_mark_read(sp: "Scan3Prep") -> None:
    """Record that a scan on the current stream read ``sp``'s ring slot (if it has one)."""
    slot = getattr(sp, "slot", None)
    if slot is not None and str(slot).startswith("k"):
        ev = torch.cuda.Event()
        ev.record()
        _S3_SLOT_LAST[str(slot)] = ev


# The scanner's per-row c granules {epoch, c} (one buffer per stream): zeroed when
# allocated, and every round on the buffer tags its granules with the next epoch, so the
# combiner workgroups of a round never take an earlier round's granule for this one's.
_S3_GRAN: dict = {}


def _s3_granules(dev, n: int, stream: int) -> list:
    key = (str(dev), stream)
    g = _S3_GRAN.get(key)
    if g is None or g[0].numel() < n + 2:  # + the round's arrival word (the last 8 bytes)
        t = torch.zeros(max(n + 2, 1 << 17), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)  # zeroed before any stream's round reads it
        g = [t, 0]
        _S3_GRAN[key] = g
    return g


def _s3_next_epoch(g: list) -> int:
    g[1] += 1
    if g[1] >= 0xFFFFFFFF:  # wrapped: start over on a zeroed buffer
        g[0].zero_()
        torch.cuda.synchronize(g[0].device)
        g[1] = 1
    return g[1]


def _s3_run_ptrs(sp: "Scan3Prep", dev, stream: int, lane: int = 0):
    """The prep's 4 model-independent workspaces + this stream's 4 run-time ones (run-time
    set ``lane`` of the stream: pipelines of one multi-pipeline launch each take their own),
    and the set's granule buffer entry [tensor, epoch]."""
    import ctypes

    sk = stream if lane == 0 else (stream, lane)
    key = (id(sp), sk)
    hit = _S3_RUN_CACHE.get(key)
    if hit is not None and hit[0] is sp and hit[3][0] is _S3_GRAN.get((str(dev), sk), [None])[0]:
        return hit[1], hit[3]
    run = []
    gran = None
    for i in _S3_SHARED:
        n = sp.bufs[i].numel()
        if S3_BUFS[i] == "cout":
            gran = _s3_granules(dev, n, sk)
            run.append(gran[0])
        else:
            run.append(_workspace(dev, n, key=f"s3_{S3_BUFS[i]}@{sk}", per_stream=False))
    ptrs = (ctypes.c_void_p * len(S3_BUFS))(*([b.data_ptr() for b in sp.bufs[:4]] +
                                              [b.data_ptr() for b in run]))
    if len(_S3_RUN_CACHE) > 256:
        _S3_RUN_CACHE.clear()
    _S3_RUN_CACHE[key] = (sp, ptrs, run, gran)
    return ptrs, gran


def linear_scan3_prepare(batch: RawBatch, R: int, S: int, dim: int, bias: bool,
                         rule: "LinearRule", slot: int = 0, stream=None,
                         hashed: bool = False) -> Scan3Prep:
    """Passes 1-3 of a v3 round into workspace set ``slot`` on ``stream`` (default: the
    current stream; an event marks completion when a stream is given). ``batch.tok``:
    32-bit category tokens, (``hashed``) int32 field-aware signed slots, or (``batch.span``
    > 0) the compact int16 field-aware slots of the engine's wire, row-major."""
    h = _s3_lib()
    if "OMLDM_S3_GRAM_VALU" in os.environ:  # A/B: pass 3 on the VALU reference kernel
        h.omldm_scan3_set_gram_valu(int(os.environ["OMLDM_S3_GRAM_VALU"]))
    if "OMLDM_S3_PREP_SPLIT" in os.environ:  # A/B: 0 = flags and Grams on one stream
        h.omldm_scan3_set_prep_split(int(os.environ["OMLDM_S3_PREP_SPLIT"]))
    dev = batch.y.device
    span = _s3_span(batch, dim)
    mode = _s3_mode(batch, hashed)
    bufs, ptrs = _s3_workspaces(dev, batch.B, R, S, batch.dn, batch.dc, span, bool(bias), slot)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    y = batch.y
    assert y.dtype in (torch.float32, torch.int8) and y.is_contiguous()
    check(h.omldm_scan3_prepare(ptr(batch.num), batch.dn, ptr(batch.tok), mode, batch.dc, ptr(y),
                                int(y.dtype == torch.int8), batch.B, R, S, dim, int(bias),
                                rule.rule, rule.variant, float(rule.C), span,
                                int(batch.cbase) if batch.span > 0 else -1, *_s3_shrink(rule),
                                float(rule.lr), ptrs, st.cuda_stream), "omldm_scan3_prepare")
    ev = torch.cuda.Event()  # pipelines on other streams that reuse the prep wait on it
    ev.record(st)
    ready = None
    if stream is not None and _S3_READY_WAIT:
        ready = _s3_ready_word(dev, slot)
        if ready is not None:
            check(h.omldm_scan3_signal(ready[0], ready[1], st.cuda_stream), "omldm_scan3_signal")
    return Scan3Prep(bufs, ptrs, _s3_key(batch, R, S, dim, bias, rule), ev, slot, ready)


def scan3_part_bounds(dim: int, dn: int, dc: int, part: int, parts: int,
                      span: int = 0) -> tuple[int, int]:
    import ctypes

    lh = (ctypes.c_longlong * 2)()
    check(native.hip().omldm_scan3_part_bounds(dim, dn, dc, span, part, parts, lh),
          "omldm_scan3_part_bounds")
    return int(lh[0]), int(lh[1])


_S3_TAIL_KERNEL = os.environ.get("OMLDM_S3_TAIL") == "kernel"

# rounds run through the v3 scan in this process (tests: the engine's default path)
SCAN3_ROUNDS = 0


def linear_scan3_round(w: torch.Tensor, batch: RawBatch, R: int, S: int, dacc: torch.Tensor,
                       rule: "LinearRule", inv_p: float, cum: torch.Tensor | None = None,
                       parts: int = 1, on_part=None, hashed: bool = False,
                       dacc_zero: bool = True) -> None:
    # ``w``: the fp32 model, or its bf16 copy (modelDtype bf16: margins on the bf16 weights;
    # linear_apply updates the fp32 master and refreshes the copy)
    """One Synchronous round through the v3 table scan (csrc/kernels/linear_scan3.hip):
    dacc[:dim] += inv_p·Σ_spokes Δ_s, dacc[dim] = dacc[dim+1] = S_act·inv_p, so
    ``linear_apply`` averages the spokes' replicas into w. Like every round kernel it
    expects dacc[:dim] = 0 on entry (``linear_apply`` leaves it so); ``dacc_zero=False``
    zeroes it first. The combine
    runs in ``parts`` launches over key ranges; ``on_part(k, lo, hi)`` is called after
    part k with the slice of dacc it completed (its collective may start then)."""
    dim = int(dacc.shape[0]) - 2
    num, y = batch.num, batch.y
    sp = batch.prep
    key = _s3_key(batch, R, S, dim, rule.bias, rule)
    if not (isinstance(sp, Scan3Prep) and sp.key == key):
        sp = linear_scan3_prepare(batch, R, S, dim, bool(rule.bias), rule, hashed=hashed,
                                  slot=_s3_slot_for(key, w.device))
        batch.prep = sp  # the next pipeline of the tick reuses it (same key)
    else:
        _s3_wait_prep(sp, w.device)
    global SCAN3_ROUNDS
    SCAN3_ROUNDS += 1
    h = _s3_lib()
    if SCAN3_ROUNDS == 1 and "OMLDM_S3_COMB" in os.environ:  # A/B: 0 = combine after the scan
        h.omldm_scan3_set_comb(int(os.environ["OMLDM_S3_COMB"]))
    parts = max(1, int(parts))
    span = _s3_span(batch, dim)
    # run-time buffers (c per row, spoke statistics, the table spill) per stream: pipelines
    # on different streams may scan the same prep concurrently
    ptrs, gran = _s3_run_ptrs(sp, w.device, native.stream_of(w))
    epoch = _s3_next_epoch(gran)
    # the round's tail runs in the scan's launch (its last scan block) on an arrival word at
    # the granule buffer's end (OMLDM_S3_TAIL=kernel: a separate kernel after the scan)
    arrive = (None if _S3_TAIL_KERNEL else
              gran[0].data_ptr() + (gran[0].numel() // 2 - 1) * 8)
    for k in range(parts):
        flags = int(bool(dacc_zero)) | (2 if w.dtype == torch.bfloat16 else 0)
        rc = h.omldm_scan3_run(ptr(w), num.shape[1], batch.dc, ptr(y), int(y.dtype == torch.int8),
                               batch.B, R, S, ptr(dacc), dim, ptr(cum), rule.rule, rule.variant,
                               rule.C, rule.eps, rule.lr, inv_p, int(rule.bias), span, ptrs, k,
                               parts, flags, epoch, arrive, _s3_shrink(rule)[0],
                               float(rule.lam), float(rule.tbase), native.stream_of(w))
        check(rc, "omldm_scan3_run")
        if on_part is not None:
            on_part(k, *scan3_part_bounds(dim, batch.dn, batch.dc, k, parts, span))
    _s3_mark_read(sp)


def scan3_max_pipes() -> int:
    return int(_s3_lib().omldm_scan3_max_pipes())


def linear_scan3_round_multi(ws: list, batch: RawBatch, R: int, S: int, daccs: list,
                             rules: list, inv_p: float, cums: list | None = None,
                             hashed: bool = False) -> None:
    """M Synchronous rounds of M pipelines on ONE batch through ONE v3 launch (BASELINE
    config 5: concurrent classifiers on the same stream; csrc/kernels/linear_scan3.hip
    s3_scan_kernel with M pipelines): one shared prep, per pipeline its model, accumulator,
    granule buffer and rule constants. Every rule must share the prep (same row scaling)
    and the update family; each accumulator ends as ``linear_scan3_round``'s would."""
    import ctypes

    M = len(ws)
    assert 1 <= M <= scan3_max_pipes() and len(daccs) == M and len(rules) == M
    assert len({w.dtype for w in ws}) == 1, "one launch: every model fp32 or every model bf16"
    r0 = rules[0]
    dim = int(daccs[0].shape[0]) - 2
    key = _s3_key(batch, R, S, dim, r0.bias, r0)
    assert all(_s3_key(batch, R, S, dim, r.bias, r) == key and r.rule == r0.rule and
               r.variant == r0.variant for r in rules), "pipelines must share the prep and rule"
    sp = batch.prep
    if not (isinstance(sp, Scan3Prep) and sp.key == key):
        sp = linear_scan3_prepare(batch, R, S, dim, bool(r0.bias), r0, hashed=hashed,
                                  slot=_s3_slot_for(key, ws[0].device))
        batch.prep = sp
    else:
        _s3_wait_prep(sp, ws[0].device)
    global SCAN3_ROUNDS
    SCAN3_ROUNDS += 1
    h = _s3_lib()
    stream = native.stream_of(ws[0])
    span = _s3_span(batch, dim)
    ptrs, epochs, arrives = [], [], []
    for m in range(M):
        pm, gran = _s3_run_ptrs(sp, ws[m].device, stream, lane=m)
        ptrs += list(pm)
        epochs.append(_s3_next_epoch(gran))
        arrives.append(None if _S3_TAIL_KERNEL else
                       gran[0].data_ptr() + (gran[0].numel() // 2 - 1) * 8)
    cums = cums if cums is not None else [None] * M
    P = lambda ts: (ctypes.c_void_p * M)(*[ptr(t) for t in ts])  # noqa: E731
    F = lambda vs: (ctypes.c_float * M)(*[float(v) for v in vs])  # noqa: E731
    num, y = batch.num, batch.y
    check(h.omldm_scan3_run_multi(
        M, P(ws), P(daccs), P(cums), F([r.C for r in rules]), F([r.eps for r in rules]),
        F([r.lr for r in rules]), F([inv_p] * M), (ctypes.c_void_p * (8 * M))(*ptrs),
        (ctypes.c_uint * M)(*epochs), (ctypes.c_void_p * M)(*arrives), num.shape[1], batch.dc,
        ptr(y), int(y.dtype == torch.int8), batch.B, R, S, dim, r0.rule, r0.variant,
        int(r0.bias), span, 1 | (2 if ws[0].dtype == torch.bfloat16 else 0),
        _s3_shrink(r0)[0], F([r.lam for r in rules]),
        F([r.tbase for r in rules]), stream), "omldm_scan3_run_multi")
    _s3_mark_read(sp)


def linear_seq_round(w: torch.Tensor, batch: RawBatch, R: int, S: int, dacc: torch.Tensor,
                     rule: LinearRule, inv_p: float, cum: torch.Tensor | None = None,
                     stats: torch.Tensor | None = None, replicas: torch.Tensor | None = None,
                     parts: int = 1, on_part=None, hashed: bool = False) -> bool:
    """One Synchronous round on the raw binary wire: S spokes, spoke s an exact
    sequential learner (the reference's per-example fit, FlinkSpoke.scala:92-107) over
    rows [s·R, (s+1)·R) on its own replica of w; tokens are hashed inside the round.

    Accumulates like ``linear_round`` (dacc[:dim] += Δ_s·inv_p, dacc[dim] and
    dacc[dim+1] += inv_p per active spoke), so ``linear_apply`` averages the replicas.
    GPU: csrc/kernels/linear_seq.hip (Gram-scan on the matrix cores, one workgroup per
    spoke; ``replicas`` is its [S, dim] fp32 scratch, allocated here if None).
    CPU: csrc/host/rawwire.cpp (the golden oracle)."""
    dim = int(dacc.shape[0]) - 2
    assert w.shape[0] == dim and dacc.dtype == torch.float32
    assert w.dtype == torch.float32 or (w.dtype == torch.bfloat16 and w.is_cuda)
    assert rule.rule in V3_RULES, "seq round: PA family / logistic (+ Pegasos on v3)"
    num, tok, y = batch.num, batch.tok, batch.y
    assert num.dtype == torch.float32
    assert tok.dtype == (torch.int16 if batch.span > 0 else torch.int32), tok.dtype
    assert y.dtype == torch.float32 or (y.dtype == torch.int8 and rule.rule != RULE_EPS)
    assert num.is_contiguous() and tok.is_contiguous() and y.is_contiguous()
    assert cum is None or cum.dtype == torch.float64
    if S <= 0 or batch.B == 0:
        return False
    if batch.span > 0:  # compact slots: the v3 round is the only consumer
        assert w.is_cuda and scan3_eligible(batch, R, rule.bias) and stats is None
    if w.is_cuda and scan3_eligible(batch, R, rule.bias) and stats is None:
        assert all(t.is_cuda for t in (num, tok, y)) and dacc.is_cuda
        linear_scan3_round(w, batch, R, S, dacc, rule, inv_p, cum, parts, on_part, hashed)
        return True
    # a shrinking rule (L2, Pegasos) or a bf16 model has no v1 / raw CPU form: the learner
    # hashes the batch and takes the spoke-table round instead (models/linear.py: seq_capable)
    assert not shrinks(rule) and w.dtype == torch.float32, \
        "shrinking rules / bf16 models take the v3 scan or the spoke-table round"
    if on_part is not None:  # the other paths complete dacc in one go
        def _report():
            for k in range(max(1, int(parts))):
                on_part(k, *part_bounds(int(dacc.shape[0]) - 2, k, max(1, int(parts)),
                                        cuda=dacc.is_cuda))
    else:
        def _report():
            pass
    if w.is_cuda:
        assert all(t.is_cuda for t in (num, tok, y)) and dacc.is_cuda
        ws = _workspace(w.device, S * WS_STAT, key="seq_ws")
        if replicas is None:
            replicas = _workspace(w.device, S * dim, key="seq_replicas")
        _log_v1_fallback(batch, R)  # v1 (csrc/kernels/linear_seq.hip)
        rc = native.hip().omldm_linear_seq_round(
            ptr(w), ptr(num), num.shape[1], ptr(tok), tok.shape[1], ptr(y),
            int(y.dtype == torch.int8), batch.B, R, S, ptr(replicas), ptr(dacc), dim,
            ptr(ws), ptr(cum), rule.rule, rule.variant, rule.C, rule.eps, rule.lr, inv_p,
            int(rule.bias), native.stream_of(w))
        check(rc, "omldm_linear_seq_round")
        if stats is not None:
            stats.copy_(ws[: S * WS_STAT].view(S, WS_STAT)[:, :STAT_W])
        _report()
    else:
        st = stats if stats is not None else torch.zeros((S, STAT_W), dtype=torch.float32)
        native.host().omldm_cpu_linear_seq_round(
            ptr(w), ptr(num), num.shape[1], ptr(tok), tok.shape[1], ptr(y),
            int(y.dtype == torch.int8), batch.B, R, S, ptr(dacc), dim, ptr(st), rule.rule,
            rule.variant, rule.C, rule.eps, rule.lr, inv_p, int(rule.bias), _cpu_threads())
        if cum is not None:
            cum[:STAT_W] += st.sum(0).double()
            cum[4] -= st[:, 4].sum().double()
        _report()
    return False


def linear_seq_round64(w: torch.Tensor, batch: RawBatch, R: int, S: int, dacc: torch.Tensor,
                       rule: "LinearRule", inv_p: float) -> None:
    """The reference semantics of one Synchronous round in DOUBLE precision (CPU; the
    reference's Breeze Double model, omldm/state/StateAccumulators.scala:5,26): spoke s fits
    rows [sR, sR + R) one at a time on its fp64 replica, dacc (fp64, [dim + 2]) collects the
    averaged deltas; ``linear_apply64`` folds it into w. The fp32 kernels' parity row."""
    assert w.dtype == torch.float64 and dacc.dtype == torch.float64 and not w.is_cuda
    num, tok, y = batch.num.contiguous(), batch.tok.contiguous(), batch.y.contiguous()
    dim = int(dacc.shape[0]) - 2
    st = torch.zeros((S, STAT_W), dtype=torch.float32)
    check(native.host().omldm_cpu_linear_seq_round64(
        ptr(w), ptr(num), num.shape[1], ptr(tok), tok.shape[1], ptr(y),
        int(y.dtype == torch.int8), batch.B, R, S, ptr(dacc), dim, ptr(st), rule.rule,
        rule.variant, rule.C, rule.eps, rule.lr, inv_p, int(rule.bias), _cpu_threads()),
        "omldm_cpu_linear_seq_round64")


def linear_apply64(w: torch.Tensor, dacc: torch.Tensor) -> None:
    """fp64 ``linear_apply``: w = (dacc[dim]·w + dacc[:dim]) / dacc[dim+1]; dacc = 0."""
    dim = int(w.shape[0])
    n = float(dacc[dim + 1])
    if n > 0:
        w.mul_(float(dacc[dim])).add_(dacc[:dim]).div_(n)
    dacc.zero_()


def linear_seq_apply(w: torch.Tensor, replicas: torch.Tensor, dacc: torch.Tensor) -> None:
    """GPU: w = model average of the (all-reduced) round accumulator, every replica ← w,
    dacc ← 0 (one pass over HBM)."""
    check(native.hip().omldm_linear_seq_apply(ptr(w), ptr(replicas), int(replicas.shape[0]),
                                              ptr(dacc), int(w.shape[0]), native.stream_of(w)),
          "omldm_linear_seq_apply")


def linear_seq_broadcast(w: torch.Tensor, replicas: torch.Tensor) -> None:
    check(native.hip().omldm_linear_seq_broadcast(ptr(w), ptr(replicas), int(replicas.shape[0]),
                                                  int(w.shape[0]), native.stream_of(w)),
          "omldm_linear_seq_broadcast")
