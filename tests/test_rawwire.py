"""Raw binary wire (32-bit category tokens hashed inside the round) and the exact
sequential Gram-scan round (csrc/kernels/linear_seq.hip) against the CPU oracle
(csrc/host/rawwire.cpp) and a pure-Python per-example golden model.

Reference semantics pinned here: each spoke fits its shard one example at a time on its
own replica (omldm/operators/spoke/FlinkSpoke.scala:92-107) and the Synchronous PS
averages the replicas.
"""
from __future__ import annotations

import struct

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, RawBatch
from omldm_amd.io.synthetic import synth_raw
from omldm_amd.ops import linear as L
from omldm_amd.ops import native
from omldm_amd.ops.ingest import hash_raw

gpu = pytest.mark.gpu


def _cuda():
    return torch.device("cuda", 0)


def _golden_round(w, batch, space, R, S, rule, C=1.0, eps=0.1, lr=0.1, bias=True):
    """Per-example sequential learners, replicas averaged (fp64, pure Python)."""
    dim = space.dim
    num = batch.num.double().numpy()
    cat = hash_raw(batch.tok, space).numpy()
    y = batch.y.double().numpy()
    B = batch.B
    deltas, n_act = [], 0
    for s in range(S):
        a, b = min(s * R, B), min(s * R + R, B)
        if a >= b:
            continue
        n_act += 1
        d = {}
        for t in range(a, b):
            idx = list(range(space.dn))
            xv = list(num[t])
            for j in range(space.dc):
                c = int(cat[t, j])
                if c == -1:
                    continue
                idx.append(c & 0x7FFFFFFF)
                xv.append(-1.0 if c < 0 else 1.0)
            if bias:
                idx.append(dim - 1)
                xv.append(1.0)
            m = sum(x * (float(w[i]) + d.get(i, 0.0)) for i, x in zip(idx, xv))
            n2 = sum(x * x for x in xv)
            if rule == L.RULE_HINGE:
                l = max(0.0, 1 - y[t] * m)
                c_ = min(C, l / n2) * y[t] if n2 > 0 else 0.0
            elif rule == L.RULE_EPS:
                err = y[t] - m
                l = max(0.0, abs(err) - eps)
                tau = min(C, l / n2) if n2 > 0 else 0.0
                c_ = tau if err >= 0 else -tau
            else:
                c_ = lr * y[t] / (1 + np.exp(y[t] * m))
            for i, x in zip(idx, xv):
                d[i] = d.get(i, 0.0) + c_ * x
        deltas.append(d)
    out = w.double().clone()
    for d in deltas:
        for i, v in d.items():
            out[i] += v / n_act
    return out


def test_raw_hash_is_field_aware_murmur3():
    """A 32-bit token hashes as murmur3_32 of its 4 little-endian bytes with the field's
    seed, into the field's own slot range (dn + f·span, span = (dim − dn − 1) / dc)."""
    space = FeatureSpace(13, 0, 26, 1 << 20)
    span = (space.dim - 13 - 1) // 26
    rng = np.random.default_rng(1)
    tok = torch.from_numpy(rng.integers(-2**31, 2**31 - 1, size=(7, 26), dtype=np.int64)
                           .astype(np.int32))
    tok[0, 3] = -1  # absent (0xFFFFFFFF)
    got = hash_raw(tok, space)
    h = native.host()
    for i in range(7):
        for j in range(26):
            t = int(tok[i, j]) & 0xFFFFFFFF
            if t == 0xFFFFFFFF:
                assert int(got[i, j]) == -1
                continue
            m = h.omldm_murmur3_32(struct.pack("<I", t), 4, 0x9747B28C + j)
            slot = 13 + j * span + (m & 0x7FFFFFFF) % span
            want = slot | 0x80000000 if m & 0x80000000 else slot
            assert int(got[i, j]) & 0xFFFFFFFF == want
            assert 13 + j * span <= (int(got[i, j]) & 0x7FFFFFFF) < 13 + (j + 1) * span


def test_synth_raw_is_a_pure_function_of_seed_and_position():
    space = FeatureSpace(13, 0, 26, 1 << 20)
    a = synth_raw(space, 100, start=50, seed=7)
    b = synth_raw(space, 40, start=80, seed=7)
    assert torch.equal(a.num[30:70], b.num[:40]) and torch.equal(a.tok[30:70], b.tok[:40])
    assert torch.equal(a.y[30:70], b.y[:40])
    c = synth_raw(space, 100, start=50, seed=8)
    assert not torch.equal(a.tok, c.tok)
    assert set(a.y.unique().tolist()) <= {-1.0, 1.0}


@pytest.mark.parametrize("rule", [L.RULE_HINGE, L.RULE_EPS, L.RULE_LOGISTIC])
def test_cpu_seq_round_matches_golden(rule):
    space = FeatureSpace(5, 0, 6, 1 << 10)
    task = 1 if rule == L.RULE_EPS else 0
    batch = synth_raw(space, 150, seed=3, task=task, missing=0.1)
    w = torch.randn(space.dim) * 0.01
    dacc = torch.zeros(space.dim + 2)
    S, R = 4, 40  # last spoke: 30 rows
    lr = L.LinearRule(rule=rule, variant=L.PA1, C=0.5, eps=0.1, lr=0.1)
    w1 = w.clone()
    L.linear_seq_round(w1, batch, R, S, dacc, lr, 1.0 / S)
    L.linear_apply(w1, None, dacc)
    ref = _golden_round(w, batch, space, R, S, rule, C=0.5)
    assert torch.allclose(w1.double(), ref, atol=1e-5, rtol=1e-4)


def test_reference_geometry_learns_faster_per_example():
    """Why the headline runs the reference's 16 sequential spokes: at equal examples, many
    small-shard replicas averaged per round learn much slower (bench/accuracy_sweep.py)."""
    space = FeatureSpace(13, 0, 26, 1 << 16)
    rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
    test = synth_raw(space, 4000, start=10**9, seed=25).hashed(space)

    def acc_after(S, R, rounds):
        w, dacc = torch.zeros(space.dim), torch.zeros(space.dim + 2)
        for k in range(rounds):
            b = synth_raw(space, S * R, start=k * S * R, seed=25)
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S)
            L.linear_apply(w, None, dacc)
        return float(((L.linear_predict(w, test) >= 0).float() * 2 - 1 == test.y).float().mean())

    ref = acc_after(16, 1024, 8)          # 131 072 examples, 16 spokes
    many = acc_after(2048, 8, 8)          # same examples, 2048 spokes
    assert ref > many + 0.02, (ref, many)


# ------------------------------------------------------------------------------ GPU
@gpu
def test_gpu_hash_raw_matches_cpu():
    space = FeatureSpace(13, 0, 26, (1 << 20) - 3)
    b = synth_raw(space, 3000, seed=5, missing=0.05)
    assert torch.equal(hash_raw(b.tok.to(_cuda()), space).cpu(), hash_raw(b.tok, space))


@pytest.fixture
def kernel(request, monkeypatch):
    monkeypatch.setattr(L, "SEQ_KERNEL", request.param)
    return request.param


def _seq_case(space, B, S, R, rule, variant=L.PA1, task=0, missing=0.0, y8=False, bias=True,
              seed=11, scale=0.01):
    batch = synth_raw(space, B, seed=seed, task=task, missing=missing)
    if y8:
        batch = RawBatch(batch.num, batch.tok, batch.y.to(torch.int8))
    w = torch.randn(space.dim, generator=torch.Generator().manual_seed(seed)) * scale
    lr = L.LinearRule(rule=rule, variant=variant, C=0.7, eps=0.1, lr=0.2, bias=bias)
    wc, dc = w.clone(), torch.zeros(space.dim + 2)
    L.linear_seq_round(wc, batch, R, S, dc, lr, 1.0 / S)
    L.linear_apply(wc, None, dc)
    dev = _cuda()
    wg, dg = w.to(dev), torch.zeros(space.dim + 2, device=dev)
    rep = torch.empty((S, space.dim), device=dev)
    L.linear_seq_broadcast(wg, rep)
    cum = torch.zeros(8, dtype=torch.float64, device=dev)
    L.linear_seq_round(wg, batch.to(dev), R, S, dg, lr, 1.0 / S, cum=cum, replicas=rep)
    L.linear_seq_apply(wg, rep, dg)
    torch.cuda.synchronize()
    return wc, wg.cpu(), rep.cpu(), cum.cpu(), batch


@gpu
@pytest.mark.parametrize("kernel", ["seq"], indirect=True)  # v3: test_scan3.py
@pytest.mark.parametrize("rule,variant,task", [(L.RULE_HINGE, L.PA1, 0), (L.RULE_HINGE, L.PA, 0),
                                               (L.RULE_HINGE, L.PA2, 0), (L.RULE_EPS, L.PA1, 1),
                                               (L.RULE_LOGISTIC, L.PA1, 0)])
def test_gpu_seq_round_matches_cpu(kernel, rule, variant, task):
    space = FeatureSpace(13, 0, 26, 1 << 16)
    # 5 spokes × 300 rows (chunks of 64: 4 full + a 44-row tail) + a 100-row last spoke
    wc, wg, rep, cum, batch = _seq_case(space, 1300, 5, 300, rule, variant, task, missing=0.05)
    assert torch.allclose(wg, wc, atol=2e-4, rtol=1e-3), (wg - wc).abs().max()
    assert torch.equal(rep, wg.unsqueeze(0).expand_as(rep))  # replicas refreshed
    assert int(cum[1]) == 1300


@gpu
@pytest.mark.parametrize("kernel", ["seq"], indirect=True)  # v3: test_scan3.py
def test_gpu_seq_round_int8_labels_no_bias_wide_dense(kernel):
    # dn + bias > 16: the 32-column dense MFMA path; int8 labels; no intercept
    space = FeatureSpace(20, 0, 8, 1 << 12)
    wc, wg, _, cum, _ = _seq_case(space, 700, 3, 256, L.RULE_HINGE, y8=True, bias=False)
    assert torch.allclose(wg, wc, atol=2e-4, rtol=1e-3), (wg - wc).abs().max()


@gpu
@pytest.mark.parametrize("kernel", ["seq"], indirect=True)  # v3: test_scan3.py
def test_gpu_seq_round_many_shared_groups_slow_path(kernel):
    """A tiny hash space makes nearly every (field, value) shared inside a chunk and many
    values collide with opposite signs: more shared groups than U columns exercises
    the exact overflow path; collisions exercise the ±1 one-hot."""
    space = FeatureSpace(3, 0, 32, 1 << 9)
    wc, wg, _, _, _ = _seq_case(space, 640, 2, 320, L.RULE_HINGE, seed=4)
    assert torch.allclose(wg, wc, atol=5e-4, rtol=2e-3), (wg - wc).abs().max()


@gpu
@pytest.mark.parametrize("kernel", ["seq"], indirect=True)  # v3: test_scan3.py
def test_gpu_learner_raw_rounds_track_cpu(kernel):
    """Several Synchronous rounds through SVM.fit(RawBatch): GPU and CPU models agree."""
    from omldm_amd.models.linear import SVM
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import Synchronous

    space = FeatureSpace(13, 0, 26, 1 << 18)
    res = {}
    for dev in ("cpu", "cuda"):
        lrn = SVM({"variant": "PA-I", "C": 1.0}, space, dev)
        proto = Synchronous(Comm(), lrn, {"virtualSpokes": 16})
        for k in range(6):
            b = synth_raw(space, 16 * 700, start=k * 16 * 700, seed=25)
            proto.round(b.to(dev) if dev == "cuda" else b)
        res[dev] = (lrn.w.cpu(), lrn.running_totals())
    assert torch.allclose(res["cuda"][0], res["cpu"][0], atol=1e-3, rtol=1e-2)
    assert res["cuda"][1]["fitted"] == res["cpu"][1]["fitted"] == 6 * 16 * 700
    assert res["cuda"][1]["overflow"] == 0  # no producer barrier timed out
    assert abs(res["cuda"][1]["mistakes"] - res["cpu"][1]["mistakes"]) <= 0.002 * 6 * 16 * 700


def _blocked_gram_scan(w, batch, space, R, S, C=1.0, chunk=64, bias=True):
    """NumPy model of linear_seq.hip's algorithm (PA-I): per spoke, chunks of 64 rows;
    round-start margins p = X·w_chunk0, G = X·Xᵀ over the hashed sparse rows, the scalar
    recurrence m_t = p_t + Σ_{s<t} c_s·G[t][s], then the rank-64 update."""
    dim = space.dim
    cat = hash_raw(batch.tok, space).numpy()
    num = batch.num.double().numpy()
    y = batch.y.double().numpy()
    B = batch.B
    out = w.double().numpy().copy()
    acc, n_act = np.zeros(dim), 0
    for s in range(S):
        a, b = min(s * R, B), min(s * R + R, B)
        if a >= b:
            continue
        n_act += 1
        W = w.double().numpy().copy()
        for c0 in range(a, b, chunk):
            rows = range(c0, min(b, c0 + chunk))
            X = np.zeros((len(rows), dim))
            n2 = np.zeros(len(rows))
            for i, t in enumerate(rows):
                X[i, :space.dn] = num[t]
                n2[i] = (num[t] ** 2).sum()
                for j in range(space.dc):
                    cc = int(cat[t, j])
                    if cc != -1:
                        X[i, cc & 0x7FFFFFFF] += -1.0 if cc < 0 else 1.0
                        n2[i] += 1.0
                if bias:
                    X[i, dim - 1] = 1.0
                    n2[i] += 1.0
            p = X @ W
            G = X @ X.T
            cvec = np.zeros(len(rows))
            for i, t in enumerate(rows):
                m = p[i] + (cvec[:i] * G[i, :i]).sum()
                loss = max(0.0, 1 - y[t] * m)
                cvec[i] = min(C, loss / n2[i]) * y[t]
            W += X.T @ cvec
        acc += W - w.double().numpy()
    return out + acc / n_act


def test_blocked_gram_scan_algorithm_matches_oracle():
    """The GPU kernel's math (blocked-exact scan with cross-field slot collisions in a
    small hash space) equals the per-example oracle."""
    space = FeatureSpace(5, 0, 8, 1 << 8)  # tiny: many collisions, also across fields
    batch = synth_raw(space, 300, seed=9, missing=0.05)
    w = torch.randn(space.dim, generator=torch.Generator().manual_seed(2)) * 0.01
    wc, dacc = w.clone(), torch.zeros(space.dim + 2)
    rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=0.7)
    L.linear_seq_round(wc, batch, 150, 2, dacc, rule, 0.5)
    L.linear_apply(wc, None, dacc)
    ref = _blocked_gram_scan(w, batch, space, 150, 2, C=0.7)
    assert np.allclose(wc.double().numpy(), ref, atol=1e-5, rtol=1e-4)


@gpu
def test_gpu_engine_field_aware_batches_take_the_scan_round():
    """The engine's field-aware hashed batches (slots already hashed) train through the
    v3 table scan on the GPU and agree with the CPU's exact sequential virtual spokes."""
    from omldm_amd.api.batch import HashedBatch
    from omldm_amd.io.synthetic import synth_batch
    from omldm_amd.models.linear import SVM
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import Synchronous

    space = FeatureSpace(13, 0, 26, 1 << 18, field_aware=True)
    res = {}
    for dev in ("cpu", "cuda"):
        lrn = SVM({"variant": "PA-I", "C": 1.0}, space, dev)
        assert dev == "cpu" or lrn._slots_scan_eligible(synth_batch(space, 64).to(dev))
        proto = Synchronous(Comm(), lrn, {"virtualSpokes": 16})
        for k in range(4):
            b = synth_batch(space, 16 * 500, start=k * 16 * 500, seed=25)
            assert type(b) is HashedBatch and b.cat_span > 0
            proto.round(b.to(dev) if dev == "cuda" else b)
        res[dev] = (lrn.w.cpu(), lrn.running_totals())
    assert torch.allclose(res["cuda"][0], res["cpu"][0], atol=1e-3, rtol=1e-2), \
        (res["cuda"][0] - res["cpu"][0]).abs().max()
    assert res["cuda"][1]["fitted"] == res["cpu"][1]["fitted"] == 4 * 16 * 500
