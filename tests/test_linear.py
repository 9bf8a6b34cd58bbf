"""Linear learners: pure-Python golden ↔ C++ CPU path ↔ HIP kernel (gpu-marked)."""
import math

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.io.synthetic import synth_batch, TASK_BINARY, TASK_REGRESSION
from omldm_amd.ops import linear as L


def python_round(w, batch, R, S, rule: L.LinearRule, inv_p=1.0):
    """Literal per-example reference of one round (SURVEY App. D rules), fp64 host."""
    dim = w.shape[0]
    num, cat, y = batch.num.double().numpy(), batch.cat.numpy(), batch.y.double().numpy()
    B = y.shape[0]
    dacc = np.zeros(dim + 2)
    stats = np.zeros((S, 6))
    for s in range(S):
        a, b = min(s * R, B), min(s * R + R, B)
        if a >= b:
            stats[s, 4] = 1
            continue
        delta = {}
        sigma = 1.0
        for t in range(a, b):
            yt = y[t]
            if math.isnan(yt):
                continue
            feats = [(j, num[t, j]) for j in range(num.shape[1]) if j < dim]
            for c in cat[t]:
                if c == -1:
                    continue
                idx = int(c) & 0x7FFFFFFF
                if idx < dim:
                    feats.append((idx, -1.0 if c < 0 else 1.0))
            if rule.bias:
                feats.append((dim - 1, 1.0))
            pm = sum(v * (float(w[i]) + delta.get(i, 0.0)) for i, v in feats)
            n2 = sum(v * v for _, v in feats)
            m = sigma * pm

            def tau(loss):
                if loss <= 0 or n2 <= 0:
                    return 0.0
                if rule.variant == L.PA:
                    return loss / n2
                if rule.variant == L.PA1:
                    return min(rule.C, loss / n2)
                return loss / (n2 + 0.5 / rule.C)

            if rule.rule == L.RULE_PEGASOS:  # η = 1/(λT), w ← (1 − 1/T)w + η·y·x·[ym < 1]
                T = rule.tbase + (t - a)
                loss = max(0.0, 1 - yt * m)
                c = yt / (rule.lam * T) if yt * m < 1 else 0.0
                stats[s, 2] += yt * m <= 0
                shrink = (T - 1) / T
            elif rule.rule == L.RULE_HINGE:
                loss = max(0.0, 1 - yt * m)
                c = tau(loss) * yt
                stats[s, 2] += yt * m <= 0
                shrink = 1 - rule.lam
            elif rule.rule == L.RULE_EPS:
                err = yt - m
                loss = max(0.0, abs(err) - rule.eps)
                c = tau(loss) * (1 if err >= 0 else -1)
                stats[s, 3] += err * err
                shrink = 1 - rule.lam
            else:
                z = yt * m
                loss = math.log1p(math.exp(-z)) if z > 0 else -z + math.log1p(math.exp(z))
                c = rule.lr * yt / (1 + math.exp(z))
                stats[s, 2] += z <= 0
                shrink = 1 - rule.lr * rule.lam
            stats[s, 0] += loss
            stats[s, 1] += 1
            sigma *= shrink
            if c:
                for i, v in feats:
                    delta[i] = delta.get(i, 0.0) + c / sigma * v
        stats[s, 4] = sigma
        for i, v in delta.items():
            dacc[i] += v * sigma * inv_p
        dacc[dim] += sigma * inv_p
        dacc[dim + 1] += inv_p
    return dacc, stats


RULES = [
    L.LinearRule(L.RULE_HINGE, L.PA1, C=0.5),
    L.LinearRule(L.RULE_HINGE, L.PA, bias=False),
    L.LinearRule(L.RULE_HINGE, L.PA2, C=2.0, lam=1e-3),
    L.LinearRule(L.RULE_EPS, L.PA1, C=1.0, eps=0.05),
    L.LinearRule(L.RULE_LOGISTIC, lr=0.05, lam=1e-4),
    L.LinearRule(L.RULE_PEGASOS, lam=0.05, tbase=40.0),
]


@pytest.mark.parametrize("rule", RULES)
def test_cpu_round_matches_python(rule):
    sp = FeatureSpace(5, 0, 7, 1 << 10)
    task = TASK_REGRESSION if rule.rule == L.RULE_EPS else TASK_BINARY
    b = synth_batch(sp, 300, task=task, seed=3)
    b.y[17] = float("nan")  # skipped row
    w = torch.randn(sp.dim) * 0.1
    R, S = 37, 9  # last spokes idle
    dacc = torch.zeros(sp.dim + 2)
    stats = torch.zeros(S, 6)
    L.linear_round(w, b, R, S, dacc, stats, rule, 1.0)
    ref_d, ref_s = python_round(w, b, R, S, rule)
    np.testing.assert_allclose(dacc.numpy(), ref_d, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(stats.numpy()[:, [1, 2, 4]], ref_s[:, [1, 2, 4]], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(stats.numpy()[:, 0], ref_s[:, 0], rtol=1e-3, atol=1e-3)


def test_apply_averages_active_workers():
    dim = 16
    w = torch.arange(dim, dtype=torch.float32)
    d = torch.zeros(dim + 2)
    d[:dim] = 2.0
    d[dim] = 1.5   # Σσ/P over 2 active workers (σ = 1, 0.5)
    d[dim + 1] = 2.0
    L.linear_apply(w, None, d)
    np.testing.assert_allclose(w.numpy(), (1.5 * np.arange(dim) + 2.0) / 2.0, rtol=1e-6)
    assert float(d.abs().sum()) == 0.0


def test_apply_no_workers_is_identity():
    w = torch.randn(64)
    w0 = w.clone()
    d = torch.zeros(66)
    L.linear_apply(w, None, d)
    assert torch.equal(w, w0)


def test_predict_matches_dense():
    sp = FeatureSpace(4, 0, 6, 1 << 9)
    b = synth_batch(sp, 50, seed=5)
    W = torch.randn(3, sp.dim)
    out = L.linear_predict(W, b)
    X = b.dense(sp.dim)
    X[:, sp.dim - 1] = 1.0  # intercept slot
    np.testing.assert_allclose(out.numpy(), (X @ W.T).numpy(), rtol=1e-5, atol=1e-5)


def test_single_spoke_learns():
    sp = FeatureSpace(13, 0, 26, 1 << 16)
    w = torch.zeros(sp.dim)
    d = torch.zeros(sp.dim + 2)
    test = synth_batch(sp, 3000, start=10**8)
    for r in range(6):
        L.linear_round(w, synth_batch(sp, 4096, start=r * 4096), 4096, 1, d, None,
                       L.LinearRule(), 1.0)
        L.linear_apply(w, None, d)
    acc = float(((L.linear_predict(w, test) >= 0).float() * 2 - 1 == test.y).float().mean())
    assert acc > 0.7


# ------------------------------------------------------------------ HIP kernels
@pytest.mark.gpu
@pytest.mark.parametrize("rule", RULES)
@pytest.mark.parametrize("shape", [(13, 26), (40, 50), (100, 120)])
def test_hip_round_matches_cpu(cuda, rule, shape):
    dn, dc = shape
    sp = FeatureSpace(dn, 0, dc, 1 << 14)
    task = TASK_REGRESSION if rule.rule == L.RULE_EPS else TASK_BINARY
    b = synth_batch(sp, 2000, task=task, seed=11)
    b.y[5] = float("nan")
    w = torch.randn(sp.dim) * 0.05
    R, S = 70, 31
    d_cpu = torch.zeros(sp.dim + 2)
    s_cpu = torch.zeros(S, 6)
    L.linear_round(w, b, R, S, d_cpu, s_cpu, rule, 1.0)
    d_gpu = torch.zeros(sp.dim + 2, device=cuda)
    s_gpu = torch.zeros(S, 6, device=cuda)
    cum = torch.zeros(8, dtype=torch.float64, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), R, S, d_gpu, s_gpu, rule, 1.0, log2cap=13, cum=cum)
    torch.cuda.synchronize()
    s_g = s_gpu.cpu()
    assert float(s_g[:, 5].sum()) == 0.0  # no LDS table overflow
    np.testing.assert_allclose(s_g[:, 1].numpy(), s_cpu[:, 1].numpy())
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(cum.cpu()[1].item(), s_cpu[:, 1].sum().item())


@pytest.mark.gpu
def test_hip_apply_and_predict(cuda):
    sp = FeatureSpace(13, 0, 26, (1 << 16) + 3)  # odd dim exercises the scalar tail
    w = torch.randn(sp.dim)
    d = torch.randn(sp.dim + 2)
    d[sp.dim] = 0.7
    d[sp.dim + 1] = 1.3
    wg, dg = w.to(cuda), d.to(cuda)
    w16 = torch.empty(sp.dim, dtype=torch.bfloat16, device=cuda)
    L.linear_apply(w, None, d)
    L.linear_apply(wg, w16, dg)
    torch.cuda.synchronize()
    np.testing.assert_allclose(wg.cpu().numpy(), w.numpy(), rtol=1e-6, atol=1e-6)
    assert float(dg[: sp.dim].abs().sum().item()) == 0.0  # counters are overwritten per round
    np.testing.assert_allclose(w16.float().cpu().numpy(), w.numpy(), rtol=1e-2, atol=1e-2)
    b = synth_batch(sp, 777, seed=9)
    W = torch.randn(4, sp.dim)
    ref = L.linear_predict(W, b)
    out = L.linear_predict(W.to(cuda), b.to(cuda))
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    out16 = L.linear_predict(W.to(cuda).bfloat16(), b.to(cuda))
    ref16 = L.linear_predict(W.bfloat16().float(), b)
    np.testing.assert_allclose(out16.cpu().numpy(), ref16.numpy(), rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_hip_bf16_model_round(cuda):
    sp = FeatureSpace(13, 0, 26, 1 << 14)
    b = synth_batch(sp, 4096, seed=2)
    w = (torch.randn(sp.dim) * 0.05).bfloat16()
    rule = L.LinearRule()
    d_cpu = torch.zeros(sp.dim + 2)
    L.linear_round(w, b, 64, 64, d_cpu, None, rule, 1.0)
    d_gpu = torch.zeros(sp.dim + 2, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), 64, 64, d_gpu, None, rule, 1.0, log2cap=12)
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("log2cap,R", [(11, 32), (12, 64)])
def test_hip_round_bucketed_table_large_dim(cuda, log2cap, R):
    """2^20-dim hashing: 256 key buckets, 8-16 slots each, overflow area; exact vs CPU."""
    sp = FeatureSpace(13, 0, 26, 1 << 20)
    S = 96
    b = synth_batch(sp, S * R, seed=7)
    w = (torch.randn(sp.dim) * 0.01)
    rule = L.LinearRule()
    d_cpu = torch.zeros(sp.dim + 2)
    s_cpu = torch.zeros(S, 6)
    L.linear_round(w, b, R, S, d_cpu, s_cpu, rule, 1.0)
    d_gpu = torch.zeros(sp.dim + 2, device=cuda)
    s_gpu = torch.zeros(S, 6, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), R, S, d_gpu, s_gpu, rule, 1.0, log2cap=log2cap)
    assert float(s_gpu[:, 5].sum()) == 0.0
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
def test_hip_round_table_overflow_spills_exactly(cuda):
    """~3000 distinct keys into 1024 + 64 LDS slots: the rest go to the HBM spill, the
    round equals the CPU round and nothing is counted as dropped."""
    sp = FeatureSpace(13, 0, 26, 1 << 20)
    S, R = 8, 128
    b = synth_batch(sp, S * R, seed=8)
    d = torch.zeros(sp.dim + 2, device=cuda)
    st = torch.zeros(S, 6, device=cuda)
    L.linear_round(torch.zeros(sp.dim, device=cuda), b.to(cuda), R, S, d, st, L.LinearRule(), 1.0,
                   log2cap=10)
    d_cpu = torch.zeros(sp.dim + 2)
    L.linear_round(torch.zeros(sp.dim), b, R, S, d_cpu, None, L.LinearRule(), 1.0)
    torch.cuda.synchronize()
    assert float(st[:, 5].sum()) == 0
    np.testing.assert_allclose(d.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 4, 7])
def test_hip_round_reduce_parts(cuda, parts):
    """Reduce issued as `parts` key-range launches (pipelined sync): the slices reported
    after each launch tile [0, dim + 2), match the kernel library's bounds, and the
    accumulator equals the CPU round; a slice is final when it is reported."""
    sp = FeatureSpace(13, 0, 26, 1 << 20)
    S, R = 96, 32
    b = synth_batch(sp, S * R, seed=9)
    w = torch.randn(sp.dim) * 0.01
    rule = L.LinearRule()
    d_cpu = torch.zeros(sp.dim + 2)
    L.linear_round(w, b, R, S, d_cpu, None, rule, 1.0)
    d_gpu = torch.zeros(sp.dim + 2, device=cuda)
    seen, snaps = [], []

    def on_part(k, lo, hi):
        seen.append((k, lo, hi))
        snaps.append(d_gpu[lo:hi].clone())  # stream-ordered: taken right after part k

    L.linear_round(w.to(cuda), b.to(cuda), R, S, d_gpu, None, rule, 1.0, log2cap=11,
                   parts=parts, on_part=on_part)
    torch.cuda.synchronize()
    assert [k for k, _, _ in seen] == list(range(parts))
    assert seen[0][1] == 0 and seen[-1][2] == sp.dim + 2
    assert all(seen[k][2] == seen[k + 1][1] for k in range(parts - 1))
    assert [(lo, hi) for _, lo, hi in seen] == [L.part_bounds(sp.dim, k, parts, cuda=False)
                                                for k in range(parts)]
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)
    final = torch.cat(snaps).cpu()
    np.testing.assert_allclose(final.numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("rule", [L.LinearRule(), L.LinearRule(rule=L.RULE_LOGISTIC, variant=0)])
def test_hip_round_int8_labels(cuda, rule):
    """Compact classification wire: ±1 labels as int8 give the same round as fp32 labels
    (and as the CPU round, which widens them)."""
    sp = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
    S, R = 64, 16
    b = synth_batch(sp, S * R, seed=11)
    b8 = HashedBatch(b.num, b.cat, b.y.to(torch.int8), cat_span=b.cat_span)
    assert torch.equal(b8.y.float(), b.y)
    w = torch.randn(sp.dim) * 0.01
    d32 = torch.zeros(sp.dim + 2, device=cuda)
    d8 = torch.zeros(sp.dim + 2, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), R, S, d32, None, rule, 1.0)
    L.linear_round(w.to(cuda), b8.to(cuda), R, S, d8, None, rule, 1.0)
    dc = torch.zeros(sp.dim + 2)
    L.linear_round(w, b8, R, S, dc, None, rule, 1.0)
    torch.cuda.synchronize()
    np.testing.assert_allclose(d8.cpu().numpy(), d32.cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d8.cpu().numpy(), dc.numpy(), rtol=2e-3, atol=2e-4)


RD_TABLE = 16  # ablate bit: force the LDS-hash-table round kernel


@pytest.mark.gpu
@pytest.mark.parametrize("rule", RULES)
@pytest.mark.parametrize("R,S", [(16, 64), (13, 40), (8, 50), (5, 33), (1, 70)])
@pytest.mark.parametrize("model_dtype", [torch.float32, torch.bfloat16])
def test_hip_register_dedup_round_matches_table_kernel_and_cpu(cuda, rule, R, S, model_dtype):
    """Field-aware compact wire, ≤ 16 rows per spoke: the register-dedup round kernel
    (deltas in registers, no LDS hash table) gives the LDS-table kernel's round and the
    CPU round. Stats (loss, n, mistakes, sq_err, σ) agree too; the last spokes are idle."""
    sp = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
    task = TASK_REGRESSION if rule.rule == L.RULE_EPS else TASK_BINARY
    B = S * R - R // 2 - 1  # ragged last spoke
    b = synth_batch(sp, B, seed=R * 131 + S, task=task)
    w = (torch.randn(sp.dim) * 0.02).to(model_dtype).float()
    out = {}
    for name, ablate in (("rd", 0), ("table", RD_TABLE)):
        d = torch.zeros(sp.dim + 2, device=cuda)
        st = torch.zeros(S, 6, device=cuda)
        L.linear_round(w.to(cuda).to(model_dtype), b.to(cuda), R, S, d, st, rule, 1.0,
                       ablate=ablate)
        out[name] = (d.cpu(), st.cpu())
    d_cpu = torch.zeros(sp.dim + 2)
    s_cpu = torch.zeros(S, 6)
    L.linear_round(w, b, R, S, d_cpu, s_cpu, rule, 1.0)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out["rd"][0].numpy(), out["table"][0].numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["rd"][1][:, :5].numpy(), out["table"][1][:, :5].numpy(),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["rd"][0].numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(out["rd"][1][:, 1].numpy(), s_cpu[:, 1].numpy())


def test_pegasos_variant_learner():
    """SVM with variant Pegasos: the per-spoke step clock advances by R per round, is
    checkpointed, and the model separates the synthetic stream."""
    from omldm_amd.models import make_learner
    from omldm_amd.models.base import RoundContext

    sp = FeatureSpace(13, 0, 26, 1 << 14)
    lr = make_learner("SVM", {"variant": "Pegasos", "lambda": 1e-3}, sp, "cpu")
    assert lr.rule.rule == L.RULE_PEGASOS and lr.hyper_parameters()["variant"] == "Pegasos"
    for r in range(6):
        b = synth_batch(sp, 2048, start=r * 2048, seed=4)
        lr.fit(b, RoundContext(spokes=16))
    assert lr.steps == 6 * 128
    sd = lr.state_dict()
    lr2 = make_learner("SVM", {"variant": "Pegasos", "lambda": 1e-3}, sp, "cpu")
    lr2.load_state_dict(sd)
    assert lr2.steps == lr.steps and torch.equal(lr2.w, lr.w)
    test = synth_batch(sp, 4096, start=10**6, seed=4)
    acc = float((lr.predict(test) == test.y).float().mean())
    assert acc > 0.7
    with pytest.raises(ValueError):
        make_learner("SVM", {"variant": "Pegasos", "lambda": 0}, sp, "cpu")
