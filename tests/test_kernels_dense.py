"""HIP kernels of the preprocessors and dense/multi-class learners vs fp32/fp64 PyTorch
references (gpu-marked), plus CPU-path math checks."""
import json
import uuid

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch, synth_json_records
from omldm_amd.models import make_learner
from omldm_amd.models.base import RoundContext
from omldm_amd.models.preprocess import MinMaxScaler, PolynomialFeatures, StandardScaler
from omldm_amd.ops import dense as D
from omldm_amd.ops import preprocess as P

SP = FeatureSpace(13, 0, 26, 1 << 14)


def test_cpu_scalers_match_numpy():
    rng = np.random.default_rng(0)
    xs = [rng.normal(3.0, 2.0, size=(n, 5)).astype(np.float32) for n in (100, 7, 300)]
    sc, mm = StandardScaler(), MinMaxScaler()
    for x in xs:
        t = torch.from_numpy(x)
        sc.fit_transform(t, True)
        mm.fit_transform(t, True)
    allx = np.concatenate(xs)
    np.testing.assert_allclose(sc.mean.numpy(), allx.mean(0), rtol=1e-5)
    np.testing.assert_allclose((sc.m2 / sc.count).numpy(), allx.var(0), rtol=1e-4)
    np.testing.assert_allclose(mm.lo.numpy(), allx.min(0))
    np.testing.assert_allclose(mm.hi.numpy(), allx.max(0))


def test_poly_expansion():
    x = torch.tensor([[1.0, 2.0, 3.0]])
    pf = PolynomialFeatures({"degree": 2})
    out = pf.fit_transform(x, True)
    assert pf.out_dim(3) == 9
    np.testing.assert_allclose(out.numpy()[0], [1, 2, 3, 1, 2, 3, 4, 6, 9])


def test_gram_cpu_and_orr_solution():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(500, 4)).astype(np.float32)
    wtrue = np.array([1.0, -2.0, 0.5, 3.0], np.float32)
    y = X @ wtrue + 0.7
    L = make_learner("ORR", {"lambda": 1e-6, "_inDim": 4}, SP, "cpu")
    from omldm_amd.api.batch import HashedBatch
    b = HashedBatch(torch.from_numpy(X), torch.full((500, 26), -1, dtype=torch.int32),
                    torch.from_numpy(y))
    L.fit(b, RoundContext())
    w = L.weights().numpy()
    np.testing.assert_allclose(w[:4], wtrue, atol=1e-3)
    assert abs(w[4] - 0.7) < 1e-3


@pytest.mark.gpu
def test_hip_colstats_scale_poly(cuda):
    torch.manual_seed(0)
    x = torch.randn(5000, 37) * 3 + 5
    for shift_rows in (1234, 3766):
        pass
    mean = torch.zeros(37, dtype=torch.float64)
    m2 = torch.zeros_like(mean)
    c = 0.0
    mg, m2g = mean.to(cuda), m2.to(cuda)
    cg = 0.0
    lo = torch.full((37,), float("inf"), device=cuda)
    hi = torch.full((37,), float("-inf"), device=cuda)
    for part in (x[:1234], x[1234:]):
        c = P.welford_update(part, c, mean, m2)
        cg = P.welford_update(part.to(cuda), cg, mg, m2g)
        P.minmax_update(part.to(cuda), lo, hi)
    np.testing.assert_allclose(mg.cpu().numpy(), mean.numpy(), rtol=1e-5)
    np.testing.assert_allclose(m2g.cpu().numpy(), m2.numpy(), rtol=1e-4)
    np.testing.assert_allclose(lo.cpu().numpy(), x.min(0).values.numpy())
    np.testing.assert_allclose(hi.cpu().numpy(), x.max(0).values.numpy())
    xs = x[:100]
    np.testing.assert_allclose(P.standardize(xs.to(cuda), mg, m2g, cg).cpu().numpy(),
                               P.standardize(xs, mean, m2, c).numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(P.minmax_scale(xs.to(cuda), lo, hi).cpu().numpy(),
                               P.minmax_scale(xs, lo.cpu(), hi.cpu()).numpy(), atol=1e-6)
    pf = PolynomialFeatures({"degree": 3})
    idx = pf._index(6, "cpu")
    np.testing.assert_allclose(P.poly_expand(xs[:, :6].to(cuda), idx.to(cuda)).cpu().numpy(),
                               P.poly_expand(xs[:, :6], idx).numpy(), rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,d", [(1000, 13), (4097, 104), (333, 30), (70001, 104), (9000, 61)])
def test_hip_gram_mfma_vs_fp64(cuda, B, d):
    torch.manual_seed(B)
    x = torch.randn(B, d)
    y = torch.randn(B)
    y[::7] = float("nan")
    ld = ((d + 2 + 31) // 32) * 32
    G = torch.zeros(ld, ld, device=cuda)
    # the running total starts past 2^31: an fp32 total would drop these increments
    base = float(2 ** 31 + 3)
    cnt = torch.full((1,), base, dtype=torch.float64, device=cuda)
    D.gram_update(x.to(cuda), y.to(cuda), G, cnt=cnt)
    ok = ~torch.isnan(y)
    assert float(cnt) - base == float(ok.sum())  # fitted-row count from the (d, d) entry
    z = torch.cat([x[ok], torch.ones(int(ok.sum()), 1), y[ok].unsqueeze(1)], 1).double()
    ref = (z.T @ z).numpy()
    got = G.cpu().double().numpy()[: d + 2, : d + 2]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-2)
    assert float(G[d + 2:, :].abs().sum()) == 0.0


@pytest.mark.parametrize("name,task,hyper", [("ORR", 1, {}), ("K-means", 0, {"k": 3}),
                                              ("NN", 0, {}), ("SVM", 1, {}),
                                              ("MultiClassPA", 2, {"nClasses": 3})])
def test_fitted_count_keeps_counting_past_2_31(name, task, hyper, device="cpu"):
    """Running totals are fp64: a count already past 2^31 still grows by every row
    (fp32 would round increments of < 2^7 away)."""
    L = make_learner(name, dict(hyper, _inDim=SP.dn), SP, device)
    assert L.cum.dtype == torch.float64
    base = 2 ** 31 + 5
    L.cum[1] = base
    b = synth_batch(SP, 96, task=task, n_classes=3).to(device)
    L.fit(b, RoundContext(spokes=4))
    assert L.running_totals()["fitted"] == base + 96


@pytest.mark.gpu
@pytest.mark.parametrize("name,task,hyper", [("ORR", 1, {}), ("K-means", 0, {"k": 3}),
                                              ("NN", 0, {}), ("SVM", 1, {}),
                                              ("MultiClassPA", 2, {"nClasses": 3}),
                                              ("HT", 2, {"nClasses": 3})])
def test_hip_fitted_count_keeps_counting_past_2_31(cuda, name, task, hyper):
    """The kernels add their per-round counts into the fp64 running totals."""
    test_fitted_count_keeps_counting_past_2_31(name, task, hyper, device=cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("d,k", [(13, 5), (30, 7), (40, 16), (130, 3)])
def test_hip_kmeans_assign(cuda, d, k):
    """Scalar kernel (k < 32): row in registers for d ≤ 64, re-read per centroid beyond."""
    torch.manual_seed(3)
    x = torch.randn(3000, d)
    cent = torch.randn(k, d)
    y = torch.zeros(3000)
    s, n, inert = torch.zeros(k, d), torch.zeros(k), torch.zeros(1)
    a_ref = D.kmeans_assign(x, y, cent, s, n, inert, want_assign=True)
    sg, ng, ig = torch.zeros(k, d, device=cuda), torch.zeros(k, device=cuda), \
        torch.zeros(1, device=cuda)
    a = D.kmeans_assign(x.to(cuda), y.to(cuda), cent.to(cuda), sg, ng, ig, want_assign=True)
    assert torch.equal(a.cpu().long(), a_ref.long())
    np.testing.assert_allclose(sg.cpu().numpy(), s.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(ng.cpu().numpy(), n.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("B,d,k", [(3000, 13, 32), (5001, 8, 50), (20000, 64, 256),
                                   (4097, 100, 40), (777, 31, 97), (2000, 20, 33),
                                   (2000, 40, 64)])
def test_hip_kmeans_assign_mfma(cuda, B, d, k):
    """k ≥ 32: matrix-core distances. The chosen centroid is a nearest one (fp64 distances,
    up to rounding ties), and sums / counts / inertia follow the kernel's own assignment."""
    torch.manual_seed(B)
    x = torch.randn(B, d)
    cent = torch.randn(k, d)
    y = torch.zeros(B)
    y[::7] = float("nan")  # forecast rows: assigned, not summed
    sg, ng, ig = torch.zeros(k, d, device=cuda), torch.zeros(k, device=cuda), \
        torch.zeros(1, device=cuda)
    a = D.kmeans_assign(x.to(cuda), y.to(cuda), cent.to(cuda), sg, ng, ig,
                        want_assign=True).cpu().long()
    dist = torch.cdist(x.double(), cent.double()) ** 2
    dmin = dist.min(1).values
    chosen = dist.gather(1, a[:, None])[:, 0]
    assert torch.all(chosen - dmin <= 1e-4 * (1 + dmin)), (chosen - dmin).max()
    tr = ~torch.isnan(y)
    s = torch.zeros(k, d, dtype=torch.float64).index_add_(0, a[tr], x[tr].double())
    n = torch.bincount(a[tr], minlength=k).double()
    np.testing.assert_allclose(sg.cpu().double().numpy(), s.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(ng.cpu().double().numpy(), n.numpy())
    np.testing.assert_allclose(ig.cpu().item(), chosen[tr].sum().item(), rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("nclass,R,S", [(4, 50, 40), (3, 16, 96), (2, 8, 64), (7, 16, 32),
                                         (12, 8, 32)])
def test_hip_multiclass_round_vs_cpu(cuda, nclass, R, S):
    b = synth_batch(SP, R * S, task=2, n_classes=nclass, seed=5)
    W = torch.randn(nclass, SP.dim) * 0.01
    st, dacc = torch.zeros(8), torch.zeros(nclass, SP.dim)
    D.multiclass_round(W, b, R, S, nclass, 1, 1.0, True, dacc, st)
    stg, daccg = torch.zeros(8, device=cuda), torch.zeros(nclass, SP.dim, device=cuda)
    D.multiclass_round(W.to(cuda), b.to(cuda), R, S, nclass, 1, 1.0, True, daccg, stg)
    torch.cuda.synchronize()
    assert float(stg[5]) == 0.0  # no LDS table overflow
    np.testing.assert_allclose(stg.cpu()[[1, 3]].numpy(), st[[1, 3]].numpy())
    np.testing.assert_allclose(stg.cpu()[[0, 2]].numpy(), st[[0, 2]].numpy(), rtol=1e-3)
    np.testing.assert_allclose(daccg.cpu().numpy(), dacc.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("nclass", [2, 4, 6])
def test_hip_multiclass_compact_flush_matches_per_class(cuda, nclass, monkeypatch):
    """The compact (key, K-vector) flush + one-launch reducer == the per-class int2 regions
    reduced one class at a time, at the learners-bench geometry (2^20 dims, 16 rows per
    spoke, split reduce blocks)."""
    from omldm_amd.api.batch import FeatureSpace

    sp = FeatureSpace(13, 0, 26, 1 << 20)
    S, R = 2048, 16
    b = synth_batch(sp, S * R, task=2, n_classes=nclass, seed=8).to(cuda)
    W = (torch.randn(nclass, sp.dim) * 0.01).to(cuda)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("OMLDM_MC_COMPACT", flag)
        st, dacc = torch.zeros(8, device=cuda), torch.zeros(nclass, sp.dim, device=cuda)
        D.multiclass_round(W, b, R, S, nclass, 1, 1.0, True, dacc, st)
        torch.cuda.synchronize()
        out.append((st.cpu(), dacc.cpu()))
    assert torch.equal(out[0][0][[1, 3, 5]], out[1][0][[1, 3, 5]])
    np.testing.assert_allclose(out[0][1].numpy(), out[1][1].numpy(), rtol=1e-5, atol=1e-6)
    assert float(out[0][1].abs().sum()) > 0


@pytest.mark.gpu
def test_hip_multiclass_round_compact_wire(cuda):
    """Field-aware uint16 categoricals, bf16 numericals and int8 class labels read
    directly by the kernel == the CPU mirror on the widened batch."""
    from omldm_amd.api.batch import FeatureSpace, HashedBatch

    sp = FeatureSpace(13, 0, 26, 1 << 18, field_aware=True)
    b = synth_batch(sp, 16 * 64, task=2, n_classes=3, seed=6)
    W = torch.randn(3, sp.dim) * 0.01
    st, dacc = torch.zeros(8), torch.zeros(3, sp.dim)
    D.multiclass_round(W, b, 16, 64, 3, 1, 1.0, True, dacc, st)
    bc = HashedBatch(b.num.to(torch.bfloat16).float(), b.cat, b.y, cat_span=b.cat_span)
    stc, daccc = torch.zeros(8), torch.zeros(3, sp.dim)
    D.multiclass_round(W, bc, 16, 64, 3, 1, 1.0, True, daccc, stc)
    g = HashedBatch(b.num.to(torch.bfloat16), b.cat, b.y.to(torch.int8), cat_span=b.cat_span)
    stg, daccg = torch.zeros(8, device=cuda), torch.zeros(3, sp.dim, device=cuda)
    D.multiclass_round(W.to(cuda), g.to(cuda), 16, 64, 3, 1, 1.0, True, daccg, stg)
    torch.cuda.synchronize()
    np.testing.assert_allclose(stg.cpu()[[1, 3]].numpy(), stc[[1, 3]].numpy())
    np.testing.assert_allclose(daccg.cpu().numpy(), daccc.numpy(), rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("name,task,hyper", [
    ("PA", 0, {}), ("RegressorPA", 1, {}), ("SVM", 0, {"modelDtype": "bf16"}),
    ("LogisticRegression", 0, {}), ("MultiClassPA", 2, {"nClasses": 3}),
    ("ORR", 1, {}), ("K-means", 0, {"k": 3}), ("NN", 0, {}), ("HT", 2, {"nClasses": 3})])
def test_learners_on_gpu(cuda, name, task, hyper):
    L = make_learner(name, hyper, SP, cuda)
    for r in range(3):
        L.fit(synth_batch(SP, 2048, start=r * 2048, task=task, n_classes=3).to(cuda),
              RoundContext(spokes=16))
    t = synth_batch(SP, 512, start=10**6, task=task, n_classes=3).to(cuda)
    loss, score, n = L.evaluate(t)
    assert n == 512 and np.isfinite(float(loss))
    assert L.running_totals()["fitted"] == 3 * 2048


@pytest.mark.gpu
def test_engine_on_gpu(cuda):
    from omldm_amd.engine.job import Job
    from omldm_amd.io.transport import MemoryBroker
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.utils.config import JobConfig

    name = uuid.uuid4().hex
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", f"memory://{name}"]
    cfg = JobConfig.from_args(args + ["--hashDim", str(SP.dim), "--timeout", "200",
                                      "--batchSize", "1000"])
    br = MemoryBroker.named(name)
    for r in synth_json_records(2000, SP):
        br.produce("trainingData", r)
    br.produce("requests", json.dumps({"id": 1, "request": "Create", "learner": {"name": "SVM"},
                                       "preProcessors": [{"name": "StandardScaler"}],
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))
    job = Job(cfg, Comm(), cuda).run()
    assert job.terminated and job.pipes[1].learner.running_totals()["fitted"] > 0
    assert json.loads(br.records("performance")[-1])["statistics"][0]["fitted"] > 0


def _mlp_case(widths, task, B, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = sum(a * b + b for a, b in zip(widths[:-1], widths[1:]))
    w = torch.randn(n, generator=g) * 0.3
    x = torch.randn(B, widths[0], generator=g)
    if task == 0:
        y = x[:, 0] * 0.5 - x[:, 1]
    elif task == 1:
        y = torch.where(x[:, 0] + x[:, 2] > 0, 1.0, -1.0)
    else:
        y = (x[:, :widths[-1]].argmax(1)).float()
    y[5] = float("nan")  # excluded row inside a mini-batch
    return w, x, y


def test_mlp_reference_learns():
    widths = [6, 16, 1]
    w, x, y = _mlp_case(widths, 1, 2048)
    dacc, st = torch.zeros_like(w), torch.zeros(8)
    for _ in range(3):
        D.mlp_round_reference(w, x, y, 256, 8, widths, 1, 0.2, dacc, st)
        w += dacc / st[3]
        dacc.zero_()
        st.zero_()
    out = D.mlp_forward_reference(w, x, widths)[:, 0]
    ok = ~torch.isnan(y)
    assert ((out[ok] >= 0) == (y[ok] > 0)).float().mean() > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("widths,task,act", [([13, 32, 32, 1], 1, 0), ([13, 32, 1], 0, 0),
                                             ([40, 64, 48, 5], 2, 0), ([7, 100, 3], 2, 0),
                                             ([13, 40, 24, 1], 1, 1), ([13, 33, 4], 2, 2),
                                             ([9, 16, 1], 0, 3)])
def test_hip_mlp_round_vs_reference(cuda, widths, task, act):
    B, R, S = 1000, 96, 11
    w, x, y = _mlp_case(widths, task, B, seed=len(widths) + task)
    lr = 0.05
    d_ref, s_ref = torch.zeros_like(w), torch.zeros(8)
    D.mlp_round_reference(w, x, y, R, S, widths, task, lr, d_ref, s_ref, act)
    wd, d_gpu, s_gpu = w.to(cuda), torch.zeros_like(w, device=cuda), torch.zeros(8, device=cuda)
    D.mlp_round(wd, x.to(cuda), y.to(cuda), R, S, widths, task, lr, d_gpu, s_gpu, act)
    torch.cuda.synchronize()
    torch.testing.assert_close(d_gpu.cpu(), d_ref, rtol=2e-3, atol=2e-4)
    torch.testing.assert_close(s_gpu.cpu()[:4], s_ref[:4], rtol=2e-3, atol=1e-2)
    out = D.mlp_forward(wd, x.to(cuda), widths, act)
    torch.testing.assert_close(out.cpu(), D.mlp_forward_reference(w, x, widths, act),
                               rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("widths,task,act", [([13, 32, 32, 1], 1, 0), ([40, 64, 48, 5], 2, 1),
                                             ([13, 64, 64, 1], 0, 0)])
def test_hip_mlp_bf16_matmul_vs_fp32_reference(cuda, widths, task, act):
    """matmulDtype bf16 (v_mfma_f32_32x32x16_bf16 operands, fp32 accumulate) tracks the
    fp32 reference to bf16 rounding; forward output likewise; an exact-integer product
    checks the operand map."""
    B, R, S = 1000, 96, 11
    w, x, y = _mlp_case(widths, task, B, seed=len(widths) + task)
    lr = 0.05
    d_ref, s_ref = torch.zeros_like(w), torch.zeros(8)
    D.mlp_round_reference(w, x, y, R, S, widths, task, lr, d_ref, s_ref, act)
    wd, d_gpu, s_gpu = w.to(cuda), torch.zeros_like(w, device=cuda), torch.zeros(8, device=cuda)
    D.mlp_round(wd, x.to(cuda), y.to(cuda), R, S, widths, task, lr, d_gpu, s_gpu,
                act | D.MLP_BF16)
    torch.cuda.synchronize()
    scale = float(d_ref.abs().max())
    torch.testing.assert_close(d_gpu.cpu(), d_ref, rtol=5e-2, atol=2e-2 * scale)
    out = D.mlp_forward(wd, x.to(cuda), widths, act | D.MLP_BF16).cpu()
    ref = D.mlp_forward_reference(w, x, widths, act)
    torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2 * float(ref.abs().max()))
    # integer-valued operands are exact in bf16: identity activation, one layer
    wi = torch.randint(-3, 4, (13 * 32 + 32 + 32 * 1 + 1,)).float()
    xi = torch.randint(-3, 4, (64, 13)).float()
    o32 = D.mlp_forward(wi.to(cuda), xi.to(cuda), [13, 32, 1], 3).cpu()
    o16 = D.mlp_forward(wi.to(cuda), xi.to(cuda), [13, 32, 1], 3 | D.MLP_BF16).cpu()
    assert torch.equal(o32, o16)


def _ht_data(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 13, generator=g)
    y = ((x[:, 3] > 0.3).long() + (x[:, 7] > 0).long()).float()  # 3 classes, axis-aligned
    return x, y


@pytest.mark.gpu
def test_hip_hoeffding_tree(cuda):
    from omldm_amd.api.batch import HashedBatch

    hyper = {"nClasses": 3, "gracePeriod": 200}
    cpu = make_learner("HT", hyper, SP, "cpu")
    gpu = make_learner("HT", hyper, SP, cuda)
    x, y = _ht_data(150)  # below the grace period: statistics only, no split yet
    b = HashedBatch(x, torch.zeros((150, 0), dtype=torch.int32), y)
    cpu.fit(b, RoundContext())
    gpu.fit(b.to(cuda), RoundContext())
    torch.cuda.synchronize()
    for name in ("cc", "S0", "S1", "S2", "lo", "hi", "since"):
        torch.testing.assert_close(getattr(gpu, name).cpu(), getattr(cpu, name), rtol=1e-5,
                                   atol=1e-4)
    for s in range(1, 30):
        x, y = _ht_data(400, seed=s)
        b = HashedBatch(x, torch.zeros((400, 0), dtype=torch.int32), y)
        cpu.fit(b, RoundContext())
        gpu.fit(b.to(cuda), RoundContext())
    x, y = _ht_data(2000, seed=99)
    b = HashedBatch(x, torch.zeros((2000, 0), dtype=torch.int32), y)
    acc_g = (gpu.predict(b.to(cuda)).cpu() == y).float().mean()
    acc_c = (cpu.predict(b) == y).float().mean()
    assert int(gpu.nnodes.item()) > 1
    assert acc_g > 0.85 and acc_c > 0.85, (acc_g, acc_c)


@pytest.mark.gpu
def test_hip_hoeffding_sorted_update_matches_atomic(cuda):
    """The counting-sort update (one reducer block per (leaf, class)) and the
    wave-aggregated atomic update add the same statistics to a grown tree, with NaN
    labels (forecast rows) skipped."""
    from omldm_amd.api.batch import HashedBatch
    from omldm_amd.ops import dense as D

    hyper = {"nClasses": 3, "gracePeriod": 200}
    L = make_learner("HT", hyper, SP, cuda)
    for s in range(1, 30):
        x, y = _ht_data(400, seed=s)
        L.fit(HashedBatch(x, torch.zeros((400, 0), dtype=torch.int32), y).to(cuda),
              RoundContext())
    assert int(L.nnodes.item()) > 1
    x, y = _ht_data(5000, seed=77)
    y[::7] = float("nan")
    xs, ys = x.to(cuda), y.to(cuda)
    base = [t.clone() for t in L._tree()]
    outs = []
    for sort in (True, False):
        tree = [t.clone() for t in base]
        nfit = torch.zeros(1, dtype=torch.float64, device=cuda)
        D.ht_update(xs, ys, 3, L.depth, tree, nfit, N=L.N, sort=sort)
        torch.cuda.synchronize()
        outs.append((tree, float(nfit)))
    (ts, ns), (ta, na) = outs
    assert ns == na == float((~torch.isnan(y)).sum())
    for a, b in zip(ts, ta):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_multiclass_learner_shadow_tracks_prototypes(cuda, dtype):
    """The key-major gather shadow follows W through apply and state loads."""
    L = make_learner("MultiClassPA", {"nClasses": 3, "modelDtype": dtype}, SP, cuda)
    for r in range(3):
        L.fit(synth_batch(SP, 4096, start=r * 4096, task=2, n_classes=3).to(cuda),
              RoundContext(spokes=64))
    tol = 0 if dtype == "fp32" else 1e-2
    torch.testing.assert_close(L.Wt[:, :3].float(), L.W.t(), rtol=tol, atol=tol * 1e-2)
    assert float(L.Wt[:, 3:].abs().sum()) == 0.0
    v = torch.randn_like(L.state_vector())
    L.load_state_vector(v)
    torch.testing.assert_close(L.Wt[:, :3].float(), L.W.t(), rtol=tol, atol=tol * 1e-2)


@pytest.mark.gpu
def test_kmeans_learner_gpu_matches_cpu(cuda):
    """Fused GPU centroid apply == the CPU learner's torch update (same seeding)."""
    from omldm_amd.api.batch import HashedBatch

    cpu = make_learner("K-means", {"k": 5}, SP, "cpu")
    gpu = make_learner("K-means", {"k": 5}, SP, cuda)
    for r in range(4):
        torch.manual_seed(r)
        x = torch.randn(3000, 13) + (r % 2)
        y = torch.zeros(3000)
        y[::9] = float("nan")  # forecast rows are not trained on
        b = HashedBatch(x, torch.zeros((3000, 0), dtype=torch.int32), y)
        cpu.fit(b, RoundContext())
        gpu.fit(b.to(cuda), RoundContext())
    torch.cuda.synchronize()
    torch.testing.assert_close(gpu.state.cpu(), cpu.state, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gpu.cum.cpu()[:2], cpu.cum[:2], rtol=1e-4, atol=1e-2)


def _poly_pairs(d):
    from omldm_amd.models.preprocess import PolynomialFeatures

    return PolynomialFeatures({"degree": 2}).pair_index(d, "cpu")


def test_orr_pipeline_fuses_polynomial_map_on_cpu():
    """Request → PolynomialFeatures(2) → ORR: training batches reach ORR unexpanded
    (PolyBatch) and its Gram equals the Gram of the expanded batch."""
    from omldm_amd.api.batch import PolyBatch
    from omldm_amd.api.schemas import Request
    from omldm_amd.engine.pipeline import Pipeline
    from omldm_amd.parallel.comm import Comm

    req = Request.from_json({"id": 1, "request": "Create", "learner": {"name": "ORR"},
                             "preProcessors": [{"name": "PolynomialFeatures",
                                                "hyperParameters": {"degree": 2}}],
                             "trainingConfiguration": {"protocol": "Synchronous"}})
    pipe = Pipeline(req, SP, Comm(), "cpu", 1, 1)
    b = synth_batch(SP, 300, task=1)
    assert isinstance(pipe._pre(b, True), PolyBatch)
    pipe.train(b)
    ref = make_learner("ORR", {"_inDim": pipe.learner.d}, SP, "cpu")
    ref.fit(pipe.preprocessors[0](b, train=True), RoundContext())
    torch.testing.assert_close(pipe.learner.G, ref.G)
    assert pipe.learner.running_totals()["fitted"] == 300
    assert pipe.predict(b).shape == (300,)


@pytest.mark.gpu
@pytest.mark.parametrize("B,d0", [(5000, 13), (70001, 13), (999, 5), (4096, 10)])
def test_hip_gram_fused_poly2_vs_expanded_and_fp64(cuda, B, d0):
    """The fused PolynomialFeatures(2) Gram (products formed in the MFMA operand fetch)
    equals the Gram of the expanded batch and the fp64 reference."""
    from omldm_amd.ops.preprocess import poly_expand

    torch.manual_seed(B + d0)
    x = torch.randn(B, d0)
    y = torch.randn(B)
    y[::5] = float("nan")
    pairs = _poly_pairs(d0)
    d = d0 + pairs.shape[0]
    ld = ((d + 2 + 31) // 32) * 32
    Gf = torch.zeros(ld, ld, device=cuda)
    Ge = torch.zeros(ld, ld, device=cuda)
    cf = torch.zeros(1, dtype=torch.float64, device=cuda)
    D.gram_update(x.to(cuda), y.to(cuda), Gf, cnt=cf, pairs=pairs)
    D.gram_update(poly_expand(x, pairs).to(cuda), y.to(cuda), Ge)
    torch.cuda.synchronize()
    ok = ~torch.isnan(y)
    assert float(cf) == float(ok.sum())
    xe = poly_expand(x, pairs)[ok]
    z = torch.cat([xe, torch.ones(int(ok.sum()), 1), y[ok].unsqueeze(1)], 1).double()
    ref = (z.T @ z).numpy()
    np.testing.assert_allclose(Gf.cpu().double().numpy()[: d + 2, : d + 2], ref, rtol=1e-4,
                               atol=2e-2)
    np.testing.assert_allclose(Gf.cpu().numpy(), Ge.cpu().numpy(), rtol=1e-5, atol=1e-2)
    assert torch.equal(Gf.cpu(), Gf.cpu().T)  # mirrored


@pytest.mark.gpu
@pytest.mark.parametrize("nclass,R,S", [(3, 16, 64), (4, 16, 80), (2, 8, 100), (4, 5, 70)])
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_hip_multiclass_register_dedup_matches_table_kernel(cuda, monkeypatch, nclass, R, S,
                                                            variant):
    """Field-aware wire, ≤ 16 rows per spoke, K ≤ 4: the register-dedup MultiClassPA round
    (K deltas per row in registers) equals the LDS-table round (OMLDM_MC_RD=0) and the CPU
    mirror; the stats agree."""
    from omldm_amd.api.batch import FeatureSpace, HashedBatch

    sp = FeatureSpace(13, 0, 26, 1 << 18, field_aware=True)
    B = S * R - R // 3
    b = synth_batch(sp, B, task=2, n_classes=nclass, seed=R * 7 + S)
    W = torch.randn(nclass, sp.dim) * 0.01
    g = HashedBatch(b.num.to(torch.bfloat16), b.cat, b.y.to(torch.int8), cat_span=b.cat_span)
    out = {}
    for rd in ("1", "0"):
        monkeypatch.setenv("OMLDM_MC_RD", rd)
        st = torch.zeros(8, device=cuda)
        dacc = torch.zeros(nclass, sp.dim, device=cuda)
        D.multiclass_round(W.to(cuda), g.to(cuda), R, S, nclass, variant, 0.7, True, dacc, st)
        torch.cuda.synchronize()
        out[rd] = (dacc.cpu(), st.cpu())
    bc = HashedBatch(b.num.to(torch.bfloat16).float(), b.cat, b.y, cat_span=b.cat_span)
    stc, daccc = torch.zeros(8), torch.zeros(nclass, sp.dim)
    D.multiclass_round(W, bc, R, S, nclass, variant, 0.7, True, daccc, stc)
    np.testing.assert_allclose(out["1"][0].numpy(), out["0"][0].numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["1"][1][:4].numpy(), out["0"][1][:4].numpy(), rtol=1e-5)
    np.testing.assert_allclose(out["1"][0].numpy(), daccc.numpy(), rtol=2e-3, atol=2e-4)
