"""Exact sequential k-means (the reference learner's per-point update, SURVEY Appendix D:
nearest centroid, c ← c + (x − c)/n_c, one point at a time as the spoke fits them,
omldm/operators/spoke/FlinkSpoke.scala:92-107) — the CPU oracle against a NumPy per-point
model, the GPU kernel (csrc/kernels/kmeans_seq.hip) against the CPU oracle, and the quality
gap of the mini-batch form at engine-sized ticks pinned."""
import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.models.dense import KMeans
from omldm_amd.models.base import RoundContext
from omldm_amd.ops import dense as D


def _blobs(B, d, k, seed):
    g = np.random.default_rng(seed)
    centers = g.normal(0, 4, size=(k, d))
    lab = g.integers(0, k, B)
    x = centers[lab] + g.normal(0, 1, size=(B, d))
    y = np.zeros(B, dtype=np.float32)
    y[g.random(B) < 0.05] = np.nan  # forecasting-like rows: not fitted
    return x.astype(np.float32), y


def _numpy_macqueen(x, y, k):
    d = x.shape[1]
    C = np.zeros((k, d), dtype=np.float32)
    n = np.zeros(k, dtype=np.float32)
    seeded, inertia, fitted = 0, 0.0, 0
    for r in range(x.shape[0]):
        if np.isnan(y[r]):
            continue
        fitted += 1
        if seeded < k:
            C[seeded], n[seeded] = x[r], 1
            seeded += 1
            continue
        dist = ((x[r][None, :] - C) ** 2).sum(1)
        j = int(np.argmin(dist))
        inertia += float(dist[j])
        n[j] += 1
        C[j] += (x[r] - C[j]) / n[j]
    return C, n, inertia, fitted


@pytest.mark.parametrize("d,k", [(3, 4), (13, 8), (40, 64)])
def test_cpu_oracle_is_macqueen(d, k):
    x, y = _blobs(3000, d, k, seed=d + k)
    C = torch.zeros(k, d)
    n = torch.zeros(k)
    cum = torch.zeros(8, dtype=torch.float64)
    for a in range(0, 3000, 700):  # chunked calls continue the same stream
        D.kmeans_seq(torch.from_numpy(x[a:a + 700]), torch.from_numpy(y[a:a + 700]), C, n, cum)
    Cr, nr, inert, fitted = _numpy_macqueen(x, y, k)
    assert np.allclose(C.numpy(), Cr, rtol=1e-4, atol=1e-4)
    assert np.array_equal(n.numpy(), nr)
    assert int(cum[1]) == fitted
    assert abs(float(cum[0]) - inert) <= 1e-4 * max(1.0, inert)


def test_learner_default_is_sequential_and_minibatch_gap_is_pinned():
    """At the engine's 65,536-row ticks the mini-batch form (assignments against the
    tick-start centroids) ends within 2 % of the sequential form's mean squared distance
    on well-separated blobs; the sequential form is the default."""
    d, k = 8, 6
    sp = FeatureSpace(d, 0, 0, 1 << 10)
    x, y = _blobs(4 * 65536, d, k, seed=3)
    y = np.nan_to_num(y, nan=0.0)
    res = {}
    for mode in ("sequential", "minibatch"):
        lrn = KMeans({"k": k, "mode": mode}, sp, "cpu")
        assert lrn.sequential == (mode == "sequential")
        for a in range(0, x.shape[0], 65536):
            b = HashedBatch(torch.from_numpy(x[a:a + 65536]),
                            torch.zeros((65536, 0), dtype=torch.int32),
                            torch.from_numpy(y[a:a + 65536]))
            lrn.fit(b, RoundContext())
        test = torch.from_numpy(_blobs(5000, d, k, seed=99)[0])
        res[mode] = float((torch.cdist(test, lrn.C) ** 2).min(1).values.mean())
    assert res["minibatch"] <= 1.02 * res["sequential"], res
    assert KMeans({"k": 3}, sp, "cpu").sequential


@pytest.mark.gpu
@pytest.mark.parametrize("form", [1, 0])
@pytest.mark.parametrize("d,k", [(3, 4), (13, 8), (13, 16), (20, 33), (64, 64), (100, 20),
                                 (13, 200), (13, 256), (30, 100), (5, 500), (2, 3), (40, 2),
                                 (128, 200), (13, 1500), (300, 40)])
def test_gpu_kernel_equals_cpu_oracle(d, k, form):
    """Both GPU forms against the CPU MacQueen oracle: form 1 = the fast one-wave kernel
    (G lanes per centroid / CPL centroids per lane; k ≤ 512, d ≤ 64, else the workgroup
    kernel), form 0 = the earlier one-wave kernel (k, d ≤ 64) and the workgroup kernel
    (centroids in LDS, up to k = 1024, d = 256). Same assignments (equal counts)."""
    prev = D.kmeans_seq_form()
    D.kmeans_seq_form(form)
    try:
        _gpu_vs_oracle(d, k)
    finally:
        D.kmeans_seq_form(prev)


def _gpu_vs_oracle(d, k):
    x, y = _blobs(20000, d, k, seed=7 * d + k)
    out = {}
    for dev in ("cpu", "cuda"):
        C = torch.zeros(k, d, device=dev)
        n = torch.zeros(k, device=dev)
        cum = torch.zeros(8, dtype=torch.float64, device=dev)
        for a in range(0, 20000, 6000):
            D.kmeans_seq(torch.from_numpy(x[a:a + 6000]).to(dev),
                         torch.from_numpy(y[a:a + 6000]).to(dev), C, n, cum)
        out[dev] = (C.cpu(), n.cpu(), cum.cpu())
    assert torch.allclose(out["cuda"][0], out["cpu"][0], rtol=1e-5, atol=1e-5), \
        (out["cuda"][0] - out["cpu"][0]).abs().max()
    assert torch.equal(out["cuda"][1], out["cpu"][1])
    assert out["cuda"][2][1] == out["cpu"][2][1]
    assert abs(float(out["cuda"][2][0] - out["cpu"][2][0])) <= 1e-5 * float(out["cpu"][2][0])
