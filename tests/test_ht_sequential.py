"""Hoeffding tree: the engine's tick-level split checks against a per-point VFDT oracle.

Reference semantics (the spoke fits one point at a time,
omldm/operators/spoke/FlinkSpoke.scala:92-107): every training point updates its leaf's
statistics, and a leaf re-evaluates its split as soon as ``gracePeriod`` points reached it
since its last check — so a split made mid-stream routes the very next point. The engine
(models/dense.py: HT, csrc/kernels/hoeffding.hip) updates the statistics of ``checkEvery``
rows at a time (default 1,024) and then checks every due leaf. The NumPy oracle below is
the per-point algorithm with the SAME split criterion (Gaussian class-conditional
statistics, nBins candidate thresholds, information gain, Hoeffding bound with tie
threshold τ); the test pins the quality gap at the engine's 65,536-row ticks on a stream
that needs several levels (checking only at tick ends: 0.93 → 0.56 accuracy).
"""
import math

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.models.base import RoundContext
from omldm_amd.models.dense import HT


def _entropy(c):
    t = c.sum(-1, keepdims=True)
    t = np.maximum(t, 1e-12)
    p = c / t
    return -(p * np.log2(np.maximum(p, 1e-12))).sum(-1)


class VFDT:
    """Per-point Hoeffding tree with models/dense.py:HT's split criterion."""

    def __init__(self, d, C, grace=200, delta=1e-7, tau=0.05, nb=16, max_nodes=255, depth=12):
        self.d, self.C, self.grace, self.delta, self.tau, self.nb = d, C, grace, delta, tau, nb
        self.N, self.depth = max_nodes, depth
        N = max_nodes
        self.feat = -np.ones(N, dtype=np.int64)
        self.thr = np.zeros(N)
        self.left = np.zeros(N, dtype=np.int64)
        self.right = np.zeros(N, dtype=np.int64)
        self.cc = np.zeros((N, C))
        self.S0 = np.zeros((N, d, C))
        self.S1 = np.zeros((N, d, C))
        self.S2 = np.zeros((N, d, C))
        self.lo = np.full((N, d), np.inf)
        self.hi = np.full((N, d), -np.inf)
        self.since = np.zeros(N)
        self.nnodes = 1

    def leaf(self, x):
        node = 0
        for _ in range(self.depth + 1):
            f = self.feat[node]
            if f < 0:
                break
            node = self.left[node] if x[f] <= self.thr[node] else self.right[node]
        return node

    def learn(self, x, y):
        n = self.leaf(x)
        c = int(min(max(y, 0), self.C - 1))
        self.cc[n, c] += 1
        self.S0[n, :, c] += 1
        self.S1[n, :, c] += x
        self.S2[n, :, c] += x * x
        self.lo[n] = np.minimum(self.lo[n], x)
        self.hi[n] = np.maximum(self.hi[n], x)
        self.since[n] += 1
        if self.since[n] >= self.grace:
            self._try_split(n)

    def _try_split(self, node):
        self.since[node] = 0
        cc = self.cc[node]
        n_total = cc.sum()
        if n_total < 2 or self.nnodes + 2 > self.N or (cc > 0).sum() < 2:
            return
        S0, S1, S2 = self.S0[node], self.S1[node], self.S2[node]
        mu = S1 / np.maximum(S0, 1)
        var = np.maximum(S2 / np.maximum(S0, 1) - mu * mu, 1e-6)
        sd = np.sqrt(var)
        lo, hi = self.lo[node], self.hi[node]
        span = np.maximum(hi - lo, 0)
        q = np.linspace(0, 1, self.nb + 2)[1:-1]
        t = lo[:, None] + span[:, None] * q[None, :]
        z = (t[:, :, None] - mu[:, None, :]) / sd[:, None, :]
        cdf = 0.5 * (1 + np.vectorize(math.erf)(z / math.sqrt(2)))
        left = S0[:, None, :] * cdf
        right = S0[:, None, :] - left
        nl, nr = left.sum(-1), right.sum(-1)
        gain = _entropy(cc) - (nl * _entropy(left) + nr * _entropy(right)) / np.maximum(nl + nr, 1e-12)
        gain = np.where(span[:, None] > 0, gain, -1.0)
        per, arg = gain.max(1), gain.argmax(1)
        order = np.argsort(-per, kind="stable")
        g1 = per[order[0]]
        g2 = per[order[1]] if self.d > 1 else 0.0
        R = math.log2(self.C)
        eps = math.sqrt(R * R * math.log(1.0 / self.delta) / (2.0 * n_total))
        if g1 > 0 and (g1 - g2 > eps or eps < self.tau):
            f = int(order[0])
            a, b = self.nnodes, self.nnodes + 1
            self.nnodes += 2
            self.feat[node], self.thr[node] = f, t[f, arg[f]]
            self.left[node], self.right[node] = a, b
            self.cc[a] = left[f, arg[f]]
            self.cc[b] = right[f, arg[f]]

    def predict(self, X):
        return np.array([self.cc[self.leaf(x)].argmax() for x in X])


def _stream(B, seed):
    """Labels from a depth-3 axis-aligned rule plus 5 % noise."""
    g = np.random.default_rng(seed)
    X = g.uniform(-1, 1, size=(B, 6)).astype(np.float32)
    y = ((X[:, 0] > 0.2) ^ ((X[:, 1] > -0.3) & (X[:, 2] < 0.5))).astype(np.float32)
    flip = g.random(B) < 0.05
    y[flip] = 1 - y[flip]
    return X, y


def test_tick_level_tree_matches_the_per_point_tree_within_two_points():
    X, y = _stream(60000, seed=1)
    Xt, yt = _stream(8000, seed=2)
    ora = VFDT(6, 2)
    for i in range(X.shape[0]):
        ora.learn(X[i].astype(np.float64), y[i])
    acc_oracle = float((ora.predict(Xt.astype(np.float64)) == yt).mean())
    sp = FeatureSpace(6, 0, 0, 1 << 8)
    res = {}
    for tick in (1000, 65536):  # the engine's default tick: checks every 1,024 rows
        ht = HT({"nClasses": 2}, sp, "cpu")
        for a in range(0, X.shape[0], tick):
            b = HashedBatch(torch.from_numpy(X[a:a + tick]),
                            torch.zeros((min(tick, X.shape[0] - a), 0), dtype=torch.int32),
                            torch.from_numpy(y[a:a + tick]))
            ht.fit(b, RoundContext())
        pred = ht.predict(HashedBatch(torch.from_numpy(Xt), torch.zeros((len(Xt), 0),
                                                                        dtype=torch.int32),
                                      torch.from_numpy(yt))).numpy()
        res[tick] = (float((pred == yt).mean()), int(ht.nnodes.item()))
    assert acc_oracle > 0.85, acc_oracle
    for tick, (acc, nodes) in res.items():
        # the gap: splits made at tick ends instead of mid-tick
        assert acc >= acc_oracle - 0.02, (tick, acc, acc_oracle, res)
        assert nodes >= 3, res


def _fit_ticks(ht, X, y, tick):
    for a in range(0, X.shape[0], tick):
        b = HashedBatch(torch.from_numpy(X[a:a + tick]).to(ht.device),
                        torch.zeros((min(tick, X.shape[0] - a), 0), dtype=torch.int32,
                                    device=ht.device),
                        torch.from_numpy(y[a:a + tick]).to(ht.device))
        ht.fit(b, RoundContext())


def _acc(ht, Xt, yt):
    b = HashedBatch(torch.from_numpy(Xt).to(ht.device),
                    torch.zeros((len(Xt), 0), dtype=torch.int32, device=ht.device),
                    torch.from_numpy(yt).to(ht.device))
    return float((ht.predict(b).cpu().numpy() == yt).mean())


def test_exact_mode_checks_at_the_grace_point_like_the_per_point_tree():
    """checkEvery 0 (the default): the tick is cut at every point where a leaf reaches its
    grace period, so the tree grows as the per-point VFDT does — the same number of nodes
    and the same first split, at 65,536-row ticks."""
    X, y = _stream(60000, seed=1)
    Xt, yt = _stream(8000, seed=2)
    ora = VFDT(6, 2)
    for i in range(X.shape[0]):
        ora.learn(X[i].astype(np.float64), y[i])
    ht = HT({"nClasses": 2}, FeatureSpace(6, 0, 0, 1 << 8), "cpu")
    assert ht.check_every == 0
    _fit_ticks(ht, X, y, 65536)
    assert abs(int(ht.nnodes.item()) - ora.nnodes) <= 2, (int(ht.nnodes.item()), ora.nnodes)
    assert int(ht.feat[0]) == int(ora.feat[0])
    acc_oracle = float((ora.predict(Xt.astype(np.float64)) == yt).mean())
    assert _acc(ht, Xt, yt) >= acc_oracle - 0.005


@pytest.mark.gpu
def test_gpu_exact_mode_matches_the_cpu_exact_mode():
    """The device path of the exact mode (ht_route + segments ending at each due point,
    csrc/kernels/hoeffding.hip) grows the tree the CPU exact mode grows."""
    X, y = _stream(60000, seed=3)
    Xt, yt = _stream(8000, seed=4)
    sp = FeatureSpace(6, 0, 0, 1 << 8)
    res = {}
    for dev in ("cpu", "cuda"):
        ht = HT({"nClasses": 2}, sp, dev)
        _fit_ticks(ht, X, y, 65536)
        res[dev] = (int(ht.nnodes.item()), int(ht.feat[0]), _acc(ht, Xt, yt))
    assert res["cuda"][1] == res["cpu"][1], res
    assert abs(res["cuda"][0] - res["cpu"][0]) <= 2, res
    assert abs(res["cuda"][2] - res["cpu"][2]) <= 0.005, res


@pytest.mark.gpu
@pytest.mark.parametrize("C,d", [(2, 6), (4, 6), (3, 13)])
def test_gpu_persistent_exact_matches_the_host_driven_loop_and_the_oracle(C, d):
    """The persistent one-launch exact mode (ht_exact_kernel) grows the tree the host-driven
    segment loop grows (same split points, same nodes), and the per-point NumPy VFDT's."""
    g = np.random.default_rng(7 + C)
    X = g.uniform(-1, 1, size=(70000, d)).astype(np.float32)
    y = ((X[:, 0] > 0.2).astype(int) + (X[:, 1] > -0.3).astype(int) * (C - 1)) % C
    y = y.astype(np.float32)
    flip = g.random(len(y)) < 0.05
    y[flip] = g.integers(0, C, int(flip.sum()))
    y[g.random(len(y)) < 0.02] = np.nan  # forecasting-like rows: not fitted
    Xt = g.uniform(-1, 1, size=(6000, d)).astype(np.float32)
    yt = (((Xt[:, 0] > 0.2).astype(int) + (Xt[:, 1] > -0.3).astype(int) * (C - 1)) % C)
    sp = FeatureSpace(d, 0, 0, 1 << 8)
    res = {}
    for mode in (True, False):
        ht = HT({"nClasses": C, "exactDevice": mode}, sp, "cuda")
        _fit_ticks(ht, X, y, 65536)
        torch.cuda.synchronize()
        n = int(ht.nnodes.item())
        res[mode] = (n, ht.feat[:n].cpu().numpy().copy(), ht.thr[:n].cpu().numpy().copy(),
                     _acc(ht, Xt, yt.astype(np.float32)), int(ht.cum[1].item()))
    dev, host = res[True], res[False]
    assert dev[4] == host[4] == int((~np.isnan(y)).sum())
    assert dev[0] == host[0], (dev[0], host[0])
    assert np.array_equal(dev[1], host[1])
    assert np.allclose(dev[2], host[2], rtol=1e-4, atol=1e-5)
    assert abs(dev[3] - host[3]) <= 0.002
    ora = VFDT(d, C)
    for i in range(X.shape[0]):
        if not np.isnan(y[i]):
            ora.learn(X[i].astype(np.float64), y[i])
    assert abs(dev[0] - ora.nnodes) <= 2, (dev[0], ora.nnodes)
    assert int(dev[1][0]) == int(ora.feat[0])
