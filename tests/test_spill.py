"""No dropped updates: the spoke learners' LDS delta tables spill to HBM (spoke_table.h:
Spill) instead of dropping an update when a spoke's distinct keys outgrow them.

Reference: every spoke fits every point, strictly in order (FlinkSpoke.scala:92-107), for
all eight learners (PipelineMap.scala:68). The GPU tests run the engine's default spoke
geometry (16 spokes per device, R = 4096 / 8192 rows, 2^20 hashed dims — a spoke then
touches ~40 K distinct keys against an 8 K-entry LDS table) and compare with the CPU
oracle (csrc/host/linear_cpu.cpp, dense_cpu.cpp), overflow counter == 0.
"""
import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.ops import dense as D
from omldm_amd.ops import linear as L
from omldm_amd.ops import native


def test_spill_sizing():
    # ≥ 2 × the spoke's key occurrences, clamped to [2^6, 2^24]
    assert L.spill_log2cap(8192, 40) == 20
    assert L.spill_log2cap(1, 1) == 6
    assert L.spill_log2cap(1 << 20, 64) == 24
    for R, k in ((4096, 40), (16, 40), (70, 57)):
        assert (1 << L.spill_log2cap(R, k)) >= 2 * R * k


BIG = FeatureSpace(13, 0, 26, 1 << 20)
SPILL_RULES = {
    "svm_l2": L.LinearRule(L.RULE_HINGE, L.PA1, C=1.0, lam=1e-4),
    "pegasos": L.LinearRule(L.RULE_PEGASOS, lam=1e-4, tbase=2.0),
    "pa1": L.LinearRule(L.RULE_HINGE, L.PA1, C=1.0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("R", [4096, 8192])
@pytest.mark.parametrize("name,dtype", [("svm_l2", torch.float32), ("pegasos", torch.float32),
                                        ("pa1", torch.bfloat16)])
def test_hip_linear_round_spills_exactly(cuda, R, name, dtype):
    """SVM with L2 shrink, Pegasos and a bf16 model at S = 16 spokes × R rows: the
    spoke-table round equals the CPU oracle with no dropped update."""
    S = 16
    rule = SPILL_RULES[name]
    b = synth_batch(BIG, S * R, seed=R + 7)
    w = (torch.randn(BIG.dim) * 0.01).to(dtype)
    d_cpu = torch.zeros(BIG.dim + 2)
    s_cpu = torch.zeros(S, 6)
    L.linear_round(w, b, R, S, d_cpu, s_cpu, rule, 1.0 / S)
    d_gpu = torch.zeros(BIG.dim + 2, device=cuda)
    s_gpu = torch.zeros(S, 6, device=cuda)
    cum = torch.zeros(8, dtype=torch.float64, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), R, S, d_gpu, s_gpu, rule, 1.0 / S, cum=cum)
    torch.cuda.synchronize()
    s_g = s_gpu.cpu()
    assert float(s_g[:, 5].sum()) == 0.0 and float(cum[5]) == 0.0  # nothing dropped
    np.testing.assert_allclose(s_g[:, 1].numpy(), s_cpu[:, 1].numpy())
    np.testing.assert_allclose(s_g[:, 2].numpy(), s_cpu[:, 2].numpy(), atol=2)
    # fp32 summation order differs (Pegasos' first steps are η = 1/(λT) ~ 5e3: scale atol)
    atol = 2e-5 * max(1.0, float(d_cpu.abs().max()))
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=atol)
    # a second round on the same (restored) spill region gives the same answer
    d2 = torch.zeros(BIG.dim + 2, device=cuda)
    L.linear_round(w.to(cuda), b.to(cuda), R, S, d2, None, rule, 1.0 / S)
    torch.cuda.synchronize()
    # (the spokes' atomic adds into dacc land in any order: cancellations leave ~ulp(max|d|))
    np.testing.assert_allclose(d2.cpu().numpy(), d_gpu.cpu().numpy(), rtol=1e-5,
                               atol=1e-6 * max(1.0, float(d_cpu.abs().max())))


@pytest.mark.gpu
def test_hip_linear_round_tiny_table_equals_big_table(cuda):
    """A 1 K-entry LDS table (most keys in the HBM spill) gives the 8 K table's round."""
    S, R = 8, 512
    b = synth_batch(BIG, S * R, seed=8).to(cuda)
    w = (torch.randn(BIG.dim) * 0.01).to(cuda)
    out = []
    for lg in (10, 13):
        d = torch.zeros(BIG.dim + 2, device=cuda)
        st = torch.zeros(S, 6, device=cuda)
        L.linear_round(w, b, R, S, d, st, L.LinearRule(), 1.0, log2cap=lg)
        torch.cuda.synchronize()
        assert float(st[:, 5].sum()) == 0.0
        out.append(d.cpu())
    np.testing.assert_allclose(out[0].numpy(), out[1].numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [4096, 8192])
def test_hip_multiclass_round_spills_exactly(cuda, R):
    """MultiClassPA, K = 4 classes, 16 spokes × R rows, 2^20 dims: equal to the CPU
    mirror, overflow == 0."""
    S, K = 16, 4
    b = synth_batch(BIG, S * R, task=2, n_classes=K, seed=R + 3)
    W = torch.randn(K, BIG.dim) * 0.01
    st, dacc = torch.zeros(8), torch.zeros(K, BIG.dim)
    D.multiclass_round(W, b, R, S, K, 1, 1.0, True, dacc, st)
    stg, daccg = torch.zeros(8, device=cuda), torch.zeros(K, BIG.dim, device=cuda)
    D.multiclass_round(W.to(cuda), b.to(cuda), R, S, K, 1, 1.0, True, daccg, stg)
    torch.cuda.synchronize()
    assert float(stg[5]) == 0.0  # no dropped update
    np.testing.assert_allclose(stg.cpu()[[1, 3]].numpy(), st[[1, 3]].numpy())
    np.testing.assert_allclose(stg.cpu()[2].item(), st[2].item(), atol=3)
    np.testing.assert_allclose(daccg.cpu().numpy(), dacc.numpy(), rtol=2e-3, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name,hyper,task", [
    ("MultiClassPA", {"nClasses": 4}, 2),
    ("SVM", {"lambda": 1e-4}, 0),
    ("SVM", {"variant": "Pegasos", "lambda": 1e-4}, 0),
    ("SVM", {"modelDtype": "bf16"}, 0),
])
def test_hip_engine_default_geometry_learner_matches_cpu(cuda, name, hyper, task):
    """The learner at the engine's default flags (16 spokes, 65536-row ticks → R = 4096,
    2^20 dims) trains the model the CPU learner trains, and reports no overflow."""
    from omldm_amd.models import make_learner
    from omldm_amd.models.base import RoundContext

    models = {}
    for dev in ("cpu", cuda):
        lr = make_learner(name, dict(hyper), BIG, dev)
        for r in range(2):
            b = synth_batch(BIG, 65536, start=r * 65536, task=task, n_classes=4, seed=11)
            lr.fit(b.to(dev) if dev != "cpu" else b, RoundContext(spokes=16, inv_p=1.0 / 16))
        tot = lr.running_totals()
        assert tot["overflow"] == 0 and tot["fitted"] == 2 * 65536
        models[str(dev)] = lr.state_vector().detach().float().cpu()
    np.testing.assert_allclose(models["cuda:0"].numpy(), models["cpu"].numpy(),
                               rtol=5e-3, atol=5e-5)


def test_spill_is_capped_by_the_memory_budget():
    """A MultiClassPA-sized spill (16 spokes, 8192 rows × 40 keys, 16-float entries) would
    take ~1.2 GB per stream; the cap keeps one workspace within the budget."""
    words = native.hip().omldm_spill_words
    lg = L.spill_log2cap(8192, 40, 16, 16)
    assert int(words(16, lg, 16)) * 4 <= L._SPILL_BUDGET
    assert lg >= 6
