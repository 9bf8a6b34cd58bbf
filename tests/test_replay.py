"""Deterministic replay: the same stream through the same protocol gives
the same model. CPU path (C++ mirror, fixed reduction order): bitwise, including a
resume from a learner+protocol state snapshot halfway. GPU path: the bucket reducer
adds LDS / L2 float atomics in hardware order, so replays agree to fp32 reassociation
(≤ 1e-5 relative), never more."""
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.models.linear import SVM
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import Synchronous

SP = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)


def _train(device, rounds, L=None, P=None, start=0):
    if L is None:
        L = SVM({"variant": "PA-I", "lambda": 1e-4}, SP, device)
        P = Synchronous(Comm(), L, {"virtualSpokes": 64})
    for r in range(start, start + rounds):
        P.round(synth_batch(SP, 64 * 16, start=r * 1024, seed=3).to(device))
    return L, P


def test_cpu_replay_is_bitwise():
    a, _ = _train("cpu", 6)
    b, _ = _train("cpu", 6)
    assert torch.equal(a.w, b.w)
    assert torch.equal(a.cum, b.cum)


def test_cpu_resume_from_snapshot_is_bitwise():
    full, _ = _train("cpu", 6)
    half, P = _train("cpu", 3)
    sd_l, sd_p = half.state_dict(), P.state_dict()
    L2 = SVM({"variant": "PA-I", "lambda": 1e-4}, SP, "cpu")
    P2 = Synchronous(Comm(), L2, {"virtualSpokes": 64})
    L2.load_state_dict(sd_l)
    P2.load_state_dict(sd_p)
    _train("cpu", 3, L2, P2, start=3)
    assert torch.equal(full.w, L2.w)


@pytest.mark.gpu
def test_gpu_replay_within_reassociation(cuda):
    a, _ = _train(cuda, 6)
    b, _ = _train(cuda, 6)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.w, b.w, rtol=1e-5, atol=1e-7)
    c, _ = _train("cpu", 6)
    torch.testing.assert_close(a.w.cpu(), c.w, rtol=2e-3, atol=2e-4)
