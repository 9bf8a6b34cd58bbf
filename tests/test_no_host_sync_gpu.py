"""No host synchronisation inside a GM / FGM / Synchronous round on the GPU.

A long device-side spin (torch.cuda._sleep) is queued in front of the rounds: if any
round waited for the stream (an ``.item()``, ``.tolist()``, a blocking copy) the host
would stall until the spin ends. The monitoring decision is read one round late through a
pinned copy recorded BEFORE the spin, so the host runs ahead (protocols.py
_LaggedDecision)."""
import time

import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.models import make_learner
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import make_protocol

pytestmark = pytest.mark.gpu

SP = FeatureSpace(13, 0, 26, 1 << 16)


@pytest.mark.parametrize("proto", ["GM", "FGM", "Synchronous"])
def test_rounds_do_not_wait_for_the_device(proto):
    dev = torch.device("cuda", 0)
    L = make_learner("SVM", {}, SP, dev)
    P = make_protocol(proto, Comm(), L, {"threshold": 0.01, "epsilon": 0.01, "virtualSpokes": 8})
    batches = [synth_batch(SP, 1024, start=i * 1024).to(dev) for i in range(6)]
    P.round(batches[0])  # buffers, first decision posted
    torch.cuda.synchronize()
    # calibrate the spin: ~200 ms of device time (the second measurement: the first
    # includes the spin kernel's first launch)
    for _ in range(2):
        t = time.perf_counter()
        torch.cuda._sleep(20_000_000)
        torch.cuda.synchronize()
        per = (time.perf_counter() - t) / 20_000_000
    cycles = int(0.2 / max(per, 1e-12))
    torch.cuda._sleep(cycles)
    # GM/FGM: the host may run one round ahead of the device (the decision of round k is
    # read in round k + 1); Synchronous never reads anything back
    ahead = batches[1:2] if proto in ("GM", "FGM") else batches[1:]
    t = time.perf_counter()
    for b in ahead:
        P.round(b)
    host_s = time.perf_counter() - t
    for b in batches[1 + len(ahead):]:
        P.round(b)
    torch.cuda.synchronize()
    total_s = time.perf_counter() - t
    assert total_s > 0.08, total_s  # the spin really ran
    assert host_s < 0.25 * total_s, (proto, host_s, total_s)
    assert L.running_totals()["fitted"] == 6 * 1024
