"""Multi-rank rehearsal on ONE GPU: two ranks share cuda:0 and talk over gloo (the
8-GPU RCCL run is the driver's). It exercises the exact multi-GPU code path of bench.py —
device-resident fused round accumulators summed by a collective, then applied — and
checks the Synchronous invariant: two ranks × S spokes == one rank × 2S spokes on the
concatenated batch, on the v3 table scan the bench runs at N > 1 (fp32 and bf16 models)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from omldm_amd.api.batch import FeatureSpace

SP = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
SP_WIDE = FeatureSpace(13, 0, 26, 1 << 16)  # not field-aware: the spoke-table round
ROUNDS = 3
# (learner hyper-parameters, spokes per rank, rows per spoke, v3 scan): "table" runs the
# spoke-table round, whose reduce really is split in key ranges (reduceParts = 3: each
# part's all-reduce starts as that part completes); the v3 scan completes its accumulator
# only at the round end, so there a reduceParts split is not applied
CASES = {"fp32": ({"variant": "PA-I"}, 16, 512, True),
         "bf16": ({"variant": "PA-I", "modelDtype": "bf16"}, 64, 16, True),
         "table": ({"variant": "PA-I", "tableLog2": 10}, 16, 256, False)}


def _space(case):
    return SP if CASES[case][3] else SP_WIDE


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank, world, r, S, R, sp=SP):
    from omldm_amd.io.synthetic import synth_batch

    return synth_batch(sp, S * R, start=(r * world + rank) * S * R, seed=7)


def _rank(rank, world, port, out, parts, case):
    import torch.distributed as dist

    from omldm_amd.models.linear import SVM
    from omldm_amd.ops import linear as OL
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import Synchronous

    hyper, S, R, _ = CASES[case]
    sp = _space(case)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    L = SVM(dict(hyper), sp, dev)
    P = Synchronous(Comm(), L, {"virtualSpokes": S, "reduceParts": parts})
    v3 = OL.SCAN3_ROUNDS
    piped = 0
    for r in range(ROUNDS):
        b = _batch(rank, world, r, S, R, sp).to(dev)
        piped += int(P._pipelined(b))
        P.round(b)
    torch.cuda.synchronize()
    torch.save({"w": L.w.cpu(), "v3": torch.tensor(OL.SCAN3_ROUNDS - v3),
                "piped": torch.tensor(piped)}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("case,parts", [("fp32", 1), ("fp32", 3), ("bf16", 1), ("table", 3)])
def test_two_ranks_one_gpu_equal_one_rank_double_spokes(cuda, case, parts):
    from omldm_amd.api.batch import HashedBatch
    from omldm_amd.models.linear import SVM
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import Synchronous

    hyper, S, R, v3 = CASES[case]
    sp = _space(case)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(2, _port(), d, parts, case), nprocs=2,
                           start_method="spawn")
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    want = ROUNDS if v3 else 0
    assert int(r0["v3"]) == int(r1["v3"]) == want, "the ranks' rounds took the wrong kernel"
    # the pipelined (key-range) reduce runs exactly where the round's kernel has parts
    assert int(r0["piped"]) == (ROUNDS if parts > 1 and not v3 else 0)
    w0, w1 = r0["w"], r1["w"]
    torch.testing.assert_close(w0, w1)
    assert float(w0.abs().sum()) > 0
    # single rank, 2S spokes, rank-0 rows then rank-1 rows (spoke s ↔ rows [sR, sR+R))
    L = SVM(dict(hyper), sp, cuda)
    P = Synchronous(Comm(), L, {"virtualSpokes": 2 * S})
    for r in range(ROUNDS):
        b = HashedBatch.cat_batches([_batch(0, 2, r, S, R, sp), _batch(1, 2, r, S, R, sp)])
        P.round(b.to(cuda))
    torch.cuda.synchronize()
    torch.testing.assert_close(L.w.cpu(), w0, rtol=1e-3, atol=1e-4)


def _proto_rank(rank, world, port, out, proto, learner, cfg):
    import torch.distributed as dist

    from omldm_amd.io.synthetic import synth_batch
    from omldm_amd.models import make_learner
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import make_protocol

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    task = 1 if learner == "ORR" else 0
    L = make_learner(learner, {}, SP, dev)
    P = make_protocol(proto, Comm(), L, cfg, spokes=16)
    for r in range(4):
        b = synth_batch(SP, 1024, start=(r * world + rank) * 1024, seed=11, task=task)
        P.round(b.to(dev))
    P.finalize()
    torch.cuda.synchronize()
    res = {"w": L.state_vector().detach().cpu()}
    for attr in ("_E", "_c"):
        if getattr(P, attr, None) is not None:
            res[attr] = getattr(P, attr).detach().cpu()
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("proto,learner,cfg", [
    ("Asynchronous", "PA", {}), ("SSP", "SVM", {"staleness": 2}),
    ("EASGD", "PA", {"tau": 2, "alpha": 0.3}), ("GM", "ORR", {"threshold": 0.01}),
    ("FGM", "SVM", {"epsilon": 0.05})])
def test_protocols_on_gpu_two_ranks(cuda, proto, learner, cfg):
    """Every distributed protocol with device tensors (fused merge kernels on the GPU):
    replicas / estimates / centres agree across ranks after the run."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_proto_rank, args=(2, _port(), d, proto, learner, cfg), nprocs=2,
                           start_method="spawn")
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    for k in ("_E", "_c"):
        if k in r0:
            torch.testing.assert_close(r0[k], r1[k], rtol=1e-5, atol=1e-6)
    if proto in ("Asynchronous", "SSP"):
        torch.testing.assert_close(r0["w"], r1["w"], rtol=1e-5, atol=1e-6)
    assert float(r0["w"].abs().sum()) > 0
