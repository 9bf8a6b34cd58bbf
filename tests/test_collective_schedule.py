"""The exact per-round communication schedule of every protocol (gloo, 2 and 4 ranks).

Every call through parallel/comm.py is traced as (kind, tag, bytes); the tests pin, round
by round, which collectives / point-to-point transfers each protocol issues and how many
bytes they carry — the schedule the RCCL path runs on a node (one process per GPU), so a
protocol change that adds a collective or a host round-trip shows up here.
Reference: the per-protocol message patterns of MLNodeGenerator.scala:20-76 /
FlinkNetwork.scala:242-293.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.models import make_learner
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import make_protocol

SP = FeatureSpace(13, 0, 26, 1 << 12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, learner, proto, cfg, rounds, task):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm()
    L = make_learner(learner, {"k": 3}, SP, "cpu")
    P = make_protocol(proto, comm, L, cfg, spokes=2, max_msg_params=1000)
    comm.stats.trace = []
    per_round = []
    for r in range(rounds):
        b = synth_batch(SP, 128, start=(r * world + rank) * 128, task=task)
        n0 = len(comm.stats.trace)
        P.round(b)
        per_round.append(list(comm.stats.trace[n0:]))
    P.finalize()
    x = L.state_vector()
    res = {"rounds": per_round, "model_bytes": x.numel() * x.element_size(),
           "delta_bytes": (L.delta_buffer().numel() * L.delta_buffer().element_size()
                           if L.supports_fused_delta else None),
           "syncs": P.stats.syncs}
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run(world, learner, proto, cfg=None, rounds=6, task=0):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, learner, proto, cfg or {},
                                          rounds, task), nprocs=world, start_method="fork")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("hubs,kind,factor", [(0, "all_reduce", 1), (1, "reduce+bcast", 2)])
def test_synchronous_one_collective_per_round(world, hubs, kind, factor):
    res = run(world, "SVM", "Synchronous", {"HubParallelism": hubs} if hubs else {})
    for r in res:
        nb = r["delta_bytes"]
        assert nb is not None
        assert r["rounds"] == [[(kind, "sync", factor * nb)]] * 6


def test_synchronous_sharded_hubs_point_to_point_world4():
    res = run(4, "SVM", "Synchronous", {"HubParallelism": 2})
    for r in res:
        assert r["rounds"] == [[("p2p_shards", "sync", 2 * r["delta_bytes"])]] * 6


@pytest.mark.parametrize("world", [2, 4])
def test_easgd_every_tau_rounds(world):
    res = run(world, "PA", "EASGD", {"tau": 2, "alpha": 0.3})
    for r in res:
        nb = r["model_bytes"]
        assert r["rounds"] == [[], [("all_reduce", "elastic", nb)]] * 3


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("proto,tag,nbytes", [("GM", "gm-flag", 8), ("FGM", "fgm-counters", 16)])
def test_monitoring_one_small_reduction_or_one_sync_per_round(world, proto, tag, nbytes):
    """GM / FGM: a round issues EITHER the 8/16-byte monitoring reduction OR (the round
    after a violation — the decision is read one round late) one full model sync; the
    schedule is identical on every rank."""
    res = run(world, "ORR", proto, {"threshold": 0.01, "epsilon": 0.01}, rounds=8, task=1)
    for r in res:
        nb = r["model_bytes"]
        for calls in r["rounds"]:
            assert calls in ([("all_reduce", tag, nbytes)], [("all_reduce", "sync", nb)]), calls
        n_sync = sum(c == [("all_reduce", "sync", nb)] for c in r["rounds"])
        assert n_sync == r["syncs"] >= 1
        assert r["rounds"] == res[0]["rounds"]
    # the first round can only monitor: a decision is never read in the round it is made
    assert res[0]["rounds"][0] == [("all_reduce", tag, nbytes)]


@pytest.mark.parametrize("world", [2, 4])
def test_single_learner_points_to_hub_only(world):
    """Points go to the hub only; the hub model reaches the replicas every
    ``broadcastEvery`` rounds (here 2), not every round."""
    res = run(world, "K-means", "SingleLearner", {"broadcastEvery": 2}, rounds=3)
    nb = res[0]["model_bytes"]
    bc = ("broadcast", "bcast", nb)
    assert res[0]["rounds"] == [[], [bc], []]  # the hub receives only
    for r in res[1:]:
        for k, calls in enumerate(r["rounds"]):
            sends = [c for c in calls if c[0] == "p2p_send"]
            assert [c[1] for c in sends] == ["gather"] * 3  # num, cat, y → hub
            assert (calls[-1] == bc) == (k == 1), (k, calls)
            assert not [c for c in calls if c[0] in ("all_reduce", "reduce+bcast")]


@pytest.mark.parametrize("proto", ["Asynchronous", "SSP"])
def test_point_to_point_protocols_issue_no_collective_per_round(proto):
    res = run(4, "PA", proto, {"staleness": 2, "HubParallelism": 2})
    for rank, r in enumerate(res):
        for calls in r["rounds"]:
            assert all(c[0] == "p2p_send" and c[1] == "async-push" for c in calls), calls
            # at most one push per remote hub shard per round
            assert len(calls) <= 2 - (1 if rank < 2 else 0)
        assert sum(len(c) for c in r["rounds"]) >= 1


def test_centralized_training_is_silent():
    res = run(2, "SVM", "CentralizedTraining")
    assert all(calls == [] for r in res for calls in r["rounds"])
