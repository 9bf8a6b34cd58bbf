"""Synchronisation protocols on real multi-process collectives (gloo, CPU, world 2 and 4).

Invariants checked per protocol:
* Synchronous (H>1 all-reduce and H=1 reduce+broadcast): replicas identical after every
  round and equal to one process running all workers' spokes;
* Asynchronous / SSP: after draining, every rank holds the same merged model;
* EASGD: centre variables identical; GM / FGM: estimates identical, syncs counted;
* SingleLearner: only the hub trains, replicas equal to the hub model.
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

SP = FeatureSpace(13, 0, 26, 1 << 14)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, learner, proto, cfg, rounds, B, task):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["OMLDM_CPU_THREADS"] = "1"
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm()
    L = make_learner(learner, {"nClasses": 3, "k": 3}, SP, "cpu")
    P = make_protocol(proto, comm, L, cfg, spokes=2, max_msg_params=1000)
    states = []
    for r in range(rounds):
        b = synth_batch(SP, B, start=(r * world + rank) * B, task=task, n_classes=3)
        P.round(b)
        states.append(L.state_vector().clone())
    P.finalize()
    res = {"final": L.state_vector().clone(), "states": states, "stats": P.stats.as_dict(),
           "fitted": L.running_totals()["fitted"]}
    for attr in ("_E", "_c"):
        if getattr(P, attr, None) is not None:
            res[attr] = getattr(P, attr).clone()
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run(world, learner, proto, cfg=None, rounds=4, B=256, task=0):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, learner, proto, cfg or {},
                                          rounds, B, task), nprocs=world, start_method="fork")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


def same(a, b, tol=1e-5):
    return torch.allclose(a, b, rtol=tol, atol=tol)


@pytest.mark.parametrize("hubs", [0, 1])
def test_synchronous_replicas_and_equivalence(hubs):
    cfg = {"HubParallelism": hubs} if hubs else {}
    res = run(2, "SVM", "Synchronous", cfg)
    for s0, s1 in zip(res[0]["states"], res[1]["states"]):
        assert same(s0, s1)
    # one process running both ranks' spokes over the concatenated shards
    L = make_learner("SVM", {}, SP, "cpu")
    P = make_protocol("Synchronous", Comm(), L, {}, spokes=4)
    for r in range(4):
        b0 = synth_batch(SP, 256, start=(r * 2) * 256)
        b1 = synth_batch(SP, 256, start=(r * 2 + 1) * 256)
        from omldm_amd.api.batch import HashedBatch
        P.round(HashedBatch.cat_batches([b0, b1]))
    assert same(L.state_vector(), res[0]["final"], 1e-4)
    assert res[0]["stats"]["modelsShipped"] == 4 * 2 * 2


def test_synchronous_pipelined_reduce_matches_one_shot():
    """reduceParts > 1: the delta is all-reduced in key-range slices as they complete —
    the same sums as one all-reduce of the whole buffer, same accounting."""
    base = run(2, "SVM", "Synchronous", {})
    piped = run(2, "SVM", "Synchronous", {"reduceParts": 3})
    for r in range(2):
        for a, b in zip(base[r]["states"], piped[r]["states"]):
            assert same(a, b, 1e-6)
    assert piped[0]["stats"]["modelsShipped"] == base[0]["stats"]["modelsShipped"]
    assert piped[0]["stats"]["bytesShipped"] == base[0]["stats"]["bytesShipped"]


def test_part_bounds_cover_accumulator():
    from omldm_amd.ops.linear import part_bounds

    for dim in (1 << 14, (1 << 20) + 7, 100):
        for parts in (1, 2, 3, 4, 8):
            sl = [part_bounds(dim, k, parts, cuda=False) for k in range(parts)]
            assert sl[0][0] == 0 and sl[-1][1] == dim + 2
            assert all(sl[k][1] == sl[k + 1][0] for k in range(parts - 1))


@pytest.mark.parametrize("proto,cfg", [("Asynchronous", {}), ("SSP", {"staleness": 2})])
def test_delayed_protocols_converge_to_same_model(proto, cfg):
    res = run(2, "PA", proto, cfg, rounds=5)
    # after finalize every rank holds the hub's global model (parallel/p2p.py)
    assert same(res[0]["final"], res[1]["final"])
    assert res[0]["fitted"] > 0 and float(res[0]["final"].abs().sum()) > 0


def test_easgd_centre_consistent():
    res = run(2, "PA", "EASGD", {"tau": 2, "alpha": 0.3}, rounds=4)
    assert same(res[0]["_c"], res[1]["_c"])


@pytest.mark.parametrize("proto", ["GM", "FGM"])
def test_monitoring_protocols(proto):
    res = run(2, "ORR", proto, {"threshold": 0.01, "epsilon": 0.01}, rounds=6, task=1)
    assert same(res[0]["_E"], res[1]["_E"])
    assert res[0]["stats"]["syncs"] >= 1
    assert res[0]["stats"]["smallMessages"] > 0


def test_fgm_linear_world4():
    res = run(4, "SVM", "FGM", {"epsilon": 0.05}, rounds=5)
    for r in res[1:]:
        assert same(r["_E"], res[0]["_E"])


def test_single_learner_hub_only():
    res = run(2, "K-means", "SingleLearner", rounds=3)
    assert same(res[0]["final"], res[1]["final"])
    assert res[0]["fitted"] > 0 and res[1]["fitted"] == 0


def test_unknown_protocol_falls_back_to_asynchronous():
    L = make_learner("PA", {}, SP, "cpu")
    assert make_protocol("Bogus", Comm(), L).NAME == "Asynchronous"
    assert make_protocol(None, Comm(), L).NAME == "Asynchronous"


def test_sharded_hubs_world4():
    """HubParallelism 2 of 4 workers: each hub owns half of the model; replicas equal to
    the all-reduce (every-rank-a-hub) result."""
    res_h2 = run(4, "SVM", "Synchronous", {"HubParallelism": 2}, rounds=3)
    res_all = run(4, "SVM", "Synchronous", {}, rounds=3)
    for r in res_h2[1:]:
        assert same(r["final"], res_h2[0]["final"])
    assert same(res_h2[0]["final"], res_all[0]["final"], 1e-5)


def _bucket_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm()
    g = torch.Generator().manual_seed(rank)
    ts = [torch.randn(n, generator=g) for n in (5, 300, 17, 1000, 3)]
    ref = [t.clone() for t in ts]
    for t in ref:
        dist.all_reduce(t)
    for cap, hubs in ((64, 0), (1 << 20, 0), (256, 1)):
        xs = [t.clone() for t in ts]
        comm.all_reduce_coalesced_(xs, hubs=hubs, bucket_bytes=cap)
        for x, r in zip(xs, ref):
            assert torch.allclose(x, r, atol=1e-5), (cap, hubs)
    torch.save({"ok": True, "collectives": comm.stats.collectives}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_coalesced_buckets_world2():
    """bucketBytes caps a coalesced collective; small caps split (and slice) buffers,
    results equal plain per-tensor all-reduces."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_bucket_worker, args=(2, _free_port(), d), nprocs=2,
                           start_method="fork")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    assert all(r["ok"] for r in res)
    assert res[0]["collectives"] > 3  # the 64-byte cap produced many buckets


def test_synchronous_world8_pipelined_and_sharded():
    """8 ranks (the size of one MI355X node): all-reduce, pipelined key-range slices and
    4 sharded hubs give the same replicas."""
    base = run(8, "SVM", "Synchronous", {}, rounds=2, B=128)
    piped = run(8, "SVM", "Synchronous", {"reduceParts": 4}, rounds=2, B=128)
    sharded = run(8, "SVM", "Synchronous", {"HubParallelism": 4}, rounds=2, B=128)
    for res in (base, piped, sharded):
        for r in res[1:]:
            assert same(r["final"], res[0]["final"])
    assert same(piped[0]["final"], base[0]["final"], 1e-6)
    assert same(sharded[0]["final"], base[0]["final"], 1e-5)


def test_ssp_world8_replicas_agree():
    res = run(8, "PA", "SSP", {"staleness": 2, "HubParallelism": 3}, rounds=4, B=128)
    for r in res[1:]:  # three hub shards, every rank installed all of them
        assert same(r["final"], res[0]["final"])


def _ckpt_worker(rank, world, port, out, learner, proto, cfg, rounds, split, B, task):
    """Run ``rounds`` rounds; when ``split`` ≥ 0 checkpoint after that many rounds, build a
    fresh learner + protocol from the saved state (a restore) and continue on it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["OMLDM_CPU_THREADS"] = "1"
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm()
    L = make_learner(learner, {}, SP, "cpu")
    P = make_protocol(proto, comm, L, cfg, spokes=2, max_msg_params=1000)
    for r in range(rounds):
        if r == split:
            f = os.path.join(out, f"ck{rank}.pt")
            torch.save({"learner": L.state_dict(), "protocol": P.state_dict()}, f)
            sd = torch.load(f, weights_only=True)
            L = make_learner(learner, {}, SP, "cpu")
            P = make_protocol(proto, comm, L, cfg, spokes=2, max_msg_params=1000)
            L.load_state_dict(sd["learner"])
            P.load_state_dict(sd["protocol"])
        b = synth_batch(SP, B, start=(r * world + rank) * B, task=task)
        P.round(b)
    torch.save({"E": P._E.clone(), "final": L.state_vector().clone(),
                "stats": P.stats.as_dict()}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run_ckpt(proto, cfg, split, learner="ORR", rounds=8, task=1):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ckpt_worker, args=(2, _free_port(), d, learner, proto, cfg, rounds,
                                               split, 128, task), nprocs=2, start_method="fork")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]


@pytest.mark.parametrize("proto", ["GM", "FGM"])
def test_monitoring_protocols_checkpoint_mid_run(proto):
    """A GM/FGM checkpoint taken between syncs (local models differ) restores the shared
    estimate E and the round state: the estimates stay bitwise equal on all ranks and
    the run is bitwise the run without the restore."""
    cfg = {"threshold": 0.02, "epsilon": 0.02}
    ref = _run_ckpt(proto, cfg, split=-1)
    res = _run_ckpt(proto, cfg, split=3)
    assert torch.equal(res[0]["E"], res[1]["E"])
    for r in range(2):
        assert torch.equal(res[r]["E"], ref[r]["E"])
        assert torch.equal(res[r]["final"], ref[r]["final"])
        assert res[r]["stats"]["syncs"] == ref[r]["stats"]["syncs"]
    assert ref[0]["stats"]["syncs"] >= 1
