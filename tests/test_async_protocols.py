"""Genuinely asynchronous Asynchronous and SSP protocols (parallel/p2p.py) on gloo, three
ranks, one of them a straggler (50 ms per round).

Reference: AsynchronousWorker / SSPWorker get unicast hub replies with no barrier
(FlinkNetwork.scala:262-271, MLNodeGenerator.scala:26-33,55-62); an SSP hub withholds the
reply of a worker more than ``staleness`` clocks ahead of the slowest.
"""
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent(r"""
    import json, os, sys, time
    sys.path.insert(0, sys.argv[1])
    import torch
    import torch.distributed as dist
    from omldm_amd.api.batch import FeatureSpace
    from omldm_amd.io.synthetic import synth_raw
    from omldm_amd.models.linear import SVM
    from omldm_amd.ops import linear as L
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import make_protocol

    proto_name, seconds, slow = sys.argv[2], float(sys.argv[3]), int(sys.argv[4])
    dev = sys.argv[6]  # "cpu", or "cuda": every rank on cuda:0, the device data plane
    dist.init_process_group("gloo")
    comm = Comm()
    rank, world = comm.rank, comm.world
    space = FeatureSpace(13, 0, 26, 1 << 12)
    lrn = SVM({"variant": "PA-I"}, space, dev)
    cfg = {"virtualSpokes": 2, "staleness": 2, "_tag": 3}
    proto = make_protocol(proto_name, comm, lrn, cfg)
    pool = [synth_raw(space, 256, start=(k * world + rank) * 256, seed=25).hashed(space).to(dev)
            for k in range(16)]
    dist.barrier()
    t0 = time.time()
    k = 0
    fixed = proto_name == "Synchronous"  # collectives: every rank runs the same rounds
    import threading
    threads = 0
    while (k < 20) if fixed else (time.time() - t0 < seconds):
        proto.round(pool[k % len(pool)])
        if rank == slow:
            time.sleep(0.05)
        k += 1
        threads = max(threads, threading.active_count())
    proto.finalize()
    elapsed = time.time() - t0
    test = synth_raw(space, 4000, start=10**9, seed=25).hashed(space).to(dev)
    acc = float(((L.linear_predict(lrn.w, test) >= 0).float() * 2 - 1 == test.y).float().mean())
    ps = getattr(proto, "_ps", None)
    out = {"rank": rank, "rounds": k, "elapsed": elapsed, "acc": acc, "w0": float(lrn.w[5]),
           "max_lead": getattr(proto, "max_lead", None),
           "plane": ps.plane if ps is not None else None,
           "w": lrn.w.detach().cpu().tolist(),
           "events": [e[0] for e in ps.events] if ps is not None else [],
           "merges": ps.merges if ps is not None else [],
           "reply_after": {str(k): v for k, v in ps.reply_after.items()} if ps is not None else {},
           "scale": ps.scale if ps is not None else None,
           "collectives": comm.stats.collectives,
           "push_msg_bytes": comm.stats.per_tag.get("async-push", 0),
           "threads": threads, "syncs": proto.stats.syncs}
    with open(os.path.join(sys.argv[5], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(proto, seconds=2.5, slow=1, world=3, dev="cpu", plane=None):
    outdir = tempfile.mkdtemp(prefix="omldm_async_")
    script = os.path.join(outdir, "worker.py")
    with open(script, "w") as f:
        f.write(WORKER)
    env = dict(os.environ, OMP_NUM_THREADS="1", OMLDM_CPU_THREADS="1")
    if plane is not None:
        env["OMLDM_P2P_PLANE"] = plane
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
                          "--master-port", str(_port()), script, ROOT, proto, str(seconds),
                          str(slow), outdir, dev], capture_output=True, text=True, timeout=120,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = {}
    for r in range(world):
        with open(os.path.join(outdir, f"rank{r}.json")) as f:
            res[r] = json.load(f)
    shutil.rmtree(outdir, ignore_errors=True)
    return res


def _replay(res, world=3, dev="cpu"):
    """Deterministic host replay of a logged Asynchronous / SSP run (parallel/p2p.py event
    log): every worker's rounds, pushes and installs re-run on the CPU in the order the
    hub merged the pushes; the n-th install of worker r takes the hub model as it stood
    after reply_after[r][n] merges. Returns the hub's final global model."""
    import torch

    from omldm_amd.api.batch import FeatureSpace
    from omldm_amd.io.synthetic import synth_raw
    from omldm_amd.models.base import RoundContext
    from omldm_amd.models.linear import SVM

    space = FeatureSpace(13, 0, 26, 1 << 12)
    ctx = RoundContext(spokes=2, inv_p=1.0)
    hub = res[0]
    scale = hub["scale"]
    pools = {r: [synth_raw(space, 256, start=(k * world + r) * 256, seed=25).hashed(space).to(dev)
                 for k in range(16)] for r in range(world)}
    lrn = {r: SVM({"variant": "PA-I"}, space, dev) for r in range(world)}
    x0 = lrn[0].w.clone()
    glob = x0.clone()
    snaps = [glob.clone()]
    st = {r: {"cur": 0, "k": 0, "inst": 0, "base": x0.clone(), "x_push": None, "pushes": 0}
          for r in range(world)}

    def advance(r, until_push=True):
        """Run worker r's events up to (and including) its next push; its δ."""
        s, ev, L = st[r], res[r]["events"], lrn[r]
        while s["cur"] < len(ev):
            e = ev[s["cur"]]
            s["cur"] += 1
            if e == "step":  # the round trained just before this step
                L.fit(pools[r][s["k"] % 16], ctx)
                s["k"] += 1
            elif e == "install":
                m = hub["reply_after"][str(r)][s["inst"]]
                s["inst"] += 1
                assert m < len(snaps), (r, m, len(snaps))
                snap = snaps[m]
                L.w.copy_(snap + (L.w - s["x_push"]))
                s["base"] = snap.clone()
                L.on_state_loaded()
            else:  # "push" / "final"
                delta = L.w - s["base"]
                s["x_push"] = L.w.clone()
                s["pushes"] += 1
                if until_push:
                    return delta
        assert not until_push, f"worker {r}: no push left to merge"
        return None

    for r, clock in hub["merges"]:
        delta = advance(r)
        assert st[r]["pushes"] == clock, (r, clock, st[r]["pushes"])
        glob.add_(delta, alpha=scale)
        snaps.append(glob.clone())
    for r in range(world):  # the final replies' installs
        advance(r, until_push=False)
    assert all(st[r]["k"] == res[r]["rounds"] for r in range(world))
    return glob.cpu()


def test_asynchronous_straggler_does_not_stall_fast_workers():
    r = _run("Asynchronous")
    slow = r[1]["rounds"]
    assert r[0]["rounds"] >= 3 * slow and r[2]["rounds"] >= 3 * slow, r
    # after finalize every rank holds the hub's global model, and it learned
    assert r[0]["w0"] == r[1]["w0"] == r[2]["w0"]
    assert min(x["acc"] for x in r.values()) > 0.7, r
    # ... and that model is exactly the deterministic replay of the logged event order
    want = _replay(r)
    for x in r.values():
        np.testing.assert_allclose(np.asarray(x["w"], dtype=np.float32), want.numpy(),
                                   rtol=0, atol=1e-6)


def test_ssp_bounds_the_lead_over_the_straggler():
    r = _run("SSP")
    slow = r[1]["rounds"]
    # the hub answers a worker only within 2 clocks of the slowest: the fast workers' rounds
    # stay within the bound (+1 for the push in flight, +1 for the final round)
    assert r[0]["rounds"] <= slow + 2 + 2 and r[2]["rounds"] <= slow + 2 + 2, r
    assert r[0]["max_lead"] <= 2, r  # rank 0 is the hub: the leads it answered
    assert r[0]["w0"] == r[1]["w0"] == r[2]["w0"]
    assert min(x["acc"] for x in r.values()) > 0.6, r
    want = _replay(r)
    for x in r.values():
        np.testing.assert_allclose(np.asarray(x["w"], dtype=np.float32), want.numpy(),
                                   rtol=0, atol=1e-6)


def test_synchronous_is_paced_by_the_straggler_for_contrast():
    r = _run("Synchronous")
    # 20 lock-step rounds: the fast ranks wait out the straggler's 20 x 50 ms
    assert r[0]["elapsed"] >= 0.9 and r[2]["elapsed"] >= 0.9, r
    assert r[0]["w0"] == r[1]["w0"] == r[2]["w0"]


@pytest.mark.gpu
@pytest.mark.parametrize("plane", ["signal", "device"])
@pytest.mark.parametrize("proto", ["Asynchronous", "SSP"])
def test_device_plane_on_gpu(proto, plane):
    """Three ranks on cuda:0: pushes and replies move through the IPC mailboxes (no
    model-sized host copy per round); same protocol guarantees as on the host plane.
    ``signal`` (the default): the push / reply control words travel in HBM too — no gloo
    header and no host thread per push; ``device``: headers on gloo."""
    r = _run(proto, seconds=2.0, dev="cuda", plane=plane)
    assert all(x["plane"] == plane for x in r.values()), r
    if plane == "signal":
        assert all(x["push_msg_bytes"] == 0 for x in r.values()), r
        # no channel-service or request threads: the main thread (+ the runtime's own)
        assert max(x["threads"] for x in r.values()) <= 3, [x["threads"] for x in r.values()]
        assert all(x["syncs"] > 0 for x in r.values()), r
    assert r[0]["w0"] == r[1]["w0"] == r[2]["w0"]
    slow = r[1]["rounds"]
    if proto == "SSP":
        assert r[0]["rounds"] <= slow + 4 and r[0]["max_lead"] <= 2, r
    else:
        assert r[0]["rounds"] >= 3 * slow and r[2]["rounds"] >= 3 * slow, r
    assert min(x["acc"] for x in r.values()) > 0.6, r
    # the device plane's merges / installs against the logged order replayed with the same
    # GPU learners (the rounds' fp32 atomics may reorder: a tolerance, not bit equality)
    want = _replay(r, dev="cuda")
    got = np.asarray(r[0]["w"], dtype=np.float32)
    np.testing.assert_allclose(got, want.numpy(), rtol=1e-3,
                               atol=1e-4 * max(1.0, float(np.abs(got).max())))
