#!/usr/bin/env python3
"""Asynchronous / SSP rounds per second in a 2-rank one-GPU rehearsal, per data plane.

Two ranks (torch.distributed.run, gloo control group) both on cuda:0, each training an
SVM (PA-I) on its own synthetic stream through the Asynchronous or SSP protocol
(parallel/protocols.py → parallel/p2p.py AsyncPS) for ``--seconds``; rank 1 optionally
sleeps ``--slow`` ms per round (a straggler). Per (protocol, plane):
rounds/s per rank and in total, pushes/s (models exchanged with the hub), the host time
spent inside the exchange per round (``AsyncPS.step``), and the final model's accuracy.

Planes: ``signal`` — push/reply control words in HBM, decided on the device (no host
message per push); ``device`` — the same IPC mailboxes with a gloo header per push and
reply on host threads; ``host`` — CPU tensors over gloo.

    python bench/async_rehearsal.py [--seconds 3 --batch 131072 --spokes 16 --log2 20]
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent(r"""
    import json, os, sys, time
    sys.path.insert(0, sys.argv[1])
    import torch
    import torch.distributed as dist
    from omldm_amd.api.batch import FeatureSpace
    from omldm_amd.io.synthetic import synth_batch
    from omldm_amd.models.linear import SVM
    from omldm_amd.ops import linear as L
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import make_protocol

    proto_name, seconds, slow_ms, batch, log2 = (sys.argv[2], float(sys.argv[3]),
                                                 float(sys.argv[4]), int(sys.argv[5]),
                                                 int(sys.argv[6]))
    outdir, spokes = sys.argv[7], int(sys.argv[8])
    dist.init_process_group("gloo")
    comm = Comm()
    rank, world = comm.rank, comm.world
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    # the bench geometry: the engine's field-aware wire (the rounds take the v3 table scan)
    space = FeatureSpace(13, 0, 26, 1 << log2, field_aware=True)
    lrn = SVM({"variant": "PA-I"}, space, dev)
    proto = make_protocol(proto_name, comm, lrn, {"virtualSpokes": spokes, "staleness": 2,
                                                  "_tag": 5})
    pool = [synth_batch(space, batch, start=(k * world + rank) * batch, seed=31).to(dev)
            for k in range(8)]
    for k in range(3):  # warm-up (kernels, mailboxes)
        proto.round(pool[k])
    proto.finalize()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    ps = getattr(proto, "_ps", None)
    t_ex = 0.0
    step0 = ps.step if ps is not None else None

    def timed(x):
        global t_ex
        t = time.perf_counter()
        out = step0(x)
        t_ex += time.perf_counter() - t
        return out

    if ps is not None:
        ps.step = timed
    def pushes_now():  # pushes sent so far (the signal plane counts them on the device)
        if ps is not None and ps.plane == "signal":
            return int(ps._sig.st[ps._sig.W_PUSHES].item())
        return proto.stats.syncs

    syncs0 = pushes_now()
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        proto.round(pool[k % len(pool)])
        if rank == 1 and slow_ms > 0:
            if dev.type == "cuda":
                torch.cuda.current_stream().synchronize()
            time.sleep(slow_ms / 1e3)
        k += 1
    if dev.type == "cuda":
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    pushes = pushes_now() - syncs0
    # Python calls made by the exchange per round (every thread): 50 more rounds profiled
    import threading
    calls = [0]

    def prof(frame, event, arg):
        if event == "call":
            calls[0] += 1

    n_prof = 50 if ps is not None else 0
    if ps is not None:
        ps.step = step0
    for j in range(n_prof):
        sys.setprofile(prof)
        threading.setprofile(prof)
        ps.step(lrn.state_vector())
        sys.setprofile(None)
        threading.setprofile(None)
        proto.learner.fit(pool[j % len(pool)], proto._ctx())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    proto.finalize()
    test = synth_batch(space, 20000, start=10**9, seed=31).to(dev)
    acc = float(((L.linear_predict(lrn.w, test) >= 0).float() * 2 - 1 == test.y).float().mean())
    out = {"rank": rank, "rounds": k, "elapsed_s": el, "rounds_per_s": k / el,
           "pushes": pushes, "exchange_host_us_per_round": 1e6 * t_ex / max(1, k),
           "plane": ps.plane if ps is not None else "collective", "acc": acc,
           "python_calls_per_exchange": calls[0] / n_prof if n_prof else None}
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
""")


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_one(proto: str, plane: str, a) -> dict:
    outdir = tempfile.mkdtemp(prefix="omldm_rehearsal_")
    script = os.path.join(outdir, "worker.py")
    with open(script, "w") as f:
        f.write(WORKER)
    env = dict(os.environ, OMLDM_P2P_PLANE=plane, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), script, ROOT, proto,
           str(a.seconds), str(a.slow), str(a.batch), str(a.log2), outdir, str(a.spokes)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=a.seconds * 4 + 240,
                         env=env)
    if out.returncode != 0:
        return {"error": out.stderr[-2000:]}
    ranks = []
    for r in range(2):
        with open(os.path.join(outdir, f"rank{r}.json")) as f:
            ranks.append(json.load(f))
    tot = sum(x["rounds_per_s"] for x in ranks)
    return {"plane": ranks[0]["plane"], "rounds_per_s_total": round(tot, 1),
            "rounds_per_s": [round(x["rounds_per_s"], 1) for x in ranks],
            "examples_per_s_total": round(tot * a.batch, 1),
            "pushes_per_s": [round(x["pushes"] / x["elapsed_s"], 1) for x in ranks],
            "exchange_host_us_per_round": [round(x["exchange_host_us_per_round"], 1)
                                           for x in ranks],
            "acc": [round(x["acc"], 4) for x in ranks],
            "python_calls_per_exchange": [x["python_calls_per_exchange"] for x in ranks]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--batch", type=int, default=131072, help="records per round per rank")
    ap.add_argument("--spokes", type=int, default=16, help="virtual spokes per rank")
    ap.add_argument("--log2", type=int, default=20, help="hashed feature space 2^log2")
    ap.add_argument("--slow", type=float, default=0.0, help="rank 1 sleeps this many ms/round")
    ap.add_argument("--protos", default="Synchronous,Asynchronous,SSP")
    ap.add_argument("--planes", default="signal,device")
    a = ap.parse_args(argv)
    res = {"metric": "Asynchronous / SSP rounds per second, 2 ranks on one MI355X (rehearsal)",
           "batch": a.batch, "features": 1 << a.log2, "seconds": a.seconds, "slow_ms": a.slow,
           "runs": {}}
    for proto in a.protos.split(","):
        for plane in (a.planes.split(",") if proto != "Synchronous" else ["signal"]):
            key = proto if proto == "Synchronous" else f"{proto}/{plane}"
            res["runs"][key] = run_one(proto, plane, a)
            sys.stderr.write(f"{key}: {res['runs'][key]}\n")
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
