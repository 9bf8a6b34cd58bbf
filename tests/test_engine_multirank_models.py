"""What the multi-rank engine's models hold, not only that it ran (gloo, CPU, one process
per rank through the supervisor).

* Synchronous pipelines: after EVERY training tick every rank holds the same replica
  (the per-tick model digests the job writes under OMLDM_TRACE_MODELS agree bit for bit),
  with 2 and 4 ranks;
* the model a G-rank job ends with scores within 0.5 accuracy points of the same stream
  trained at the same total spoke count P = S·G on one rank (the reference's P spokes,
  FlinkSpoke.scala:92-107, with the Synchronous hub averaging their replicas), on a
  fresh test set.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

from omldm_amd import launch
from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.parse import parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import FileBroker
from omldm_amd.ops import linear as L

SP = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
N_TRAIN = 24000
P_TOTAL = 8


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _topics(root):
    br = FileBroker(str(root))
    br.create_topic("trainingData", 8)
    for i, r in enumerate(synth_json_records(N_TRAIN, SP, seed=11)):
        br.produce("trainingData", r, partition=i % 8)
    for pid, learner, proto in ((1, "SVM", "Synchronous"), (2, "PA", "FGM")):
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create", "learner": {"name": learner},
            "trainingConfiguration": {"protocol": proto}}))
    return br


def _run(tmp_path, world):
    data = tmp_path / f"topics{world}"
    _topics(data)
    trace = tmp_path / f"trace{world}"
    addr = f"file://{data}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--fieldAware", "true", "--device", "cpu",
             "--batchSize", "1000", "--timeout", "1500", "--parallelism", str(P_TOTAL),
             "--testSetSize", "64", "--parseThreads", "2", "--watchdogTimeout", "120000"]
    env_before = dict(os.environ)
    os.environ.update(OMP_NUM_THREADS="1", OMLDM_TRACE_MODELS=str(trace))
    try:
        logs = []
        rc = launch.supervise(world, args, max_restarts=0, min_nproc=world, port=_port(),
                              log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    digests = []
    for r in range(world):
        with open(trace / f"rank{r}.jsonl") as f:
            digests.append([json.loads(x) for x in f])
    final = {r: torch.load(trace / f"rank{r}_final_1.pt", weights_only=True)
             for r in range(world)}
    return digests, final


def _accuracy(w):
    fc = synth_json_records(6000, SP, start=10**7, seed=11)
    batch, _, _ = parse_records(fc, SP)
    s = L.linear_predict(w, batch.without_raw())
    return float(((s >= 0).float() * 2 - 1 == batch.y).float().mean())


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_replicas_agree_every_tick_and_accuracy_matches_one_rank(tmp_path, world):
    digests, final = _run(tmp_path, world)
    # the ranks train the same ticks (the flag all-reduce decides), so the traces align
    n = len(digests[0])
    assert n >= 2 and all(len(d) == n for d in digests), [len(d) for d in digests]
    sync_ticks = 0
    for k in range(n):
        recs = [d[k] for d in digests]
        assert len({(r["tick"], r["pid"]) for r in recs}) == 1, recs
        if recs[0]["protocol"] == "Synchronous":
            assert len({r["crc"] for r in recs}) == 1, (k, recs)
            sync_ticks += 1
    assert sync_ticks >= 2
    for r in range(1, world):
        assert torch.equal(final[r], final[0])
    # the same stream on one rank with P = S·G spokes
    one, final1 = _run(tmp_path, 1)
    acc_g, acc_1 = _accuracy(final[0]), _accuracy(final1[0])
    assert acc_1 > 0.75, acc_1
    assert abs(acc_g - acc_1) <= 0.005, (acc_g, acc_1)
