"""Failure detection, fault injection and restart-from-checkpoint, on CPU
ranks with gloo: a rank is killed mid-stream, the supervisor relaunches the job from the
last checkpoint on FEWER ranks, and the stream is consumed exactly once."""
import json
import os
import socket
import time

import pytest

from omldm_amd import launch
from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import Consumer, FileBroker
from omldm_amd.utils.fault import FaultPlan, Watchdog


def test_fault_plan_parsing_and_drop():
    fp = FaultPlan("kill:rank=1:tick=3; drop:rank=0:tag=push:every=2; delay:rank=0:ms=1",
                   rank=0, attempt=0)
    assert [r["kind"] for r in fp.rules] == ["drop", "delay"]
    assert [fp.drop("push") for _ in range(4)] == [False, True, False, True]
    assert not fp.drop("sync")
    assert not FaultPlan("kill:rank=0:tick=1", rank=0, attempt=1)  # attempt-0 only


def test_watchdog_fires_without_beats():
    hit = []
    wd = Watchdog(0.2, on_expire=lambda: hit.append(1))
    time.sleep(0.6)
    assert hit == [1] and wd.expired
    ok = []
    wd2 = Watchdog(0.3, on_expire=lambda: ok.append(1))
    for _ in range(8):
        wd2.beat()
        time.sleep(0.05)
    wd2.stop()
    assert not ok


def test_dropped_push_loses_contribution():
    import torch

    from omldm_amd.parallel.comm import Comm

    c = Comm()
    c.fault = FaultPlan("drop:tag=push", rank=0, attempt=0)
    t = torch.ones(4)
    c.all_reduce_(t, tag="push")
    assert float(t.sum()) == 0.0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_kill_rank_restart_on_fewer_ranks(tmp_path):
    data = tmp_path / "topics"
    br = FileBroker(str(data))
    sp = FeatureSpace(13, 0, 26, 1 << 14)
    br.create_topic("trainingData", 4)
    recs = synth_json_records(6000, sp, seed=3)
    for i, r in enumerate(recs):
        br.produce("trainingData", r, partition=i % 4)
    br.produce("requests", json.dumps({"id": 1, "request": "Create", "learner": {"name": "PA"},
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))
    addr = f"file://{data}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(sp.dim), "--device", "cpu", "--batchSize", "100",
             "--timeout", "2000", "--checkpointing", "true", "--checkInterval", "0",
             "--stateBackend", str(tmp_path / "ckpt"), "--watchdogTimeout", "60000",
             "--jobName", "fault-test", "--faults", "kill:rank=1:tick=8", "--parseThreads", "2"]
    env_before = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        logs = []
        rc = launch.supervise(2, args, max_restarts=2, min_nproc=1, shrink=True, port=_port(),
                              log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    assert any("exited with 17" in m for m in logs), logs
    assert any("on 1 rank(s)" in m for m in logs), logs
    perf = Consumer(br, "performance", all_partitions=True).poll(10)
    js = json.loads(perf[-1])
    # JobStatistics.parallelism is the spoke parallelism (16 spokes on the one rank left)
    assert js["jobName"] == "fault-test" and js["parallelism"] == 16
    assert js["metrics"]["ranks"] == 1
    st = js["statistics"][0]
    # every partition fully consumed; the restored rank trained on the rest of the stream
    man = sorted((tmp_path / "ckpt").glob("ckpt-*/manifest.json"))[-1]
    assert json.loads(man.read_text())["world"] == 1
    assert st["score"] > 0.7
