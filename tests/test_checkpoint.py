"""Checkpoint writer semantics: the snapshot is taken when save() returns even
though the file is written later, and a crashed attempt's leftover files never complete a
manifest."""
import json
import os
import uuid

import torch

from omldm_amd.utils.checkpoint import Checkpointer, host_copy
from tests.test_engine import SP, create, make_job
from omldm_amd.io.synthetic import synth_json_records


def test_host_copy_is_deep_and_detached():
    t = torch.arange(4.0)
    sd = {"a": t, "b": [t, (t, 3)], "c": "x"}
    c = host_copy(sd)
    t += 100
    assert torch.equal(c["a"], torch.arange(4.0)) and torch.equal(c["b"][1][0], torch.arange(4.0))
    assert c["b"][1][1] == 3 and c["c"] == "x"


def test_snapshot_is_not_torn_by_later_ticks(tmp_path):
    name = uuid.uuid4().hex
    ck = ["--checkpointing", "true", "--checkInterval", "3600000", "--stateBackend",
          f"file://{tmp_path}"]
    job, br, _ = make_job(ck, name=name)
    for r in synth_json_records(900, SP):
        br.produce("trainingData", r)
    create(br, 1, "SVM", pre=["StandardScaler"])
    for _ in range(3):
        job.tick()
    sd_now = host_copy(job.state_dict())
    job.checkpointer.wait()
    # hold the writer until live state has changed in place
    import threading

    gate = threading.Event()
    real = torch.save

    def slow_save(obj, f, *a, **k):
        gate.wait(10)
        return real(obj, f, *a, **k)

    torch.save = slow_save
    try:
        d = job.checkpointer.save(job)
        sc = job.pipes[1].preprocessors[0]
        for v in sc.state_dict().values():
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                v.add_(1000.0)
        ring = job.holdout.state_dict()
        for v in ring.values():
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                v.add_(1000.0)
    finally:
        gate.set()
        job.checkpointer.wait()
        torch.save = real
    saved = torch.load(os.path.join(d, "rank-0.pt"), weights_only=True)

    def same(a, b):
        if isinstance(a, torch.Tensor):
            if a.is_floating_point():
                return a.shape == b.shape and torch.allclose(a, b, rtol=0, atol=0, equal_nan=True)
            return torch.equal(a, b)
        if isinstance(a, dict):
            return a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
        if isinstance(a, (list, tuple)):
            return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
        return a == b

    assert same(saved["pipelines"][1]["preprocessors"], sd_now["pipelines"][1]["preprocessors"])
    assert same(saved["holdout"], sd_now["holdout"])


def test_stale_done_markers_do_not_complete_a_manifest(tmp_path):
    """A crash left rank-1's files of checkpoint N; the restarted job's rank 0 must not
    publish N's manifest from them."""

    class Cfg:
        stateBackend = f"file://{tmp_path}"
        checkInterval = 0
        checkpointExport = False

    class FakeJob:
        ticks = 7
        pipes: dict = {}

        def state_dict(self):
            return {"w": torch.ones(3)}

    ck = Checkpointer(Cfg(), 0, 2, nonce="run2")
    ck.WAIT_S = 0.5
    d = tmp_path / "ckpt-000000"
    d.mkdir()
    (d / "rank-1.pt").write_bytes(b"old")
    (d / "rank-1.done").write_text("1")  # round-3 style marker of a crashed attempt
    ck.save(FakeJob())
    try:
        ck.wait()
        raise AssertionError("rank 0 published a manifest from stale files")
    except RuntimeError as e:
        assert "did not finish" in str(e)
    assert not (d / "manifest.json").exists()
    # the live rank 1 of the same attempt completes it
    # an earlier RUN's marker for the same index and tick (a deterministic replay reaches
    # index 0 at tick 7 again) does not match this run's attempt either
    (d / "rank-1.done").write_text("run1:0:7")
    ck.n = 0
    ck.save(FakeJob())
    try:
        ck.wait()
        raise AssertionError("rank 0 published a manifest from an earlier run's marker")
    except RuntimeError as e:
        assert "did not finish" in str(e)
    assert not (d / "manifest.json").exists()
    # the live rank 1 of the same attempt (same run nonce, broadcast by the Job) completes it
    ck1 = Checkpointer(Cfg(), 1, 2, nonce="run2")
    ck1.n = 0
    ck.n = 0
    ck.WAIT_S = 30
    ck.save(FakeJob())
    ck1.save(FakeJob())
    ck1.wait()
    ck.wait()
    man = json.loads((d / "manifest.json").read_text())
    assert man["attempt"] == "run2:0:7" and man["world"] == 2
