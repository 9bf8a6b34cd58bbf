"""End-to-end engine tests on the in-process broker (CPU): the reference's request →
train → forecast → query → termination flow, record buffering, holdout semantics,
checkpoint/restore (with the spoke pipelines restored, SURVEY §2.8 Q1 fixed)."""
import json
import uuid

import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.holdout import HoldoutSet
from omldm_amd.engine.job import Job
from omldm_amd.io.synthetic import synth_batch, synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

SP = FeatureSpace(13, 0, 26, 1 << 16)


def make_job(extra=(), name=None):
    name = name or uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--batchSize", "500", "--timeout", "200",
             "--parallelism", "4", *extra]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 4)
    return Job(cfg, Comm(), "cpu"), br, cfg


def create(br, pid, learner, protocol="Synchronous", pre=None, hyper=None):
    br.produce("requests", json.dumps({
        "id": pid, "request": "Create",
        "learner": {"name": learner, "hyperParameters": hyper or {}},
        "preProcessors": [{"name": p} for p in (pre or [])],
        "trainingConfiguration": {"protocol": protocol}}))


def test_e2e_create_train_forecast_query_terminate():
    job, br, cfg = make_job()
    for r in synth_json_records(1500, SP):
        br.produce("trainingData", r)
    create(br, 1, "SVM", pre=["StandardScaler"])
    create(br, 2, "ORR", "FGM", pre=["PolynomialFeatures"])
    create(br, 3, "K-means", hyper={"k": 3})
    for _ in range(5):
        job.tick()
    assert set(job.pipes) == {1, 2, 3}
    for r in synth_json_records(7, SP, start=50, operation="forecasting"):
        br.produce("forecastingData", r)
    br.produce("requests", json.dumps({"id": 1, "request": "Query", "requestId": 42}))
    for _ in range(3):
        job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert len(preds) == 21 and {p["mlpId"] for p in preds} == {1, 2, 3}
    resp = [json.loads(x) for x in br.records("responses")]
    assert resp[-1]["responseId"] == 42 and resp[-1]["dataFitted"] > 0
    assert 0.0 <= resp[-1]["score"] <= 1.0
    job.run()  # idle timeout → final statistics → performance topic
    assert job.terminated
    perf = json.loads(br.records("performance")[-1])
    assert perf["jobName"] == cfg.jobName
    assert [s["pipeline"] for s in perf["statistics"]] == [1, 2, 3]
    syn = perf["statistics"][0]
    assert syn["protocol"] == "Synchronous" and syn["fitted"] > 0 and syn["modelsShipped"] > 0


def test_records_buffered_until_create_and_delete():
    job, br, _ = make_job()
    for r in synth_json_records(300, SP):
        br.produce("trainingData", r)
    job.tick()
    assert job._buffered == 300 and not job.pipes
    create(br, 5, "PA")
    job.tick()
    job.tick()
    assert job.record_buffer == [] and job.pipes[5].learner.running_totals()["fitted"] > 0
    br.produce("requests", json.dumps({"id": 5, "request": "Delete"}))
    job.tick()
    assert 5 not in job.pipes


def test_update_changes_hyper_parameters():
    job, br, _ = make_job()
    create(br, 1, "PA", hyper={"C": 0.5})
    job.tick()
    br.produce("requests", json.dumps({"id": 1, "request": "Update",
                                       "learner": {"name": "PA", "hyperParameters": {"C": 0.01}}}))
    job.tick()
    assert abs(job.pipes[1].learner.rule.C - 0.01) < 1e-9


def test_invalid_records_counted_not_fatal():
    job, br, _ = make_job()
    create(br, 1, "PA")
    job.tick()
    br.produce("trainingData", "EOS")
    br.produce("trainingData", "{broken")
    br.produce("trainingData", json.dumps({"numericalFeatures": [1.0], "operation": "training"}))
    for r in synth_json_records(10, SP):
        br.produce("trainingData", r)
    job.tick()
    assert job.counters["invalid"] == 3 and job.counters["records"] == 10


def test_holdout_reference_semantics():
    h = HoldoutSet(SP, 4, "cpu")
    b = synth_batch(SP, 10)
    out = h.route(b)
    assert out.B == 8 and h.filled == 2           # positions 8, 9 held out
    out = h.route(synth_batch(SP, 20, start=10))
    assert h.filled == 4 and out.B == 16 + 2      # 4 more held: 2 evictions trained
    big = h.route(synth_batch(SP, 100, start=30))
    assert h.filled == 4 and big.B == 80 + 4 + 16  # 20 held: ring + 16 spill trained
    assert h.test_set().B == 4


def test_checkpoint_restore_roundtrip(tmp_path):
    name = uuid.uuid4().hex
    extra = ["--checkpointing", "true", "--checkInterval", "0", "--stateBackend",
             f"file://{tmp_path}"]
    job, br, _ = make_job(extra, name=name)
    for r in synth_json_records(800, SP):
        br.produce("trainingData", r)
    create(br, 1, "SVM")
    create(br, 2, "HT", hyper={"nClasses": 2})
    for _ in range(4):
        job.tick()
    w = job.pipes[1].learner.state_vector().clone()
    fitted = job.pipes[1].learner.running_totals()["fitted"]
    job.checkpointer.save(job)
    job2, _, _ = make_job(["--restore", "true", "--stateBackend", f"file://{tmp_path}"], name=name)
    assert set(job2.pipes) == {1, 2}
    assert torch.equal(job2.pipes[1].learner.state_vector(), w)
    assert job2.pipes[1].learner.running_totals()["fitted"] == fitted
    assert (job2.holdout.filled == job.holdout.filled).all()
    for a, b in zip(job2.holdout.test_sets(), job.holdout.test_sets()):
        assert torch.equal(a.y, b.y)
    assert job2.train_in.offsets == job.consumer_offsets()["train"]


def test_rescale_owners_partition_old_ranks():
    from omldm_amd.utils.checkpoint import rescale_owners

    for old in (1, 2, 3, 4, 8):
        for new in (1, 2, 3, 4, 8):
            owned = [rescale_owners(old, new, r) for r in range(new)]
            flat = sorted(o for x in owned for o in x)
            assert flat == list(range(old))  # every old rank has exactly one new owner


def test_shrink_restore_merges_buffers_holdout_and_counters(tmp_path):
    """2 → 1 restore: both old ranks' buffered records (taken before any Create), their
    holdout rows and their running counters all land on the single new rank — nothing
    lost, nothing counted twice."""
    import os

    name = uuid.uuid4().hex
    sds = []
    for r in range(2):
        job, br, _ = make_job(["--testSetSize", "16"], name=f"{name}-{r}")
        for rec in synth_json_records(300, SP, seed=r):
            br.produce("trainingData", rec)
        job.tick()                               # no pipeline yet → records buffered
        assert job._buffered == 300
        create(br, 1, "SVM")
        for rec in synth_json_records(200, SP, seed=10 + r):
            br.produce("trainingData", rec)
        job.tick()                               # Create + train (buffer replayed)
        for rec in synth_json_records(150, SP, seed=20 + r):
            br.produce("trainingData", rec)
        sd = job.state_dict()
        sd["record_buffer"] = [s.encode() if isinstance(s, str) else s
                               for s in synth_json_records(40 + r, SP, seed=30 + r)]
        sds.append(sd)
    d = tmp_path / "ckpt-000000"
    d.mkdir()
    for r, sd in enumerate(sds):
        torch.save(sd, os.path.join(d, f"rank-{r}.pt"))
    (d / "manifest.json").write_text(json.dumps({"index": 0, "world": 2, "time": 0,
                                                 "ticks": 2, "pipelines": [1]}))
    job2, _, _ = make_job(["--restore", "true", "--stateBackend", f"file://{tmp_path}",
                           "--testSetSize", "16"], name=f"{name}-new")
    assert job2._buffered == 40 + 41
    fit = [sd["pipelines"][1]["learner"]["cum"][1].item() for sd in sds]
    assert job2.pipes[1].learner.running_totals()["fitted"] == int(sum(fit))
    held = sum(sum(sd["holdout"]["filled"]) for sd in sds)
    spill = job2._restored_train.B if getattr(job2, "_restored_train", None) is not None else 0
    # 2 ranks × 4 spokes → 4 spokes: each new spoke merges two old rings, keeps 16 points
    assert job2.holdout.n_test + spill == held
    assert (job2.holdout.filled == job2.holdout.size).all() and job2.holdout.size == 16
    assert spill == held - 4 * 16 > 0
    assert job2.counters["records"] == sum(sd["counters"]["records"] for sd in sds)
    job2.tick()  # the spilled holdout rows are trained on (not held out again)
    assert job2.pipes[1].learner.running_totals()["fitted"] >= int(sum(fit)) + spill


def test_parallelism_gate_buffers_creates_until_the_job_grows_back(tmp_path):
    """FlinkSpoke.scala:69-71,145-156,345-348: a job restored onto fewer spokes than it
    ran at keeps new Create requests waiting (checkpointed); restored at that parallelism
    or more it creates them first thing, and the recorded parallelism grows with it."""
    name = uuid.uuid4().hex
    ck = ["--checkpointing", "true", "--checkInterval", "0", "--stateBackend",
          f"file://{tmp_path}"]
    job, br, _ = make_job(ck + ["--spokesPerDevice", "8"], name=name)
    create(br, 1, "PA")
    job.tick()
    assert job.spoke_parallelism == 8 and set(job.pipes) == {1}
    job.checkpointer.save(job)
    job.checkpointer.wait()  # the background write is done before the next job restores
    # restored on 4 spokes: pipeline 1 comes back, the new Create waits
    job2, _, _ = make_job(ck + ["--restore", "true", "--spokesPerDevice", "4"], name=name)
    assert job2.parallelism == 4 and job2.spoke_parallelism == 8
    create(br, 2, "SVM")
    job2.tick()
    job2.tick()
    assert set(job2.pipes) == {1} and [m[0] for m in job2.request_buffer] == [2]
    job2.checkpointer.save(job2)
    job2.checkpointer.wait()
    # restored on 16 spokes: the buffered Create is applied, the job records 16
    job3, _, _ = make_job(ck + ["--restore", "true", "--spokesPerDevice", "16"], name=name)
    assert job3.spoke_parallelism == 16 and len(job3.request_buffer) == 1
    job3.tick()
    assert set(job3.pipes) == {1, 2} and job3.request_buffer == []
    # the gate can be switched off
    job4, _, _ = make_job(ck + ["--restore", "true", "--spokesPerDevice", "2",
                                "--parallelismGate", "false"], name=name)
    create(br, 3, "PA")
    job4.tick()
    assert 3 in job4.pipes
