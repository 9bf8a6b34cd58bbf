"""The per-record forecasting lane on a CPU job (engine/forecast_server.py without the
serving wave): every pipeline kind answers each forecasting record on the lane as it
arrives (FlinkSpoke.scala:101-105 → FlinkNetwork.scala:243-257), equal to the batched
predict; records that arrive before any pipeline wait in a bounded queue and are answered
by the first tick after a Create; a checkpoint saves answered offsets + the waiting
records, so a restore neither skips nor repeats a forecast."""
import json
import uuid

import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.io.parse import parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

SP = FeatureSpace(13, 0, 26, 1 << 16)


def _job(name=None, extra=()):
    name = name or uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--batchSize", "2000", "--timeout", "300",
             "--parallelism", "4", "--forecastServer", "true", *extra]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    return Job(cfg, Comm(), "cpu"), br


def _create(br, pid, name, hyper=None, pre=None):
    br.produce("requests", json.dumps({
        "id": pid, "request": "Create", "learner": {"name": name, "hyperParameters": hyper or {}},
        "preProcessors": [{"name": p} for p in (pre or [])],
        "trainingConfiguration": {"protocol": "Synchronous"}}))


def test_lane_answers_every_pipeline_kind_per_record():
    job, br = _job()
    specs = [(1, "SVM", None, None), (2, "PA", None, ["StandardScaler"]),
             (3, "NN", {"hiddenLayers": [8]}, None), (4, "ORR", None, ["MinMaxScaler"]),
             (5, "K-means", {"k": 3}, None), (6, "HT", {"nClasses": 2}, None)]
    for pid, name, hyper, pre in specs:
        _create(br, pid, name, hyper, pre)
    for r in synth_json_records(3000, SP):
        br.produce("trainingData", r)
    for _ in range(3):
        job.tick()
    fs = job.fserver
    assert fs is not None and fs.serving and fs._spec is None
    assert [pid for pid, _ in fs._direct] == [1, 2, 3, 4, 5, 6]
    fc = synth_json_records(9, SP, start=50000, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    job.tick()
    assert fs.served == 9 and not fs.fallback
    preds = [json.loads(x) for x in br.records("predictions")]
    assert len(preds) == 6 * 9
    batch, _, _ = parse_records(fc, job.space)
    batch = batch.without_raw()
    for pid, name, _, _ in specs:
        want = job.pipes[pid].predict(batch).float()
        got = torch.tensor([p["prediction"] for p in preds if p["mlpId"] == pid])
        assert torch.allclose(got, want, rtol=1e-5, atol=1e-5), (name, got, want)
        assert [p["dataPoint"] for p in preds if p["mlpId"] == pid] == [json.loads(r) for r in fc]
    fam = fs.family_percentiles()
    assert {"SVM", "PA", "NN", "ORR", "K-means", "HT"} <= set(fam), fam
    job.fserver.close()


def test_records_before_any_pipeline_wait_bounded_then_are_answered():
    job, br = _job(extra=["--recordBufferSize", "5"])
    fc = synth_json_records(8, SP, start=10, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    job.tick()
    job.fserver.catch_up()
    job.tick()  # no pipeline: kept, at most recordBufferSize of them
    assert len(job.fserver.fallback) == 5 and job.counters["dropped_buffer"] == 3
    _create(br, 1, "SVM")
    job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert [p["dataPoint"] for p in preds] == [json.loads(r) for r in fc[3:]]
    job.fserver.close()


def test_checkpoint_keeps_waiting_forecasts_and_answered_offsets(tmp_path):
    name = uuid.uuid4().hex
    extra = ["--checkpointing", "true", "--checkInterval", "0", "--stateBackend",
             f"file://{tmp_path}"]
    job, br = _job(name, extra)
    fc = synth_json_records(4, SP, start=10, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    job.tick()
    assert job.fserver.catch_up()
    done, pending = job.fserver.snapshot()
    assert sum(done.values()) == 4 and len(pending) == 4  # polled, handed back, waiting
    sd = job.state_dict()
    assert sd["consumers"]["forecast"]["offsets"] == done
    assert [json.loads(r) for r in sd["forecast_pending"]] == [json.loads(r) for r in fc]
    job.checkpointer.save(job)
    job.checkpointer.wait()
    job.fserver.close()
    job2, br2 = _job(name, ["--restore", "true", "--stateBackend", f"file://{tmp_path}"])
    assert len(job2.fserver.fallback) == 4
    _create(br2, 1, "SVM")
    job2.tick()
    job2.tick()
    preds = [json.loads(x) for x in br2.records("predictions")]
    assert [p["dataPoint"] for p in preds] == [json.loads(r) for r in fc]  # once each
    job2.fserver.close()
