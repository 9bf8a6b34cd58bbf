"""Per-record forecasting on the resident serving wave inside the engine
(engine/forecast_server.py; reference FlinkSpoke.scala:101-105 → FlinkNetwork.scala:243-257).

* every forecasting record gets one Prediction per pipeline, equal to the batched predict
  of the same model;
* pipelines the wave cannot score (a dense learner) send records to the batched path;
* the record-in → Prediction-out latency is measured per record.
"""
import json
import uuid

import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.io.parse import parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

pytestmark = pytest.mark.gpu

SP = FeatureSpace(13, 0, 26, 1 << 18)


def _job(extra=()):
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--batchSize", "2000", "--timeout", "300",
             "--parallelism", "8", *extra]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    return Job(cfg, Comm(), "cuda"), br


def _create(br, pid, learner, hyper=None):
    br.produce("requests", json.dumps({"id": pid, "request": "Create",
                                       "learner": {"name": learner,
                                                   "hyperParameters": hyper or {}},
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))


def test_wave_answers_every_record_like_the_batched_predict():
    job, br = _job()
    assert job.fserver is not None
    _create(br, 1, "SVM")
    _create(br, 2, "PA")
    for r in synth_json_records(6000, SP):
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    assert job.fserver.serving  # both pipelines live in the model store
    fc = synth_json_records(40, SP, start=70000, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert len(preds) == 80
    batch, _, _ = parse_records(fc, SP)
    batch = batch.without_raw().to("cuda")
    for pid in (1, 2):
        want = job.pipes[pid].predict(batch).float().cpu()
        got = torch.tensor([p["prediction"] for p in preds if p["mlpId"] == pid])
        assert torch.equal(got, want), (pid, got, want)
        dps = [p["dataPoint"] for p in preds if p["mlpId"] == pid]
        assert dps == [json.loads(r) for r in fc]  # the DataInstance is echoed in order
    lat = job.fserver.latency_percentiles()
    assert lat["n"] == 40 and lat["p50"] is not None and lat["p50"] < 5000, lat
    job.run()
    perf = json.loads(br.records("performance")[-1])
    assert perf["metrics"]["forecastRecordLatencyUs"]["n"] == 40


def test_dense_pipeline_sends_records_to_the_batched_path():
    job, br = _job()
    _create(br, 1, "SVM")
    _create(br, 2, "NN", {"hiddenLayers": [8]})
    for r in synth_json_records(4000, SP):
        br.produce("trainingData", r)
    for _ in range(3):
        job.tick()
    assert not job.fserver.serving  # the NN is not in the model store
    for r in synth_json_records(10, SP, start=50000, operation="forecasting"):
        br.produce("forecastingData", r)
    for _ in range(2):
        job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert sorted(p["mlpId"] for p in preds) == [1] * 10 + [2] * 10
    # deleting the dense pipeline brings the wave back
    br.produce("requests", json.dumps({"id": 2, "request": "Delete"}))
    job.tick()
    assert job.fserver.serving
    job.fserver.close()
