"""Per-record forecasting on the resident serving wave inside the engine
(engine/forecast_server.py; reference FlinkSpoke.scala:101-105 → FlinkNetwork.scala:243-257).

* every forecasting record gets one Prediction per pipeline, equal to the batched predict
  of the same model;
* pipelines the wave cannot score (preprocessors, dense learners) are answered per record
  by one-row predicts on the lane's stream;
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
    batch, _, _ = parse_records(fc, job.space)
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


def test_every_pipeline_kind_is_answered_per_record():
    """SVM (wave), SVM behind a StandardScaler, NN, ORR, MultiClassPA, K-means and a
    Hoeffding tree in one job: every forecasting record is answered on the lane for all
    seven pipelines (one-row predicts on the lane's stream for the six the wave does not
    score), equal to the batched predict of the same models; latency per family."""
    job, br = _job()
    specs = [(1, "SVM", None, None), (2, "SVM", None, ["StandardScaler"]),
             (3, "NN", {"hiddenLayers": [8]}, None), (4, "ORR", None, ["MinMaxScaler"]),
             (5, "MultiClassPA", {"nClasses": 2}, None), (6, "K-means", {"k": 3}, None),
             (7, "HT", {"nClasses": 2}, ["PolynomialFeatures"])]
    for pid, name, hyper, pre in specs:
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create",
            "learner": {"name": name, "hyperParameters": hyper or {}},
            "preProcessors": [{"name": p} for p in (pre or [])],
            "trainingConfiguration": {"protocol": "Synchronous"}}))
    for r in synth_json_records(6000, SP):
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    fs = job.fserver
    assert fs.serving and [pid for pid, _, _ in fs._served] == [1]
    assert [pid for pid, _ in fs._direct] == [2, 3, 4, 5, 6, 7]
    fc = synth_json_records(12, SP, start=70000, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    job.tick()
    assert not fs.fallback and fs.served == 12
    preds = [json.loads(x) for x in br.records("predictions")]
    assert sorted(p["mlpId"] for p in preds) == sorted(list(range(1, 8)) * 12)
    batch, _, _ = parse_records(fc, job.space)
    batch = batch.without_raw().to("cuda")
    for pid, name, _, _ in specs:
        want = job.pipes[pid].predict(batch).float().cpu()
        got = torch.tensor([p["prediction"] for p in preds if p["mlpId"] == pid])
        assert torch.allclose(got, want, rtol=1e-4, atol=1e-4), (name, got, want)
    fam = fs.family_percentiles()
    assert set(fam) >= {"linear-store", "SVM", "NN", "ORR", "MultiClassPA", "K-means", "HT"}, fam
    assert all(v["n"] >= 12 and v["p50"] < 20000 for v in fam.values()), fam
    # deleting pipelines reconfigures the lane; the rest keep being answered
    br.produce("requests", json.dumps({"id": 3, "request": "Delete"}))
    job.tick()
    assert [pid for pid, _ in fs._direct] == [2, 4, 5, 6, 7]
    job.fserver.close()


def test_default_flag_svm_trains_through_the_v3_scan():
    """A job started with default flags (field-aware compact slots) and a default SVM
    Create trains through the exact v3 table scan (csrc/kernels/linear_scan3.hip), fed the
    compact int16 slots as they are; its weights match the CPU engine's exact spokes."""
    from omldm_amd.ops import linear as L

    job, br = _job()
    assert job.space.field_aware and job.space.cat_span > 0
    _create(br, 1, "SVM")
    for r in synth_json_records(8000, SP):
        br.produce("trainingData", r)
    n0 = L.SCAN3_ROUNDS
    for _ in range(4):
        job.tick()
    assert L.SCAN3_ROUNDS > n0
    assert job.pipes[1].learner.running_totals()["fitted"] > 0
    job.fserver.close()


def test_wave_reads_the_requested_bank():
    """The resident wave scores against the weight bank each request names (the request
    line's last dword, checksummed): bank 0 / bank 1 answers are those of w0 / w1."""
    from omldm_amd.io.synthetic import synth_batch
    from omldm_amd.ops import linear as L
    from omldm_amd.ops.serving import PredictServer

    b = synth_batch(SP, 8, seed=3)
    w0 = torch.randn(2, SP.dim) * 0.1
    w1 = torch.randn(2, SP.dim) * 0.1
    srv = PredictServer(w0.cuda(), SP.dn, SP.dc, True, cat_span=0, w1=w1.cuda())
    srv.start(lifetime_us=5_000_000)
    try:
        for i in range(8):
            pt = b.slice(i, i + 1)
            for bank, w in ((0, w0), (1, w1), (0, w0)):
                got = torch.tensor(srv.request(pt, bank=bank))
                want = L.linear_predict(w, pt)[0]
                assert torch.allclose(got, want, rtol=1e-5, atol=1e-5), (i, bank, got, want)
    finally:
        srv.close()


def test_forecasts_read_a_published_model_version():
    """Between ticks the lane's answers equal the batched predict of the model after the
    last round (the publish copy adopted once complete); the banks alternate per round, and
    the live store rows are never what the wave reads."""
    job, br = _job()
    _create(br, 1, "SVM")
    fs = job.fserver
    banks_seen = set()
    for t in range(5):
        for r in synth_json_records(2000, SP, start=t * 2000):
            br.produce("trainingData", r)
        job.tick()
        torch.cuda.synchronize()
        assert fs._banks is not None and fs._banks[0].data_ptr() != job.store.W.data_ptr()
        fc = synth_json_records(3, SP, start=90000 + 10 * t, operation="forecasting")
        n0 = len(br.records("predictions"))
        for r in fc:
            br.produce("forecastingData", r)
        assert fs.catch_up(10.0)
        banks_seen.add(fs._bank)
        preds = [json.loads(x) for x in br.records("predictions")[n0:]]
        batch, _, _ = parse_records(fc, job.space)
        want = job.pipes[1].predict(batch.without_raw().to("cuda")).float().cpu()
        got = torch.tensor([p["prediction"] for p in preds])
        assert torch.equal(got, want), (t, got, want)
    assert banks_seen == {0, 1}
    fs.close()
