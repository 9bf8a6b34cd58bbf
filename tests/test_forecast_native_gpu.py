"""The native forecast lane (csrc/host/fcst_lane.cpp): with file topics and every pipeline
on the serving wave, the engine answers forecasting records from a C++ thread — poll,
parse, mailbox, Prediction formatting and append without the Python interpreter
(reference: FlinkSpoke.scala:101-105 → FlinkNetwork.scala:243-257, one Prediction per
pipeline per record as it arrives).

* the answers equal the batched predict of the same model, one per pipeline, the
  DataInstance echoed;
* across ticks the lane reads a published model version (the GPU flips the pinned bank
  word after each publish copy);
* the lane's offsets are the checkpoint view; stopping it hands them back to the Python
  consumer.
"""
import json
import os

import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.io.parse import parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import FileBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

pytestmark = pytest.mark.gpu

SP = FeatureSpace(13, 0, 26, 1 << 18)


def _job(root):
    addr = f"file://{root}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--batchSize", "2000", "--timeout", "300",
             "--parallelism", "8"]
    cfg = JobConfig.from_args(args)
    br = FileBroker(root)
    for t in ("trainingData", "forecastingData", "requests", "predictions", "responses",
              "performance"):
        br.create_topic(t, 2 if t in ("trainingData", "forecastingData") else 1)
    return Job(cfg, Comm(), "cuda"), br


def _create(br, pid, learner):
    br.produce("requests", json.dumps({"id": pid, "request": "Create",
                                       "learner": {"name": learner},
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))


def _preds(br):
    out = []
    d = os.path.join(br.root, "predictions")
    for f in sorted(os.listdir(d)):
        with open(os.path.join(d, f), "rb") as fh:
            out += [json.loads(x) for x in fh.read().splitlines() if x.strip()]
    return out


def test_native_lane_answers_like_the_batched_predict(tmp_path):
    job, br = _job(str(tmp_path))
    _create(br, 1, "SVM")
    _create(br, 2, "PA")
    for r in synth_json_records(6000, SP):
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    fs = job.fserver
    assert fs.serving and fs.native, "file topics + wave pipelines: the native lane"
    fc = synth_json_records(40, SP, start=70000, operation="forecasting")
    for r in fc:
        br.produce("forecastingData", r)
    assert fs.catch_up(10.0)
    preds = _preds(br)
    assert len(preds) == 80
    batch, _, _ = parse_records(fc, job.space)
    batch = batch.without_raw().to("cuda")
    for pid in (1, 2):
        want = job.pipes[pid].predict(batch).float().cpu()
        mine = [p for p in preds if p["mlpId"] == pid]
        got = sorted((json.dumps(p["dataPoint"], sort_keys=True), p["prediction"]) for p in mine)
        ref = sorted((json.dumps(json.loads(r), sort_keys=True), float(w))
                     for r, w in zip(fc, want.tolist()))
        assert got == ref, pid
    st = fs.native_stats()
    assert st["served"] == 40 and st["write_errors"] == 0
    assert set(st["stage_us"]) == {"poll", "parse", "wave", "format", "produce", "record"}
    lat = fs.latency_percentiles()
    assert lat["n"] == 40 and lat["p50"] is not None
    done, waiting = fs.snapshot()
    assert not waiting and all(done[p] == os.path.getsize(
        os.path.join(br.root, "forecastingData", f"{p}.jsonl")) for p in done)
    job.close()


def test_native_lane_reads_a_published_model_version(tmp_path):
    job, br = _job(str(tmp_path))
    _create(br, 1, "SVM")
    fs = job.fserver
    n_seen = 0
    for t in range(5):
        for r in synth_json_records(2000, SP, start=t * 2000):
            br.produce("trainingData", r)
        job.tick()
        torch.cuda.current_stream().synchronize()  # (not the device: the resident wave)
        assert fs.native
        fc = synth_json_records(3, SP, start=90000 + 10 * t, operation="forecasting")
        for r in fc:
            br.produce("forecastingData", r)
        assert fs.catch_up(10.0)
        preds = _preds(br)[n_seen:]
        n_seen += len(preds)
        batch, _, _ = parse_records(fc, job.space)
        want = job.pipes[1].predict(batch.without_raw().to("cuda")).float().cpu()
        got = {json.dumps(p["dataPoint"], sort_keys=True): p["prediction"] for p in preds}
        ref = {json.dumps(json.loads(r), sort_keys=True): float(w)
               for r, w in zip(fc, want.tolist())}
        assert got == ref, t
    job.close()
