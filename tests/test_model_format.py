"""Model export / import in the reference's only portable model format: the QueryResponse
``learner`` JSON (parameters / hyperParameters / dataStructure), bucketed by 10,000
parameters as ``name[start-end]`` (omldm/network/FlinkNetwork.scala:48-240), fed back as
a Create request's ``learner.parameters`` (FlinkSpoke.scala:198-219 passes the request's
learner POJO to node creation). For every learner: train → Query → merge the bucketed
responses → Create a second pipeline with those parameters → identical predictions.
"""
import json
import uuid

import pytest

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.api.schemas import VALID_LEARNERS
from omldm_amd.engine.job import Job
from omldm_amd.engine.statistics import merge_bucketed
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

HYPER = {"MultiClassPA": {"nClasses": 3}, "K-means": {"k": 3}, "HT": {"nClasses": 3},
         "NN": {"hiddenLayers": [16]}}
TASK = {"RegressorPA": 1, "ORR": 1, "MultiClassPA": 2, "HT": 2}
PRE = {"ORR": "PolynomialFeatures", "NN": "StandardScaler", "K-means": "MinMaxScaler"}


def _job(device, dim_log2=16):
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(1 << dim_log2), "--batchSize", "400", "--timeout", "500",
             "--parallelism", "4", "--numFeatures", "5", "--catFeatures", "6"]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    return Job(cfg, Comm(), device), br, FeatureSpace(5, 0, 6, 1 << dim_log2)


def _round_trip(learner, device):
    job, br, sp = _job(device)
    task = TASK.get(learner, 0)
    pre = [{"name": PRE[learner]}] if learner in PRE else []
    hyper = HYPER.get(learner, {})
    br.produce("requests", json.dumps({"id": 7, "request": "Create",
                                       "learner": {"name": learner, "hyperParameters": hyper},
                                       "preProcessors": pre,
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))
    for r in synth_json_records(1600, sp, task=task):
        br.produce("trainingData", r)
    for _ in range(5):
        job.tick()
    br.produce("requests", json.dumps({"id": 7, "request": "Query", "requestId": 31}))
    job.tick()
    resp = [json.loads(x) for x in br.records("responses")]
    mine = sorted((r for r in resp if r.get("responseId") == 31), key=lambda r: r["id"])
    assert mine and mine[-1]["dataFitted"] > 0
    # the user's side: merge the buckets of the response back into one learner map
    params, pres = {}, None
    for r in mine:
        params.update((r.get("learner") or {}).get("parameters") or {})
        pres = r.get("preprocessors") or pres
    params = merge_bucketed(params)
    assert params, learner
    create = {"id": 8, "request": "Create",
              "learner": {"name": learner, "hyperParameters": hyper, "parameters": params},
              "preProcessors": pres or [],
              "trainingConfiguration": {"protocol": "Synchronous"}}
    br.produce("requests", json.dumps(create))
    job.tick()
    assert 8 in job.pipes, job.counters
    for r in synth_json_records(64, sp, start=7000, operation="forecasting", task=task):
        br.produce("forecastingData", r)
    for _ in range(2):
        job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    p7 = [p["prediction"] for p in preds if p["mlpId"] == 7]
    p8 = [p["prediction"] for p in preds if p["mlpId"] == 8]
    assert len(p7) == len(p8) == 64
    for a, b in zip(p7, p8):
        assert abs(float(a) - float(b)) <= 1e-4 * max(1.0, abs(float(a))), (learner, a, b)
    return len(mine)


@pytest.mark.parametrize("learner", VALID_LEARNERS)
def test_query_create_round_trip(learner):
    n = _round_trip(learner, "cpu")
    if learner in ("PA", "SVM", "RegressorPA", "MultiClassPA"):
        assert n > 2  # 2^16 hashed weights travel in several 10,000-parameter buckets


@pytest.mark.gpu
@pytest.mark.parametrize("learner", VALID_LEARNERS)
def test_query_create_round_trip_gpu(cuda, learner):
    _round_trip(learner, cuda)
