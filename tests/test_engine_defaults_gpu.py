"""Every learner through the engine at the DEFAULT flags on the GPU: the reference's
parallelism (16 spokes), 2^20 hashed features, 13 numerical + 26 categorical features,
the field-aware wire, 65536-record ticks (4096 rows per spoke), GPU parse, read-ahead, the
XCD ingest lane. Only the broker addresses are set. A learner whose round drops updates at
this geometry (a spoke table past LDS, the overflow counter) fails the tick
(utils/health.py); the test also reads each learner's running totals: every training
record fitted, overflow 0, a finite loss (FlinkSpoke.scala:92-107, PipelineMap.scala:68)."""
import json
import math
import uuid

import pytest

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.api.schemas import EXTENSION_LEARNERS, VALID_LEARNERS
from omldm_amd.engine.job import Job
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

HYPER = {"MultiClassPA": {"nClasses": 4}, "HT": {"nClasses": 4}}
TASK = {"RegressorPA": 1, "ORR": 1, "MultiClassPA": 2, "HT": 2}
N_UNIQUE, REPEAT = 20000, 4  # 80000 records: one full 65536-record tick and a partial one


@pytest.fixture(scope="module")
def streams():
    sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
    out = {}
    for task in (0, 1, 2):
        uniq = list(synth_json_records(N_UNIQUE, sp, task=task, seed=11))
        out[task] = (uniq * REPEAT,
                     list(synth_json_records(5, sp, start=10 ** 7, operation="forecasting",
                                             task=task)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("learner", [*VALID_LEARNERS, *EXTENSION_LEARNERS])
def test_default_flags_engine_gpu(cuda, streams, learner):
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    cfg = JobConfig.from_args(args)
    assert (cfg.parallelism, cfg.hashDim, cfg.batchSize, cfg.fieldAware) == (16, 1 << 20,
                                                                            65536, True)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    job = Job(cfg, Comm(), cuda)
    try:
        _drive(job, br, cfg, streams, learner)
    finally:
        job.close()


def _drive(job, br, cfg, streams, learner):
    br.produce("requests", json.dumps({
        "id": 7, "request": "Create",
        "learner": {"name": learner, "hyperParameters": HYPER.get(learner, {})},
        "trainingConfiguration": {"protocol": "Synchronous"}}))
    train, fc = streams[TASK.get(learner, 0)]
    for r in train:
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    pipe = job.pipes[7]
    tot = pipe.learner.running_totals()
    assert tot["overflow"] == 0, tot
    # every record but the holdout's is fitted (the holdout keeps testSetSize per spoke
    # at most)
    assert len(train) - 16 * cfg.testSetSize <= tot["fitted"] <= len(train), tot
    assert math.isfinite(tot["loss_sum"]), tot
    for r in fc:
        br.produce("forecastingData", r)
    br.produce("requests", json.dumps({"id": 7, "request": "Query", "requestId": 3}))
    for _ in range(3):
        job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert len(preds) == 5 and all(p["mlpId"] == 7 for p in preds)
    resp = [json.loads(x) for x in br.records("responses")]
    final = [r for r in resp if r.get("responseId") == 3 and r.get("loss") is not None]
    assert final and final[-1]["dataFitted"] == tot["fitted"], (final[-1:], tot)
    for k in ("loss", "score"):
        v = final[-1].get(k)
        assert v is None or math.isfinite(float(v)), (k, v)
