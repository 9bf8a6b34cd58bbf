#!/usr/bin/env python3
"""Quickstart: the reference's user flow in one process, no Kafka needed.

OMLDM users drive a running job through topics: JSON *requests* create / update / query /
delete ML pipelines, *trainingData* and *forecastingData* carry DataInstance records, and
*predictions*, *responses* and *performance* come back. This script does the same against
the in-process broker (``memory://``), on the GPU when one is visible:

    python examples/quickstart.py            # GPU if available, else CPU
    python examples/quickstart.py --cpu

The same Job runs under ``torchrun`` with ``--trainingDataAddr host:9092`` (Kafka) or
``file:///dir`` topics — see examples/single_node.sh.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.engine.job import Job  # noqa: E402
from omldm_amd.io.synthetic import synth_json_records  # noqa: E402
from omldm_amd.io.transport import MemoryBroker  # noqa: E402
from omldm_amd.parallel.comm import Comm  # noqa: E402
from omldm_amd.utils.config import JobConfig  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--records", type=int, default=20000)
    a = ap.parse_args(argv)
    device = "cuda" if torch.cuda.is_available() and not a.cpu else "cpu"

    # 1. a job whose topics all live on the in-process broker "quickstart"
    addr = "memory://quickstart"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    cfg = JobConfig.from_args(args + ["--hashDim", str(1 << 18), "--batchSize", "4096",
                                      "--timeout", "500"])
    br = MemoryBroker.named("quickstart")
    br.create_topic(cfg.trainingDataTopic, 4)
    job = Job(cfg, Comm(), device)
    space = FeatureSpace(13, 0, 26, 1 << 18)

    # 2. pipelines are created by requests (learner, preprocessors, protocol)
    def request(body: dict) -> None:
        br.produce(cfg.requestsTopic, json.dumps(body))

    request({"id": 1, "request": "Create",
             "learner": {"name": "SVM", "hyperParameters": {"C": 1.0}},
             "preProcessors": [{"name": "StandardScaler"}],
             "trainingConfiguration": {"protocol": "Synchronous"}})
    request({"id": 2, "request": "Create",
             "learner": {"name": "PA", "hyperParameters": {"variant": "PA-II", "C": 0.5}},
             "trainingConfiguration": {"protocol": "Asynchronous"}})

    # 3. a labelled stream, then a few points to forecast
    for r in synth_json_records(a.records, space, seed=7):
        br.produce(cfg.trainingDataTopic, r)
    for _ in range(8):
        job.tick()
    for r in synth_json_records(5, space, start=10**6, seed=7, operation="forecasting"):
        br.produce(cfg.forecastingDataTopic, r)
    request({"id": 1, "request": "Query", "requestId": 100})
    request({"id": 2, "request": "Query", "requestId": 200})
    for _ in range(3):
        job.tick()

    # 4. read what came back
    for p in [json.loads(x) for x in br.records(cfg.predictionsTopic)][:4]:
        print("prediction:", {k: p[k] for k in ("mlpId", "prediction")})
    # a query answer is a series of QueryResponse messages: the learner's parameters in
    # buckets (name[start-end]), the last one carrying the statistics
    resp = [json.loads(x) for x in br.records(cfg.responsesTopic)]
    for rid in sorted({r["responseId"] for r in resp}):
        parts = [r for r in resp if r["responseId"] == rid]
        last = parts[-1]
        print(f"response {rid}: {len(parts)} message(s);",
              {k: last.get(k) for k in ("mlpId", "dataFitted", "score", "loss")})

    # 5. an idle stream ends the run; the job statistics go to the performance topic
    job.run()
    perf = json.loads(br.records(cfg.performanceTopic)[-1])
    print("performance:", {k: perf[k] for k in ("jobName", "parallelism")},
          [(s["pipeline"], s["protocol"], s["fitted"]) for s in perf["statistics"]])
    return 0


if __name__ == "__main__":
    sys.exit(main())
