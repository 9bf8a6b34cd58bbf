#!/usr/bin/env python3
"""End-to-end engine throughput: DataInstance records (JSON, or --format dib: the binary
DIB record, omldm_amd/io/dib.py) in a topic → parse + hash
→ HBM → holdout routing → protocol round → statistics, through the real Job loop
(the path a reference user exercises; the headline bench replays pre-hashed batches).

    python bench/engine_e2e.py [--records 2000000 --batch 65536 --pipelines 1]
Prints one JSON line: records/s of the training stream through the whole engine.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.engine.job import Job  # noqa: E402
from omldm_amd.io.synthetic import synth_json_records  # noqa: E402
from omldm_amd.io.transport import FileBroker  # noqa: E402
from omldm_amd.parallel.comm import init_distributed  # noqa: E402
from omldm_amd.utils import tracing  # noqa: E402
from omldm_amd.utils.config import JobConfig  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--pipelines", type=int, default=1)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--warmup-ticks", type=int, default=4)
    ap.add_argument("--ingest-cus", type=int, default=None,
                    help="engine ingestCUs (XCD-local ingest copies; 0 = plain streams)")
    ap.add_argument("--ingest-copy", default=None, choices=["pull", "sdma"],
                    help="engine ingestCopy (staging copy: pull kernel or SDMA)")
    ap.add_argument("--forecast-frac", type=float, default=0.0,
                    help="share of the records sent to forecastingData (→ predictions)")
    ap.add_argument("--spokes", type=int, default=0,
                    help="spokesPerDevice (0: the job default, parallelism / world = 16)")
    ap.add_argument("--model-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--forecast-server", default="auto", help="engine forecastServer flag")
    ap.add_argument("--unique", type=int, default=100_000,
                    help="distinct JSON records generated; the topic replays them")
    ap.add_argument("--learners", default="",
                    help="comma list of pipelines' learners instead of --pipelines SVMs, "
                         "each NAME or NAME:key=value/key=value (e.g. SVM,K-means:k=16)")
    ap.add_argument("--format", default="json", choices=["json", "dib"],
                    help="topic records: DataInstance JSON (≈ 507 B) or the binary DIB "
                         "record of the same objects (≈ 162 B, omldm_amd/io/dib.py)")
    a = ap.parse_args(argv)
    comm, device = init_distributed()
    sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
    with tempfile.TemporaryDirectory() as root:
        br = FileBroker(root)
        br.create_topic("trainingData", a.partitions)
        t = time.time()
        uniq = synth_json_records(min(a.unique, a.records), sp, start=0, seed=3)
        n_fc = int(a.records * a.forecast_frac)
        fc = synth_json_records(min(a.unique, max(n_fc, 1)), sp, start=10**7, seed=3,
                                operation="forecasting") if n_fc else []
        if a.format == "dib":
            from omldm_amd.io.dib import records_to_dib

            uniq = records_to_dib(uniq, sp.n_numerical, sp.n_discrete, sp.dc)
            fc = records_to_dib(fc, sp.n_numerical, sp.n_discrete, sp.dc) if fc else []
        else:
            uniq = [r.encode() for r in uniq]
            fc = [r.encode() for r in fc]
        rec_bytes = sum(len(r) + 1 for r in uniq) / max(1, len(uniq))
        br.create_topic("forecastingData", min(8, a.partitions))  # a small topic
        for topic, n, src in (("trainingData", a.records - n_fc, uniq),
                              ("forecastingData", n_fc, fc)):
            np_ = a.partitions if topic == "trainingData" else min(8, a.partitions)
            per_part = [[] for _ in range(np_)]
            for i in range(n):
                per_part[i % np_].append(src[i % len(src)])
            for p, recs in enumerate(per_part):
                if recs:
                    br.produce_block(topic, p, b"\n".join(recs) + b"\n")
        del per_part
        gen_s = time.time() - t
        specs = []
        for spec in [t for t in a.learners.split(",") if t]:
            name, _, kv = spec.partition(":")
            hyper = {}
            for item in [t for t in kv.split("/") if t]:
                k, _, v = item.partition("=")
                hyper[k] = json.loads(v) if v[:1] in "-0123456789[{tf" else v
            specs.append((name, hyper))
        if not specs:
            specs = [("SVM", {"modelDtype": a.model_dtype, "tableLog2": 11})] * a.pipelines
        for i, (name, hyper) in enumerate(specs):
            br.produce("requests", json.dumps({
                "id": i + 1, "request": "Create",
                "learner": {"name": name, "hyperParameters": hyper},
                "trainingConfiguration": {"protocol": "Synchronous"}}))
        addr = f"file://{root}"
        args = []
        for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
                  "predictionsAddr", "performanceAddr"):
            args += [f"--{k}", addr]
        cfg = JobConfig.from_args(args + ["--hashDim", str(sp.dim), "--fieldAware", "true",
                                          "--batchSize", str(a.batch), "--timeout", "1000",
                                          "--spokesPerDevice", str(a.spokes),
                                          "--forecastServer", a.forecast_server,
                                          "--parseThreads", str(a.threads), "--jobName", "e2e"]
                                  + (["--ingestCUs", str(a.ingest_cus)]
                                     if a.ingest_cus is not None else [])
                                  + (["--ingestCopy", a.ingest_copy]
                                     if a.ingest_copy is not None else []))
        job = Job(cfg, comm, device)
        while not job.pipes:  # pipeline creation (and first-touch setup) is not timed
            job.tick()
        for _ in range(a.warmup_ticks):  # staging slots grow to the record size
            job.tick()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        r0 = job.counters["records"]
        tracing.reset()
        t0 = time.time()
        # forecasting records on the per-record lane are not counted by the tick
        want = (a.records - (n_fc if job.fserver is not None else 0)) // comm.world
        stall = 0
        while job.counters["records"] + job.counters["invalid"] < want and stall < 200:
            seen = job.counters["records"] + job.counters["invalid"]
            job.tick()
            stall = 0 if job.counters["records"] + job.counters["invalid"] > seen else stall + 1
        job.egress.flush()  # predictions are in their topic
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        wall = time.time() - t0
        stages = tracing.report()
        if job.fserver is not None:  # the forecast lane finishes (not in the training wall)
            job.fserver.catch_up(30.0)
        fs = job.fserver
        lane = {"served": fs.served, **fs.latency_percentiles()} if fs is not None else None
        job.run()  # idle timeout → final statistics
        if comm.rank == 0:
            print(json.dumps({
                "metric": "end-to-end engine records/s (%s topics → training + predictions)"
                          % ("JSON" if a.format == "json" else "DIB binary"),
                "format": a.format, "record_bytes": round(rec_bytes, 1),
                "value": round((job.counters["records"] - r0) * comm.world / max(wall, 1e-9), 1),
                "unit": "records/s", "n_gpus": comm.world, "records": job.counters["records"],
                "pipelines": len(specs), "learners": [n for n, _ in specs], "batch": a.batch, "wall_s": round(wall, 3),
                "spokes": job.spokes, "model_dtype": a.model_dtype,
                "forecast_frac": a.forecast_frac, "predictions": job.counters["predictions"],
                "forecast_lane": lane,
                "generate_s": round(gen_s, 1), "stages_ms": stages,
                "ticks_timed": stages.get("poll", {}).get("calls"),
                "device": str(device)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
