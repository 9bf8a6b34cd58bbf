#!/usr/bin/env python3
"""BASELINE config 5 through the engine: 16 HETEROGENEOUS pipelines created through the
requests topic, trained on one DataInstance stream by the Job's tick loop, each model
compared with the same pipeline trained alone on the same stream.

The pipelines (reference: every record is fed to every pipeline of a spoke,
FlinkSpoke.scala:97,101,105): PA-I with six C values, PA-II with two, PA, logistic
regression with three learning rates, RegressorPA with two ε, MultiClassPA with 2 and 4
classes. The engine fuses the pipelines that share a v3 prep (same rule family and row
scaling) into one launch (engine/job.py `_fused_groups`) and runs the other groups on
`--streams` pipeline streams (the process has 4 hardware queues on this pool; copy, prep,
aux and serving streams take some of them).

    python bench/config5_engine.py [--records 1048576 --batch 131072 --streams 2]
Prints one JSON line: ms per tick (all 16 pipelines), pipeline-examples/s, per pipeline
the max |Δw| against its one-pipeline run.
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
from omldm_amd.utils.config import JobConfig  # noqa: E402

PIPES = ([("SVM", {"variant": "PA-I", "C": c}) for c in (0.25, 0.5, 1.0, 2.0, 4.0, 8.0)]
         + [("SVM", {"variant": "PA-II", "C": c}) for c in (0.5, 1.0)]
         + [("PA", {})]
         + [("LogisticRegression", {"learningRate": lr}) for lr in (0.05, 0.1, 0.2)]
         + [("RegressorPA", {"epsilon": e}) for e in (0.1, 0.5)]
         + [("MultiClassPA", {"nClasses": k}) for k in (2, 4)])


def _job(root, args_extra, device, comm):
    addr = f"file://{root}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    cfg = JobConfig.from_args(args + args_extra)
    return Job(cfg, comm, device)


def run(pipes, recs_block, n_blocks, a, device, comm, trace=False):
    """One engine run over the same stream with ``pipes``: (job, ms per tick, models)."""
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as root:
        br = FileBroker(root)
        for t, n_p in (("trainingData", 16), ("forecastingData", 1), ("requests", 1),
                       ("predictions", 1), ("responses", 1), ("performance", 1)):
            br.create_topic(t, n_p)
        for i in range(n_blocks):
            br.produce_block("trainingData", i % 16, recs_block)
        for pid, (name, hyper) in pipes:
            br.produce("requests", json.dumps({
                "id": pid, "request": "Create", "learner": {"name": name, "hyperParameters": hyper},
                "trainingConfiguration": {"protocol": "Synchronous"}}))
        job = _job(root, ["--batchSize", str(a.batch), "--parallelism", "16", "--test", "false",
                          "--pipelineStreams", str(a.streams), "--timeout", "1000",
                          "--forecastServer", "false"], device, comm)
        while len(job.pipes) < len(pipes):
            job.tick()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        prof = None
        if trace and device.type == "cuda":  # in-process kernel trace (torch.profiler)
            prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA,
                                                      torch.profiler.ProfilerActivity.CPU])
            prof.__enter__()
        t0 = time.perf_counter()
        ticks = 0
        want = n_blocks * a.block
        while job.counters["records"] < want:
            job.tick()
            ticks += 1
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        wall = time.perf_counter() - t0
        if prof is not None:
            prof.__exit__(None, None, None)
            table = prof.key_averages().table(sort_by="self_device_time_total", row_limit=40)
            with open(trace, "w") as f:
                f.write(f"# {len(pipes)} pipelines, {ticks} ticks, {wall * 1e3 / max(1, ticks):.3f} ms "
                        f"per tick (profiled run)\n" + table + "\n")
        models = {pid: p.learner.state_vector().detach().float().cpu().clone()
                  for pid, p in job.pipes.items()}
        recs = job.counters["records"]
        job.close()
    return job, wall * 1e3 / max(1, ticks), ticks, recs, models


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--block", type=int, default=16384, help="distinct records replayed")
    ap.add_argument("--batch", type=int, default=131072, help="records per tick")
    ap.add_argument("--streams", type=int, default=2, help="engine pipelineStreams")
    ap.add_argument("--solo", type=int, default=1, help="one-pipeline reference runs")
    ap.add_argument("--trace", default="", help="write a kernel summary of the 16-pipeline run")
    a = ap.parse_args(argv)
    comm, device = init_distributed()
    sp = FeatureSpace(13, 0, 26, 1 << 20)
    block = ("\n".join(synth_json_records(a.block, sp, seed=5)) + "\n").encode()
    n_blocks = max(1, a.records // a.block)
    pipes = [(i + 1, p) for i, p in enumerate(PIPES)]
    job, ms_tick, ticks, recs, models = run(pipes, block, n_blocks, a, device, comm)
    if a.trace:
        run(pipes, block, n_blocks, a, device, comm, trace=a.trace)
    out = {"metric": "BASELINE config 5 through the engine: 16 heterogeneous pipelines "
                     "(requests topic → Job ticks), ms per tick and pipeline-examples/s",
           "ms_per_tick": round(ms_tick, 3), "ticks": ticks, "records": recs,
           "pipelines": len(pipes),
           "pipeline_examples_per_s": round(recs * len(pipes) / (ms_tick * ticks / 1e3), 1),
           "streams": a.streams, "batch": a.batch, "per_pipeline": {}}
    if a.solo:
        for pid, spec in pipes:
            _, ms1, _, _, m1 = run([(pid, spec)], block, n_blocks, a, device, comm)
            d = float((models[pid] - m1[pid]).abs().max())
            scale = float(m1[pid].abs().max()) or 1.0
            out["per_pipeline"][pid] = {"learner": spec[0], "hyper": spec[1],
                                        "max_abs_dw_vs_alone": float(f"{d:.3e}"),
                                        "rel_dw_vs_alone": float(f"{d / scale:.3e}"),
                                        "alone_ms_per_tick": round(ms1, 3)}
        out["alone_ms_per_tick_sum"] = round(sum(v["alone_ms_per_tick"]
                                                 for v in out["per_pipeline"].values()), 3)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
