#!/usr/bin/env python3
"""Headline benchmark: online linear SVM (PA-I) training throughput (examples/s, whole
node) + p50 single-point predict latency, 1/2/4/8 MI355X GPUs (BASELINE.json), at the
reference's semantics and precision.

Workload (what the reference computes, FlinkSpoke.scala:92-107 + the Synchronous PS):
P = 16 spokes per GPU (the reference's default parallelism, DefaultJobParameters.scala:5),
each an EXACT sequential PA-I learner over its shard of the stream on its own fp32 model
replica; every round the parameter server averages the replicas of all spokes of all
GPUs. 2^20 hashed features: 13 numerical + 26 categorical fields + intercept.

One step == one Synchronous round on every GPU, all inside the timed region:
  pinned host micro-batch on the raw binary wire (fp32 numerical features, 32-bit
  category TOKENS, int8 labels) ──pull-copy kernel on a CU-masked ingest lane (copy of
  batch k+1 overlaps the round on batch k)──► HBM
  → passes 1-3 of the v3 round (csrc/kernels/linear_scan3.hip) on their own CU-masked
    stream as soon as the batch lands: murmur3 hashing of the tokens, the per-field
    occurrence sort (LDS slot-table flags), then every 64-row chunk's Gram G and cross
    Gram X1 over the whole GPU — overlapping the previous round's scan (--prep-ahead)
  → the scan: per spoke, a w0-margin workgroup sums the round-start model over every
    occurrence ahead of the scan; the scan workgroup's scanner wave runs the exact PA-I
    recurrence on the Grams, its helper waves keep the spoke's updates in an LDS slot
    table (no dense replicas)
  → in-launch combiners sum the spokes' updates into the round accumulator → RCCL
    all-reduce over xGMI (N > 1) → apply: w += average update.
Also reported (rank 0): the engine's per-record forecast latency (a JSON record produced
into the forecasting topic → its Prediction, `engine_forecast_*`) and the engine's
end-to-end JSON training rate (`engine_e2e_*`).
Quality is reported next to the speed: holdout accuracy of the trained model and of the
CPU reference-semantics learner (csrc/host/rawwire.cpp, P = 16·N sequential spokes) on
exactly the same stream and example count.

Launch: python bench.py [--gpus 1 --steps 20 --warmup 5]; for N > 1 the driver uses
python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from omldm_amd.api.batch import FeatureSpace, RawBatch  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.models.linear import SVM, LogisticRegression  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402
from omldm_amd.ops import native  # noqa: E402
from omldm_amd.parallel.comm import init_distributed  # noqa: E402
from omldm_amd.parallel.protocols import Synchronous  # noqa: E402

METRIC = "training examples/sec (whole node) + p50 predict latency, linear SVM 1/2/4/8 GPU"
TEST_START = 10**12  # holdout examples: a stream segment no rank trains on


class PackedRaw:
    """num | tok | y of one micro-batch in ONE contiguous (pinned) buffer: one copy."""

    def __init__(self, space: FeatureSpace, B: int, device, pin: bool, y_dtype=torch.int8):
        ysz = torch.tensor([], dtype=y_dtype).element_size()
        self.sizes = [B * space.dn * 4, B * space.dc * 4, B * ysz]
        offs = [0]
        for s in self.sizes:
            offs.append(offs[-1] + ((s + 255) // 256) * 256)
        self.flat = torch.empty(offs[-1], dtype=torch.uint8, device=device,
                                pin_memory=pin and str(device) == "cpu")
        f = self.flat
        self.batch = RawBatch(
            f[offs[0]:offs[0] + self.sizes[0]].view(torch.float32).view(B, space.dn),
            f[offs[1]:offs[1] + self.sizes[1]].view(torch.int32).view(B, space.dc),
            f[offs[2]:offs[2] + self.sizes[2]].view(y_dtype).view(B))

    @property
    def wire_bytes(self) -> int:
        return sum(self.sizes)


def shard_start(k: int, rank: int, world: int, B: int) -> int:
    """Stream position of pool batch k of rank r: the global stream round-robins ranks."""
    return (k * world + rank) * B


def engine_forecast_latency(n: int, train_records: int = 4_000_000) -> dict:
    """Record produced into the forecasting topic → its Prediction in the predictions
    topic, through the engine with a trained linear SVM pipeline: file topics, so the
    forecast lane is the native thread (csrc/host/fcst_lane.cpp: pread → native parse →
    resident serving wave → native Prediction formatting → append; no Python on the
    record's path). t_in is taken before the record's append, t_out by the lane right after
    its Prediction's append (both CLOCK_MONOTONIC); the bench thread waits in a native call
    (GIL released), not in a Python spin. Measured twice: with the engine idle between
    ticks, and while its tick thread trains on a pre-filled training topic (JSON records
    through the engine's e2e path) — only records answered while training ran count there.
    Per-stage µs (the lane's own clock) are reported with each."""
    import tempfile
    import threading

    from omldm_amd.engine.job import Job
    from omldm_amd.io.synthetic import synth_json_records
    from omldm_amd.io.transport import FileBroker
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.utils.config import JobConfig

    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    with tempfile.TemporaryDirectory(dir=shm) as root:
        br = FileBroker(root)
        for t, n_p in (("trainingData", 16), ("forecastingData", 1), ("requests", 1),
                       ("predictions", 1), ("responses", 1), ("performance", 1)):
            br.create_topic(t, n_p)
        args = []
        for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
                  "predictionsAddr", "performanceAddr"):
            args += [f"--{k}", f"file://{root}"]
        args += ["--batchSize", "524288", "--parallelism", "16", "--test", "false"]
        cfg = JobConfig.from_args(args)
        sp = FeatureSpace(cfg.numFeatures, 0, cfg.catFeatures, cfg.hashDim)
        job = Job(cfg, Comm.local(), torch.device("cuda", torch.cuda.current_device()))
        br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                           "learner": {"name": "SVM"},
                                           "trainingConfiguration": {"protocol": "Synchronous"}}))
        block = ("\n".join(r if isinstance(r, str) else r.decode()
                            for r in synth_json_records(20000, sp)) + "\n").encode()
        tfds = [os.open(os.path.join(root, "trainingData", f"{p}.jsonl"), os.O_WRONLY | os.O_APPEND)
                for p in range(16)]
        os.write(tfds[0], block)
        for _ in range(3):
            job.tick()
        fs = job.fserver
        lane = "native" if fs.native else "python"
        recs = [r if isinstance(r, bytes) else r.encode()
                for r in synth_json_records(2 * n + 40, sp, start=10**9, operation="forecasting")]
        ffd = os.open(os.path.join(root, "forecastingData", "0.jsonl"), os.O_WRONLY | os.O_APPEND)

        def send(batch, gap_s, while_=None):
            lat = []
            for i, r in enumerate(batch):
                if while_ is not None and not while_():
                    break
                k = fs.native_stats()["served"] if fs.native else None
                t_in = time.perf_counter()
                os.write(ffd, r.replace(b"\n", b" ") + b"\n")
                if fs.native:
                    if not fs.native_wait(k + 1, 2.0):
                        raise RuntimeError("native forecast lane: no answer within 2 s")
                    t_out = fs.native_tout(k)
                else:
                    assert fs.catch_up(2.0)
                    t_out = time.perf_counter()
                lat.append((t_out - t_in) * 1e6)
                t = time.perf_counter()
                while time.perf_counter() - t < gap_s:  # records arrive one at a time
                    time.sleep(0)
            return lat

        def pct(lat):
            lat = sorted(lat)
            if not lat:
                return None, None
            return (round(lat[len(lat) // 2], 2),
                    round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 2))

        send(recs[:20], 100e-6)                      # wave start, warm caches
        s0 = fs.native_stats() if fs.native else None
        idle = send(recs[20:20 + n], 100e-6)
        s1 = fs.native_stats() if fs.native else None

        def stage_delta(a, b):
            if a is None or b is None:
                return None
            d = max(1, b["served"] - a["served"])
            return {k: round((b["stage_us"][k] * b["served"] - a["stage_us"][k] * a["served"])
                             / d, 3) for k in b["stage_us"]}

        # under training: the tick thread trains on a pre-filled JSON training topic
        reps = max(1, train_records // 20000)
        for i in range(reps):
            os.write(tfds[i % 16], block)
        end = {p: os.path.getsize(os.path.join(root, "trainingData", f"{p}.jsonl"))
               for p in range(16)}
        busy = threading.Event()
        busy.set()
        trained = {"records": 0, "s": 0.0}

        def trainer():
            t0 = time.perf_counter()
            f0 = job.pipes[1].learner.running_totals()["fitted"]
            while any(job.train_in.offsets.get(p, 0) < o for p, o in end.items()
                      if p in job.train_in.offsets):
                job.tick()
            torch.cuda.current_stream().synchronize()  # (a device sync waits for the wave)
            trained["s"] = time.perf_counter() - t0
            trained["records"] = job.pipes[1].learner.running_totals()["fitted"] - f0
            busy.clear()

        th = threading.Thread(target=trainer)
        th.start()
        s2 = fs.native_stats() if fs.native else None
        under = send(recs[20 + n:], 100e-6, while_=busy.is_set)
        s3 = fs.native_stats() if fs.native else None
        th.join()
        job.close()
        for fd in tfds + [ffd]:
            os.close(fd)
    p50, p99 = pct(idle)
    u50, u99 = pct(under)
    return {"p50": p50, "p99": p99, "lane": lane, "stage_us": stage_delta(s0, s1),
            "train_p50": u50, "train_p99": u99, "train_n": len(under),
            "train_stage_us": stage_delta(s2, s3),
            "train_records_per_s": round(trained["records"] / trained["s"], 1)
            if trained["s"] > 0 else None,
            "what": f"{len(idle)} JSON forecasting records, each appended to the forecasting "
                    f"file topic → its Prediction appended to the predictions topic ({lane} "
                    "forecast lane: pread + native parse + resident serving wave + native "
                    "Prediction formatting + append), trained SVM, engine idle between ticks; "
                    f"train_*: {len(under)} records answered while the engine's tick thread "
                    "trained on a pre-filled JSON training topic"}


def cpu_baseline() -> dict | None:
    """The reference-class CPU baseline measured on the MI355X host (same stream shape,
    P = 16): bench/baselines/cpu_reference_mi355x_host_p16.json (a copy of
    profiles/round4/'s; profiles/ does not travel to the GPU box)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench", "baselines",
                        "cpu_reference_mi355x_host_p16.json")
    try:
        with open(path) as f:
            d = json.loads(f.read().strip().splitlines()[-1])
        return {"value": float(d["value"]), "source": os.path.relpath(path, os.path.dirname(
            os.path.abspath(__file__)))}
    except (OSError, ValueError, KeyError):
        return None


def engine_e2e_rate(records: int, batch: int = 131072, fmt: str = "json") -> dict:
    """Records/s of the training stream through the whole engine (rank 0, one GPU): JSON
    DataInstance records in a file topic → pinned staging → GPU parse + feature hashing →
    holdout routing → Synchronous round of a linear SVM (fp32, the job's default spokes)
    → statistics. Record generation is not timed; the topic replays 20,000 distinct
    records (bench/engine_e2e.py is the standalone, multi-GPU form)."""
    import tempfile

    from omldm_amd.engine.job import Job
    from omldm_amd.io.synthetic import synth_json_records
    from omldm_amd.io.transport import FileBroker
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.utils.config import JobConfig

    sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
    # partitions are read concurrently (one GIL-free pread each; 8 MB regions): one per
    # spoke of the reference's parallelism (16: JSON 93.7 / DIB 250 M records/s vs 91.6 /
    # 241 M with 8, profiles/round5/e2e/parts_*.json)
    parts = int(os.environ.get("OMLDM_E2E_PARTS", "16"))
    with tempfile.TemporaryDirectory() as root:
        br = FileBroker(root)
        br.create_topic("trainingData", parts)
        br.create_topic("forecastingData", 8)
        uniq = synth_json_records(20000, sp, start=0, seed=3)
        if fmt == "dib":  # the same records as binary DIB records (omldm_amd/io/dib.py)
            from omldm_amd.io.dib import records_to_dib

            uniq = records_to_dib(uniq, sp.n_numerical, sp.n_discrete, sp.dc)
        else:
            uniq = [r.encode() for r in uniq]
        total = records + 4 * batch  # the untimed Create / warmup ticks read some first
        import math

        period = len(uniq) // math.gcd(parts, len(uniq))  # partition p replays uniq[p::parts]
        for p in range(parts):
            n_p = len(range(p, total, parts))
            cyc = b"".join(uniq[(p + parts * j) % len(uniq)] + b"\n" for j in range(period))
            tail = b"".join(uniq[(p + parts * j) % len(uniq)] + b"\n"
                            for j in range(n_p - n_p % period, n_p))
            br.produce_block("trainingData", p, cyc * (n_p // period) + tail)
        br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                           "learner": {"name": "SVM"},
                                           "trainingConfiguration": {"protocol": "Synchronous"}}))
        args = []
        for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
                  "predictionsAddr", "performanceAddr"):
            args += [f"--{k}", f"file://{root}"]
        cfg = JobConfig.from_args(args + ["--hashDim", str(sp.dim), "--fieldAware", "true",
                                          "--batchSize", str(batch), "--timeout", "1000",
                                          "--test", "false", "--jobName", "bench-e2e"]
                              + os.environ.get("OMLDM_E2E_ARGS", "").split())
        dev = torch.device("cuda", torch.cuda.current_device())
        job = Job(cfg, Comm.local(), dev)
        while not job.pipes:
            job.tick()
        for _ in range(2):  # staging slots grow to the record size
            job.tick()
        torch.cuda.synchronize(dev)
        from omldm_amd.utils import tracing

        tracing.reset()
        r0, k0 = job.counters["records"], job.ticks
        t0 = time.perf_counter()
        while job.counters["records"] + job.counters["invalid"] < r0 + records:
            job.tick()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        n = job.counters["records"] - r0
        ticks = job.ticks - k0
        # host time per tick of every stage (tick thread; ingest_* on the reader / staging
        # threads, which run beside it)
        stages = {k: round(v["host_ms"] / max(1, ticks), 4) for k, v in tracing.report().items()}
        job.close()
    return {"records_per_s": round(n / max(wall, 1e-9), 1), "records": n,
            "spokes": job.spokes, "batch": batch, "ticks": ticks,
            "ms_per_tick": round(wall * 1e3 / max(1, ticks), 4), "stage_ms_per_tick": stages,
            "record_bytes": round(sum(len(r) + 1 for r in uniq) / len(uniq), 1)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--spokes", type=int, default=16,
                    help="sequential spokes per GPU (the reference's default parallelism)")
    ap.add_argument("--rows", type=int, default=8192, help="examples per spoke per round")
    ap.add_argument("--dim-log2", type=int, default=20)
    ap.add_argument("--learner", default="SVM", choices=["SVM", "LogisticRegression"])
    ap.add_argument("--model-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: the learner's modelDtype (margins on bf16 weights, fp32 "
                         "master and arithmetic; BASELINE config 2 names a bf16 model)")
    ap.add_argument("--pool", type=int, default=8, help="pinned host batches per rank")
    ap.add_argument("--ingest", default="pinned", choices=["pinned", "device"],
                    help="pinned: H2D copy of every batch inside the timed loop")
    ap.add_argument("--h2d", default="pull", choices=["pull", "sdma"])
    ap.add_argument("--slots", type=int, default=3, help="HBM staging buffers")
    ap.add_argument("--ingest-cus", type=int, default=16)
    ap.add_argument("--cu-layout", type=int, default=1)
    ap.add_argument("--pull-blocks", type=int, default=16)
    ap.add_argument("--settle-ms", type=float, default=500.0,
                    help="GPU clock settle before the warmup: dense matmuls for this long on "
                         "a scratch tensor (no model state; a fresh box's first process ran "
                         "~15%% slower without it)")
    ap.add_argument("--ahead", type=int, default=2,
                    help="batches copied (and prepped) ahead of the round (≤ slots − 1)")
    ap.add_argument("--host-ahead-wait", type=int, default=1,
                    help="the host waits for a staging slot's last round before its copy "
                         "(no device-side barrier in the copy stream)")
    ap.add_argument("--pull-wt", type=int, default=1,
                    help="pull copy stores write-through (the batch leaves the copy XCD's L2)")
    ap.add_argument("--lane", default="split", choices=["split", "plain"])
    ap.add_argument("--scan-cus", type=int, default=0,
                    help="CUs the prep stream leaves to the round's scan (split lane)")
    ap.add_argument("--prep-ahead", type=int, default=1,
                    help="v3 round: hash, occurrence sort and chunk Grams of batch k+1 on their own stream")
    ap.add_argument("--hubs", type=int, default=0, help="HubParallelism (1 = reduce+bcast)")
    ap.add_argument("--latency-samples", type=int, default=2000)
    ap.add_argument("--ref", default="auto", choices=["auto", "on", "off"],
                    help="CPU reference-semantics accuracy on the same stream (rank 0)")
    ap.add_argument("--ref-max-examples", type=float, default=6e7)
    ap.add_argument("--engine-e2e", type=int, default=8388608,
                    help="JSON (and DIB) records timed through the whole engine (rank 0; 0 = "
                         "skip): 16 ticks of 524288 records, the steady state")
    ap.add_argument("--e2e-batch", type=int, default=524288,
                    help="records per engine tick in the e2e runs (16 spokes × 8192-row "
                         "rounds: 4 Synchronous rounds per tick, --roundRows)")
    ap.add_argument("--engine-latency", type=int, default=300,
                    help="forecasting records timed through the engine (rank 0; 0 = skip)")
    a = ap.parse_args(argv)

    comm, device = init_distributed()
    rank, world = comm.rank, comm.world
    on_gpu = device.type == "cuda"
    space = FeatureSpace(13, 0, 26, 1 << a.dim_log2)
    S, R = a.spokes, a.rows
    B = S * R

    # ---- the rank's shard of the synthetic raw stream, pinned, replayed like a Kafka log
    pool = []
    for k in range(a.pool):
        pb = PackedRaw(space, B, "cpu", on_gpu)
        tmp = synth_raw(space, B, start=shard_start(k, rank, world, B), seed=25)
        pb.batch.num.copy_(tmp.num)
        pb.batch.tok.copy_(tmp.tok)
        pb.batch.y.copy_(tmp.y.to(torch.int8))  # ±1 exactly
        pool.append(pb)
    nslots = a.pool if a.ingest == "device" else a.slots
    dev = [PackedRaw(space, B, device, False) for _ in range(nslots)]
    if a.ingest == "device":
        for d, p in zip(dev, pool):
            d.flat.copy_(p.flat)

    if a.learner == "SVM":
        learner = SVM({"variant": "PA-I", "C": 1.0, "modelDtype": a.model_dtype}, space, device)
    else:
        learner = LogisticRegression({"learningRate": 0.1, "modelDtype": a.model_dtype}, space,
                                     device)
    assert learner.seq_capable()
    proto = Synchronous(comm, learner, {"virtualSpokes": S,
                                        **({"HubParallelism": a.hubs} if a.hubs else {})})
    proto.time_collectives = on_gpu and world > 1

    # ---- ingest lane: the pull copy runs on a CU-masked slice inside one XCD and the
    # round on the complementary CUs ("split"), or both on ordinary streams ("plain")
    raw_streams = []
    lane = {"copy": None, "compute": None}
    if on_gpu:
        native.hip().omldm_pull_copy_set_wt(int(a.pull_wt))
        lane = {"copy": torch.cuda.Stream(device), "compute": torch.cuda.current_stream(device)}
        if a.lane == "split" and a.ingest_cus > 0:
            raw = native.hip().omldm_stream_create_cumask_ex(a.ingest_cus, 0, a.cu_layout)
            rawc = native.hip().omldm_stream_create_cumask_ex(a.ingest_cus, 1, a.cu_layout)
            assert raw and rawc, "hipExtStreamCreateWithCUMask failed"
            raw_streams += [raw, rawc]
            lane = {"copy": torch.cuda.ExternalStream(raw, device=device),
                    "compute": torch.cuda.ExternalStream(rawc, device=device)}
    # passes 1-2 of the next round (hash + chunk Grams, model-independent) run on their own
    # stream as soon as its batch has landed, overlapping the current round's scan
    prep_stream = None
    v3 = on_gpu and L.scan3_eligible(dev[0].batch, R, learner.rule.bias)
    if on_gpu and a.prep_ahead and v3:
        if a.lane == "split" and a.ingest_cus > 0:
            # the prep kernels fill every CU they may use; a few CUs (spread over the
            # XCDs) kept for the compute stream let the next scan start on time instead
            # of waiting for prep workgroups to drain from a CU (each scan workgroup
            # takes a whole CU's LDS)
            from omldm_amd.ops.ingest import copy_cu_bits, cumask_stream, reserve_cu_bits
            total = torch.cuda.get_device_properties(device).multi_processor_count
            taken = copy_cu_bits(total, a.ingest_cus, a.cu_layout)
            keep = reserve_cu_bits(total, a.scan_cus, taken)
            prep_stream, rawp = cumask_stream(set(range(total)) - taken - keep, total, device)
            raw_streams.append(rawp)
        else:
            prep_stream = torch.cuda.Stream(device)
    copied = [torch.cuda.Event() for _ in range(nslots)] if on_gpu else None
    consumed = [torch.cuda.Event() for _ in range(nslots)] if on_gpu else None
    # device time of each batch's copy and each round: timing-event pairs recorded in the
    # loop, read after the final sync (no synchronisation inside the timed window), so the
    # record says which lane bounded the step
    ev_copy: dict = {}
    ev_round: dict = {}

    def _tev():
        return torch.cuda.Event(enable_timing=True)

    def h2d(dst: torch.Tensor, src: torch.Tensor):
        if a.h2d == "pull":  # the GPU pulls the pinned batch over PCIe (csrc/kernels/ingest.hip)
            native.check(native.hip().omldm_pull_copy(src.data_ptr(), dst.data_ptr(), src.numel(),
                                                      a.pull_blocks, lane["copy"].cuda_stream),
                         "pull_copy")
        else:
            dst.copy_(src, non_blocking=True)

    def prepare(slot: int, after=None):
        if prep_stream is None:
            return
        if after is not None:
            prep_stream.wait_event(after)
        b = dev[slot].batch  # passes 1-3 of the table scan (csrc/kernels/linear_scan3.hip)
        b.prep = L.linear_scan3_prepare(b, R, S, space.dim, bool(learner.rule.bias),
                                        learner.rule, slot=slot, stream=prep_stream)

    def prefetch(k: int):
        if a.ingest == "device":
            return
        slot, src = k % nslots, pool[k % a.pool]
        if on_gpu:
            cs = lane["copy"]
            with torch.cuda.stream(cs):
                # the host keeps at most `nslots - 1` rounds ahead of the device: it waits for
                # the round that last used this slot, so the copy needs no device-side wait
                # (a cross-stream barrier packet held every copy ≈ 11 µs behind the previous
                # one, and the copies are the step's bound)
                if a.host_ahead_wait:
                    consumed[slot].synchronize()
                else:
                    cs.wait_event(consumed[slot])
                e0, e1 = _tev(), _tev()
                e0.record(cs)
                h2d(dev[slot].flat, src.flat)
                e1.record(cs)
                ev_copy[k] = (e0, e1)
                copied[slot].record(cs)
            prepare(slot, copied[slot])
        else:
            dev[slot].flat.copy_(src.flat)

    def _round(k: int, batch):
        if not on_gpu:
            proto.round(batch)
            return
        e0, e1 = _tev(), _tev()
        e0.record()
        proto.round(batch)
        e1.record()
        ev_round[k] = (e0, e1)

    def _step(k: int):
        if a.ingest == "device":
            if prep_stream is not None:  # the next batch's passes 1-2 overlap this scan
                nb = (k + 1) % a.pool
                prep_stream.wait_stream(torch.cuda.current_stream(device))
                prepare(nb)
            _round(k, dev[k % a.pool].batch)
            return
        slot = k % nslots
        if ahead == 1 and k + 1 < n_rounds:
            prefetch(k + 1)
        if on_gpu and not (v3 and prep_stream is not None):
            # (with a prep made ahead the round waits on the prep's event, which follows the
            # copy: a second cross-stream wait cost the round's launch ≈ 7 µs per step)
            torch.cuda.current_stream().wait_event(copied[slot])
        _round(k, dev[slot].batch)
        if on_gpu:
            consumed[slot].record()
        if ahead > 1 and k + ahead < n_rounds:
            # the copy of batch k + ahead goes after this round is queued: the host may wait
            # for round k + ahead − nslots (its slot) while the device already has round k
            # (no copy of a batch past the last round: the final sync would wait for it)
            prefetch(k + ahead)

    def step(k: int):
        if on_gpu:
            with torch.cuda.stream(lane["compute"]):
                _step(k)
        else:
            _step(k)

    def sync():
        if on_gpu:
            torch.cuda.synchronize(device)
        comm.barrier()
        if on_gpu:
            torch.cuda.synchronize(device)

    if on_gpu and a.settle_ms > 0:
        # leave the idle power state before anything is timed: the device runs dense
        # matmuls on scratch tensors (nothing of the model or the stream is touched)
        xs = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16)
        t_end = time.perf_counter() + a.settle_ms / 1e3
        while time.perf_counter() < t_end:
            for _ in range(8):
                xs = torch.tanh(xs @ xs)
            torch.cuda.synchronize(device)
        del xs
    if on_gpu:
        for e in consumed:
            e.record()
    ahead = max(1, min(int(a.ahead), nslots - 1)) if a.ingest != "device" else 1
    n_rounds = a.warmup + a.steps
    for j in range(min(ahead, n_rounds)):
        prefetch(j)
    for k in range(a.warmup):
        step(k)
    sync()
    if proto.time_collectives:
        proto.collective_time_ms()  # drop the warmup rounds' events
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        step(k)
    t_enq = time.perf_counter() - t0  # the host's enqueue time (the device may lag behind)
    sync()
    elapsed = time.perf_counter() - t0
    coll_ms = proto.collective_time_ms() if proto.time_collectives else None
    timed = range(a.warmup, a.warmup + a.steps)

    def _dev_ms(evs):
        v = [evs[k][0].elapsed_time(evs[k][1]) for k in timed if k in evs]
        return round(sum(v) / len(v), 4) if v else None

    copy_dev_ms = _dev_ms(ev_copy) if on_gpu else None
    round_dev_ms = _dev_ms(ev_round) if on_gpu else None
    # the v3 round's in-launch combiners never gave up on a spoke (a timeout would leave a
    # spoke's update out of the round accumulator): checked after the timed window
    comb_err = int(native.hip().omldm_scan3_comb_err()) if on_gpu else 0
    if comb_err:
        raise RuntimeError("v3 scan: a combiner workgroup timed out during the bench rounds")
    el = torch.tensor([elapsed, coll_ms or 0.0], dtype=torch.float64,
                      device=device if comm.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el[0].item())
    rounds = a.warmup + a.steps

    # ---- model quality: the trained model and the CPU reference-semantics learner
    test = synth_raw(space, 20000, start=TEST_START, seed=25)
    testh = test.hashed(space)

    def accuracy(w: torch.Tensor) -> float:
        s = L.linear_predict(w.detach().float().cpu(), testh)
        return float(((s >= 0).float() * 2 - 1 == testh.y).float().mean())

    acc = accuracy(learner.w) if rank == 0 else None
    fitted = learner.running_totals()["fitted"]
    ref_acc = ref64_acc = ref64_maxdw = None
    P_ref = S * world
    do_ref = a.ref == "on" or (a.ref == "auto" and rounds * B * world <= a.ref_max_examples)
    if rank == 0 and do_ref:
        # same global stream, same rounds: round k of rank r trained pool batch k % pool
        wref, dref = torch.zeros(space.dim), torch.zeros(space.dim + 2)
        ref_rule = learner.rule
        gpool = []
        for k in range(min(a.pool, rounds)):
            parts = [synth_raw(space, B, start=shard_start(k, r, world, B), seed=25)
                     for r in range(world)]
            gpool.append(RawBatch(torch.cat([p.num for p in parts]),
                                  torch.cat([p.tok for p in parts]),
                                  torch.cat([p.y for p in parts])))
        w64, d64 = torch.zeros(space.dim, dtype=torch.float64), \
            torch.zeros(space.dim + 2, dtype=torch.float64)
        for k in range(rounds):
            L.linear_seq_round(wref, gpool[k % a.pool], R, P_ref, dref, ref_rule, 1.0)
            L.linear_apply(wref, None, dref)
            if a.learner == "SVM":  # the reference's Double learner on the same stream
                L.linear_seq_round64(w64, gpool[k % a.pool], R, P_ref, d64, ref_rule, 1.0)
                L.linear_apply64(w64, d64)
        ref_acc = accuracy(wref)
        if a.learner == "SVM":
            ref64_acc = accuracy(w64.float())
            ref64_maxdw = float((w64 - learner.w.detach().double().cpu()).abs().max())

    # ---- p50 single-point predict latency: the persistent serving wave reading a pinned
    # mailbox (raw tokens, hashed by the wave), against the trained fp32 model
    lat_us = []
    if rank == 0 and on_gpu and a.latency_samples > 0:
        from omldm_amd.ops.serving import PredictServer

        torch.cuda.synchronize(device)
        server = PredictServer(learner.w, space.dn, space.dc, True, cat_span=-1)
        server.start(lifetime_us=20_000_000)
        num_h = test.num[0].contiguous()
        tok_h = test.tok[0].contiguous()
        got = None
        for i in range(a.latency_samples + 50):
            t = time.perf_counter()
            got = server.request_raw(num_h.data_ptr(), tok_h.data_ptr())
            if i >= 50:
                lat_us.append((time.perf_counter() - t) * 1e6)
        server.close()
        ref = float(L.linear_predict(learner.w.cpu(), testh.slice(0, 1))[0])
        assert abs(got[0] - ref) <= 1e-3 * max(1.0, abs(ref)), (got, ref)
    p50 = statistics.median(lat_us) if lat_us else None
    p99 = sorted(lat_us)[int(0.99 * (len(lat_us) - 1))] if lat_us else None

    eng = engine_forecast_latency(a.engine_latency) if (rank == 0 and on_gpu and
                                                         a.engine_latency > 0) else None
    e2e = engine_e2e_rate(a.engine_e2e, a.e2e_batch) \
        if (rank == 0 and on_gpu and a.engine_e2e > 0) else None
    e2e_dib = engine_e2e_rate(a.engine_e2e, a.e2e_batch, fmt="dib") if e2e is not None else None

    total_examples = a.steps * B * world
    value = total_examples / elapsed
    if rank == 0:
        wire = pool[0].wire_bytes
        base = cpu_baseline() if a.learner == "SVM" else None
        out = {
            "metric": METRIC if a.learner == "SVM" else
                      "training examples/sec (whole node), online logistic regression, "
                      "1M-dim hashed features (BASELINE config 2)",
            "value": round(value, 1), "unit": "examples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "host_enqueue_ms_per_step": round(t_enq / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base["value"], 2) if base else None,
            "baseline": {"value": base["value"], "source": base["source"],
                         "what": "reference-class CPU baseline (BASELINE.md: the reference "
                                 "publishes no number): the reference's semantics in C++, "
                                 "P = 16 sequential PA-I spokes + averaging (the reference's "
                                 "default parallelism), measured on the MI355X box's host "
                                 "CPU (bench/cpu_reference.py)"} if base else None,
            "dtype": a.model_dtype,
            "ingest_pipeline": None if a.ingest != "pinned" else {
                "batches_copied_ahead": ahead,
                "pcie_copies_in_timed_window": max(0, a.steps - ahead),
                "note": "each round's batch is pulled over PCIe `ahead` rounds before it "
                        "trains (the copies of the first timed rounds' batches ran during "
                        "the warmup; no batch past the last round is copied); the rate over "
                        "--steps 100 is the steady-state check"},
            "data": "synthetic (Criteo-shaped raw stream: fp32 numerical features, 32-bit "
                    "category tokens hashed on the GPU inside the timed round, int8 ±1 labels; "
                    f"{wire // B} B/example on the wire; pinned host pool replayed, H2D in "
                    "timed loop)" if a.ingest == "pinned" else
                    "synthetic (HBM-resident replay, tokens hashed in the round)",
            "config": {"model": ("linear SVM PA-I" if a.learner == "SVM" else
                                 "logistic regression (SGD)") +
                                f", 2^{a.dim_log2} hashed features (13 num + 26 cat + bias), " +
                                ("fp32" if a.model_dtype == "fp32" else
                                 "bf16 model (margins on the bf16 weights, fp32 master)"),
                       "global_batch": B * world, "seq_len": None,
                       "parallelism": f"dp{world}", "protocol": "Synchronous",
                       "spokes_per_gpu": S, "rows_per_spoke_per_round": R,
                       "semantics": "exact sequential per spoke, replicas averaged per round"},
            "device_copy_ms_per_step": copy_dev_ms,
            "device_round_ms_per_step": round_dev_ms,
            "step_bound": None if copy_dev_ms is None or round_dev_ms is None else
                          ("copy (H2D)" if copy_dev_ms > round_dev_ms else "round"),
            "device_time_semantics": "mean device time of the timed steps' batch copies "
                                     "(copy lane) and rounds (compute lane, prep + scan + "
                                     "apply), from timing-event pairs read after the final "
                                     "sync (the copies of the first `batches_copied_ahead` "
                                     "timed rounds ran in the warmup)",
            "p50_predict_latency_us": None if p50 is None else round(p50, 2),
            "p99_predict_latency_us": None if p99 is None else round(p99, 2),
            "engine_forecast_p50_us": None if eng is None else eng["p50"],
            "engine_forecast_p99_us": None if eng is None else eng["p99"],
            "engine_forecast_lane": None if eng is None else eng["lane"],
            "engine_forecast_stage_us": None if eng is None else eng["stage_us"],
            "engine_forecast_training_p50_us": None if eng is None else eng["train_p50"],
            "engine_forecast_training_p99_us": None if eng is None else eng["train_p99"],
            "engine_forecast_training_n": None if eng is None else eng["train_n"],
            "engine_forecast_training_stage_us": None if eng is None else eng["train_stage_us"],
            "engine_forecast_training_records_per_s":
                None if eng is None else eng["train_records_per_s"],
            "engine_forecast_semantics": None if eng is None else eng["what"],
            "engine_e2e_records_per_s": None if e2e is None else e2e["records_per_s"],
            "engine_e2e_semantics": None if e2e is None else
            f"JSON DataInstance file topic -> GPU parse + hashing -> holdout -> Synchronous "
            f"linear SVM fp32, {e2e['spokes']} spokes, {e2e['records']} records timed "
            f"(one GPU, rank 0), {e2e['record_bytes']} B/record, ticks of {e2e['batch']} "
            f"records = rounds of <= 8192 rows per spoke",
            "engine_e2e_dib_records_per_s": None if e2e_dib is None else e2e_dib["records_per_s"],
            "engine_e2e_stage_ms_per_tick": None if e2e is None else {
                "json": {"ms_per_tick": e2e["ms_per_tick"], **e2e["stage_ms_per_tick"]},
                "dib": {"ms_per_tick": e2e_dib["ms_per_tick"], **e2e_dib["stage_ms_per_tick"]}},
            "engine_e2e_dib_semantics": None if e2e_dib is None else
            f"the same records as binary DIB records ({e2e_dib['record_bytes']} B/record, "
            f"omldm_amd/io/dib.py) through the same engine path, {e2e_dib['records']} timed",
            "per_gpu_examples_per_s": round(value / world, 1),
            "holdout_accuracy": None if acc is None else round(acc, 4),
            "ref_holdout_accuracy": None if ref_acc is None else round(ref_acc, 4),
            "ref_semantics": f"CPU sequential PA-I, P={P_ref} spokes, same stream and "
                             f"{rounds * B * world} examples (csrc/host/rawwire.cpp)",
            "ref64_holdout_accuracy": None if ref64_acc is None else round(ref64_acc, 4),
            "ref64_accuracy_gap_pt": None if ref64_acc is None or acc is None
                                     else round((ref64_acc - acc) * 100, 3),
            "ref64_max_abs_dw": None if ref64_maxdw is None else float(f"{ref64_maxdw:.3e}"),
            "ref64_semantics": "the same sequential PA-I learner in DOUBLE precision (the "
                               "reference's Breeze Double model, StateAccumulators.scala:5,26)"
                               ", same stream, spokes and rounds; holdout accuracy and the "
                               "max |w64 - w| against the GPU's fp32 model",
            "accuracy_gap_pt": None if ref_acc is None or acc is None
                               else round((ref_acc - acc) * 100, 3),
            "fitted_examples_rank0": fitted,
            "backend": comm.backend, "rccl_ranks": world if comm.backend == "nccl" else 0,
            "collective_us_per_step": None if coll_ms is None
                                      else round(float(el[1].item()) * 1e3 / a.steps, 2),
            "combiner_timeouts": comb_err,
            "round_kernel": ("linear_scan3 (v3 table scan)" if v3 else "linear_seq (v1)") if on_gpu
                            else "cpu",
            "numa": comm.placement, "ingest_lane": a.lane if on_gpu else None,
            "device": torch.cuda.get_device_name(device) if on_gpu else "cpu",
        }
        print(json.dumps(out), flush=True)
    if on_gpu:
        torch.cuda.synchronize(device)
        for evs in (copied, consumed):
            if evs:
                evs.clear()
        lane.clear()
        import gc

        gc.collect()
        for rs in raw_streams:
            native.hip().omldm_stream_destroy(rs)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if os.environ.get("OMLDM_DUMP_MAPS"):  # diagnostics: attribute exit-time crash addresses
        with open("/proc/self/maps") as f, open(os.environ["OMLDM_DUMP_MAPS"], "w") as g:
            g.write(f.read())
    return 0


if __name__ == "__main__":
    sys.exit(main())
