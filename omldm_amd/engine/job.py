"""The per-rank streaming job: control plane, data plane, queries, statistics, termination.

Reference dataflow (omldm/Job.scala:35-168, omldm/job/FlinkLearning.scala:33-152):
requests → PipelineMap (p=1) → broadcast to every spoke; training ∪ forecasting data →
FlinkSpoke (holdout routing, per-pipeline learning, predictions, query answers) ↔ FlinkHub
(parameter server, statistics) with the hub→spoke leg through the Kafka psMessages
topic; ResponseConstructor reduces query answers; StatisticsOperator detects idleness
and emits JobStatistics to the performance topic, which kills the job.

MI355X-native redesign. One process per GPU; every process runs this loop in lockstep
("tick" = one micro-batch per rank):
  1. rank 0 drains the requests topic through PipelineMap; the resulting control
     messages are broadcast to all ranks (one small object broadcast per tick);
  2. each rank polls its partitions of trainingData/forecastingData, parses them with
     the C++ scanner into one HashedBatch, and moves it to HBM;
  3. forecasting rows → every pipeline's predict kernel → predictions topic;
  4. training rows → holdout routing → every pipeline's protocol round (the parameter
     server is an RCCL collective inside the round, not a Kafka loop);
  5. Query requests are answered from the holdout set with one all-reduce
     (ResponseConstructor semantics) and written by rank 0 to the responses topic;
  6. a 2-float all-reduce per tick carries global activity and the termination flag
     (idle timeout → final statistics → performance topic → graceful stop);
  7. optional asynchronous checkpoint every ``checkInterval`` ms.
"""
from __future__ import annotations

import collections
import json
import os
import time
from contextlib import nullcontext as _nullcontext

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.api.schemas import Prediction, Request
from omldm_amd.engine.holdout import HoldoutSet
from omldm_amd.engine.ingest import TickBlock, TickIngest
from omldm_amd.engine.model_store import ModelStore
from omldm_amd.engine.pipeline import Pipeline
from omldm_amd.engine.pipeline_map import ALL, PipelineMap
from omldm_amd.engine import statistics as ST
from omldm_amd.io.egress import EgressWriter, RawRecords, format_predictions_chunks
from omldm_amd.io.parse import OP_FORECASTING, OP_TRAINING, RawView, parse_block
from omldm_amd.io.transport import join_block
from omldm_amd.io.transport import Consumer, broker_for
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import Synchronous
from omldm_amd.utils.config import JobConfig
from omldm_amd.utils import tracing


EMPTY_BLOCK = (b"", np.zeros(1, dtype=np.int64))


def concat_blocks(blocks: list) -> tuple[bytes, np.ndarray]:
    blocks = [b for b in blocks if len(b[1]) > 1]
    if not blocks:
        return EMPTY_BLOCK
    if len(blocks) == 1:
        return blocks[0]
    offs, base = [np.zeros(1, dtype=np.int64)], 0
    for buf, o in blocks:
        offs.append(o[1:] + base)
        base += len(buf)
    return b"".join(b for b, _ in blocks), np.concatenate(offs)


class Job:
    def __init__(self, cfg: JobConfig, comm: Comm, device):
        self.cfg = cfg
        self.comm = comm
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.rank, self.world = comm.rank, comm.world
        self.space = FeatureSpace(cfg.numFeatures, cfg.discreteFeatures, cfg.catFeatures,
                                  cfg.hashDim, field_aware=cfg.fieldAware)
        self.spokes = cfg.spokesPerDevice or max(1, cfg.parallelism // self.world)
        # spoke-parallelism gate (FlinkSpoke.scala:69-71,145-156,345-348): the job records
        # the largest spoke parallelism it has run at (kept in checkpoints); while it runs
        # below it — restored onto fewer spokes — Create requests wait in request_buffer,
        # and a restore at that parallelism or more creates them first thing
        self.parallelism = self.spokes * self.world
        self.spoke_parallelism = self.parallelism
        self.request_buffer: list = []
        b = {k: broker_for(getattr(cfg, k + "Addr")) for k in
             ("trainingData", "forecastingData", "requests", "responses", "predictions",
              "performance")}
        self.brokers = b
        self.train_in = Consumer(b["trainingData"], cfg.trainingDataTopic, self.rank, self.world)
        self.fcst_in = Consumer(b["forecastingData"], cfg.forecastingDataTopic, self.rank,
                                self.world)
        self.req_in = Consumer(b["requests"], cfg.requestsTopic, all_partitions=True) \
            if self.rank == 0 else None
        self.pmap = PipelineMap() if self.rank == 0 else None
        # this rank's training ∪ forecasting records, one pinned block per tick, read one
        # tick ahead on a background thread (engine/ingest.py)
        # GPU ranks: the ingest copies run on one XCD's CUs, everything else on the rest
        self.lanes = None
        if self.device.type == "cuda" and cfg.gpuParse and cfg.ingestCUs > 0:
            from omldm_amd.ops.ingest import XcdLanes

            self.lanes = XcdLanes.get(self.device, cfg.ingestCUs)
        # forecasting records: a per-record low-latency lane on the resident serving wave
        # (engine/forecast_server.py) on GPU ranks; otherwise batched with the training rows
        fs = str(cfg.forecastServer).lower()
        self.fserver = None
        if fs in ("true", "1") or (fs == "auto" and self.device.type == "cuda"):
            from omldm_amd.engine.forecast_server import ForecastServer

            self.fserver = ForecastServer(self)
        self.ingest = TickIngest([self.train_in] if self.fserver else
                                 [self.train_in, self.fcst_in], cfg.batchSize,
                                 pinned=self.device.type == "cuda",
                                 prefetch=str(cfg.prefetch).lower() in ("true", "1") or (
                                     str(cfg.prefetch).lower() == "auto" and
                                     self.device.type == "cuda"),
                                 device=self.device if cfg.gpuParse else None,
                                 space=self.space if cfg.gpuParse else None,
                                 copy_blocks=16 if self.lanes else 128,
                                 copy_method=str(cfg.ingestCopy).lower(),
                                 copy_stream=self.lanes.copy if self.lanes else None,
                                 parse_stream=self.lanes.aux if self.lanes else None)
        self._committed = None  # consumer offsets after the last processed block
        # predictions leave through a producer thread (formatted natively, io/egress.py)
        self.egress = EgressWriter(b["predictions"], enabled=self.device.type == "cuda")
        self.pipes: dict[int, Pipeline] = {}
        # one counter + FIFO test set per virtual spoke (FlinkSpoke.scala:38-41,95-104)
        self.holdout = HoldoutSet(self.space, cfg.testSetSize, self.device, spokes=self.spokes)
        self.store = ModelStore(self.space.dim, self.device)
        self.record_buffer: list = []          # blocks (buf, offsets) waiting for a Create
        self._buffered = 0
        self.idle = ST.IdleDetector(cfg.timeout)
        self.ticks = 0
        self.terminated = False
        self.final_stats = None
        self.counters = {"records": 0, "invalid": 0, "predictions": 0, "responses": 0,
                         "dropped_buffer": 0}
        self._fc_lat: collections.deque = collections.deque(maxlen=4096)  # ms per forecast batch
        self._gpu_parser = None
        if self.device.type == "cuda" and cfg.gpuParse:
            from omldm_amd.ops.ingest import GpuJsonParser

            self._gpu_parser = GpuJsonParser(self.device)
        self._trained_global = 0
        # per-tick control flags: [active records, terminate, training rows, pending
        # requests, checkpoint due] — a host tensor reduced over the gloo control group
        self._flags = torch.zeros(5, dtype=torch.float64)
        # multi-rank control plane: rank 0 polls requests at the end of a tick and the
        # tick's flag all-reduce says whether the next tick must broadcast them — ticks
        # without requests (nearly all) cost no object broadcast
        self._ctrl_pending: list = []
        self._ctrl_due = True
        from omldm_amd.utils.fault import FaultPlan, Watchdog

        self.faults = FaultPlan.from_config(cfg, self.rank)
        if self.faults:
            comm.fault = self.faults
        self.watchdog = Watchdog(cfg.watchdogTimeout / 1000.0, self.rank) \
            if cfg.watchdogTimeout > 0 else None
        self.checkpointer = None
        if cfg.checkpointing or cfg.restore:
            from omldm_amd.utils.checkpoint import Checkpointer

            import uuid

            nonce = uuid.uuid4().hex if self.rank == 0 else None
            if self.world > 1:  # every rank tags its done markers with rank 0's run nonce
                nonce = comm.broadcast_object(nonce, src=0)
            self.checkpointer = Checkpointer(cfg, self.rank, self.world, nonce=nonce)
            if cfg.restore:
                self.checkpointer.restore(self)
        if self.fserver is not None:
            self.fserver.reconfigure()
            self.fserver.start()
        # device time of the training rounds and of the coalesced collectives (lagged
        # event pairs, no host sync: utils/devtimer.py)
        self._train_timer = self._coll_timer = None
        self._health = None
        self._ready_ev = None          # the staging slot's parse event (route ahead)
        self._route_stream = None
        self._holdout_read_ev = None   # compute-stream reads of the holdout rings (queries)
        if self.device.type == "cuda":
            from omldm_amd.utils.devtimer import LaggedTimer
            from omldm_amd.utils.health import DeviceHealth

            self._train_timer, self._coll_timer = LaggedTimer(), LaggedTimer()
            # dropped updates / combiner timeouts fail the job, read one tick late
            self._health = DeviceHealth(self.device)
        self._t_start = time.time()
        # diagnostics / multi-rank tests: a per-tick digest of every pipeline's model
        # (replica agreement across ranks) and the final models, under this directory
        self._trace_dir = os.environ.get("OMLDM_TRACE_MODELS") or None

    def _trace_models(self, final: bool = False) -> None:
        os.makedirs(self._trace_dir, exist_ok=True)
        if final:
            for pid, pipe in self.pipes.items():
                torch.save(pipe.learner.state_vector().detach().cpu(),
                           os.path.join(self._trace_dir, f"rank{self.rank}_final_{pid}.pt"))
            return
        import zlib

        recs = []
        for pid in sorted(self.pipes):
            v = self.pipes[pid].learner.state_vector().detach().float().cpu().contiguous()
            recs.append({"tick": self.ticks, "pid": pid,
                         "protocol": self.pipes[pid].protocol_name,
                         "crc": zlib.crc32(v.numpy().tobytes()), "sum": float(v.double().sum())})
        with open(os.path.join(self._trace_dir, f"rank{self.rank}.jsonl"), "a") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")

    def _coll_device(self):
        return self.device if self.comm.backend == "nccl" else torch.device("cpu")

    # ------------------------------------------------------------------ control
    def _poll_requests(self) -> list:
        msgs = []
        for rec in self.req_in.poll(self.cfg.requestBufferSize):
            for m in self.pmap.process(rec):
                msgs.append((m.network_id, m.destination, m.request.to_obj()))
        return msgs

    def _control(self):
        if self.world == 1:
            msgs = getattr(self, "_restored_ctrl", []) + self._poll_requests()
            self._restored_ctrl = []
        elif self._ctrl_due:
            msgs = self.comm.broadcast_object(self._ctrl_pending if self.rank == 0 else None,
                                              src=0)
            self._ctrl_pending = []
        else:
            msgs = []
        gated = self.cfg.parallelismGate and self.parallelism < self.spoke_parallelism
        if self.request_buffer and not gated:
            msgs = self.request_buffer + list(msgs)
            self.request_buffer = []
        queries = []
        moves = self.fserver is not None and any(
            Request.from_json(robj).request in ("Create", "Delete") for _, _, robj in msgs)
        if moves:
            self.fserver.suspend()  # a Create may grow (move) the model store arena
        for net, dest, robj in msgs:
            req = Request.from_json(robj)
            if dest not in (ALL, self.rank) and req.request != "Query":
                continue
            if req.request == "Create":
                if gated:
                    if len(self.request_buffer) < self.cfg.requestBufferSize:
                        self.request_buffer.append((net, dest, robj))
                    else:
                        self._bad_request(req, "request buffer full")
                elif net not in self.pipes:
                    try:
                        self.pipes[net] = Pipeline(req, self.space, self.comm, self.device,
                                                   self.spokes, self.cfg.parallelism,
                                                   self.cfg.maxMsgParams, store=self.store,
                                                   seed=self.cfg.seed)
                    except (ValueError, TypeError, KeyError) as e:
                        # an ill-typed configuration (every rank fails the same way): the
                        # request is dropped and counted, the job goes on
                        self._bad_request(req, e)
            elif req.request == "Update" and net in self.pipes:
                try:
                    self.pipes[net].update(req)
                except (ValueError, TypeError, KeyError) as e:
                    self._bad_request(req, e)
            elif req.request == "Delete":
                old = self.pipes.pop(net, None)
                if old is not None:
                    old.close()
            elif req.request == "Query" and net in self.pipes:
                queries.append(req)
        if moves:
            self.fserver.reconfigure()
        return len(msgs), queries

    def _bad_request(self, req, err) -> None:
        self.counters["invalid_requests"] = self.counters.get("invalid_requests", 0) + 1
        if self.rank == 0:
            print(f"[omldm] request {req.request} id={req.id} dropped: {err}", flush=True)

    # --------------------------------------------------------------------- data
    def _poll(self):
        """This tick's records: a pinned ``TickBlock`` (no per-record Python objects), a
        (bytes, offsets) block when records buffered before the first Create are
        replayed, or ``EMPTY_BLOCK``."""
        blk = self.ingest.next()
        self._committed = blk.offsets
        nrec = blk.n
        if not self.pipes:
            # reference: points wait in a bounded record buffer until a pipeline exists
            room = max(0, self.cfg.recordBufferSize - self._buffered)
            if nrec:
                buf, offs = blk.to_bytes()
                if nrec > room:
                    self.counters["dropped_buffer"] += nrec - room
                    buf, offs = buf[:int(offs[room])], offs[:room + 1]
                    nrec = room
                if nrec:
                    self.record_buffer.append((buf, offs))
                    self._buffered += nrec
            return EMPTY_BLOCK
        if self.record_buffer:
            block = concat_blocks(self.record_buffer + [blk.to_bytes()])
            self.record_buffer, self._buffered = [], 0
            return block
        return blk

    def consumer_offsets(self, fc_lane: dict | None = None) -> dict:
        """Offsets after the last block this job processed (the prefetcher may have read
        further; those records are re-read after a restore). With the per-record lane the
        forecasting offsets are ``fc_lane`` (ForecastServer.snapshot: answered or handed
        back), never the live consumer position (records polled but not yet answered)."""
        train = dict(self._committed[0]) if self._committed is not None else \
            dict(self.train_in.offsets)
        if fc_lane is not None:
            fc = fc_lane
        elif self._committed is not None and len(self._committed) > 1:
            fc = self._committed[1]
        else:
            fc = self.fcst_in.offsets
        return {"train": train, "forecast": dict(fc)}

    def _forecast(self, batch: HashedBatch, raw: RawRecords | None):
        """Predictions of every pipeline for the forecasting rows; ``raw`` holds their
        JSON records, echoed in each Prediction (one native-formatted block per
        pipeline, io/egress.py)."""
        prod = self.brokers["predictions"]
        out: dict[int, np.ndarray] = {}
        # pipelines whose weights live in the HBM model store: ONE multi-model launch
        groups: dict[bool, list] = {}
        for pid in sorted(self.pipes):
            p = self.pipes[pid]
            if p.store is not None:
                groups.setdefault(bool(p.learner.rule.bias), []).append(p)
        for bias, pipes in groups.items():
            with tracing.range("predict:store"):
                s = self.store.scores(batch, [p.store_row for p in pipes], bias=bias)
                for j, p in enumerate(pipes):
                    out[p.id] = p.scores_to_predictions(s[:, j]).float().cpu().numpy()
        for pid in sorted(self.pipes):
            if pid not in out:
                with tracing.range(f"predict:{pid}"):
                    out[pid] = self.pipes[pid].predict(batch).float().cpu().numpy()
        with tracing.range("egress"):
            for pid in sorted(out):
                preds = out[pid]
                if raw is not None:
                    for block, offs in format_predictions_chunks(raw, pid, preds):
                        self.egress.submit(self.cfg.predictionsTopic, block, offs)
                else:
                    for p in preds.tolist():
                        prod.produce(self.cfg.predictionsTopic, Prediction(pid, None, p).to_json())
                self.counters["predictions"] += len(preds)

    def _forecast_fallback(self) -> None:
        """Forecasting records the lane handed back (no pipeline existed when they came):
        predicted in one batch by every pipeline, like the batched path."""
        recs = self.fserver.take_fallback()
        if not recs:
            return
        if not self.pipes:  # no pipeline yet: keep them, bounded like the record buffer
            room = self.cfg.recordBufferSize
            if len(recs) > room:
                self.counters["dropped_buffer"] += len(recs) - room
                recs = recs[len(recs) - room:]
            self.fserver.fallback.extendleft(reversed(recs))
            return
        buf, offs = join_block(recs)
        batch, op, _ = parse_block(buf, offs, self.space, self.cfg.parseThreads)
        fidx = np.nonzero(op == OP_FORECASTING)[0]
        self.counters["invalid"] += int(len(recs) - len(fidx))
        if len(fidx):
            raw = RawRecords.from_view(batch.raw, fidx)
            self._forecast(batch.without_raw().select(torch.from_numpy(fidx)).to(self.device), raw)

    def _route_ahead(self, batch: HashedBatch):
        """GPU ticks whose training rows are a parsed staging slot (``self._ready_ev``):
        the holdout routing and the v3 prep of the linear pipelines run on the route stream,
        which waits only for that slot's parse — not for the previous tick's round on the
        compute stream — so they overlap it; the compute stream waits for them. None: the
        caller routes on the compute stream."""
        ev_in = self._ready_ev
        rr = int(self.cfg.roundRows)
        if ev_in is None or self.device.type != "cuda" or not batch.B or \
                (rr > 0 and batch.B > rr * self.spokes) or \
                str(self.cfg.routeAhead).lower() in ("false", "0"):
            return None
        if self._route_stream is None:
            self._route_stream = self.lanes.prep if self.lanes is not None else \
                torch.cuda.Stream(self.device)
        ps, cur = self._route_stream, torch.cuda.current_stream(self.device)
        ps.wait_event(ev_in)
        if self._holdout_read_ev is not None:  # queries read the rings the route rewrites
            ps.wait_event(self._holdout_read_ev)
            self._holdout_read_ev = None
        with torch.cuda.stream(ps):
            routed = self.holdout.route(batch)
            p = self._linear_prep_pipe()  # one prep per tick (other prep keys make theirs)
            if p is not None:
                p.learner.prepare_ahead(routed, p.protocol._ctx(fused=True), ps)
        padded = routed._padded[1] if routed._padded is not None else None
        for b in (routed, padded):
            if b is not None:
                for t in (b.num, b.cat, b.y):
                    t.record_stream(cur)  # allocated on the route stream, read on compute
        ev = torch.cuda.Event()
        ev.record(ps)
        cur.wait_event(ev)
        return routed

    def _train(self, batch: HashedBatch, direct: HashedBatch | None = None):
        """One round of every pipeline. Synchronous pipelines train first and their
        round buffers are summed over ranks in ONE coalesced collective per hub layout
        (one flat bucket instead of one launch per pipeline); the other
        protocols run their own rounds."""
        with tracing.range("route"):
            routed = self._route_ahead(batch) if direct is None else None
            if routed is None:
                routed = self.holdout.route(batch)
        if direct is not None and direct.B:  # rows that bypass the holdout (no spoke layout)
            routed = HashedBatch.cat_batches([direct, routed]) if routed.B else direct
        parts = self._round_split(routed)
        if len(parts) > 1:
            self._prep_parts_ahead(parts)
        for part in parts:
            self._train_round(part)

    def _linear_prep_pipe(self):
        """The first hashed-linear pipeline without preprocessors (whose v3 prep every
        linear pipeline of the tick shares), or None."""
        from omldm_amd.models.linear import LinearLearner

        for pid in sorted(self.pipes):
            p = self.pipes[pid]
            if isinstance(p.learner, LinearLearner) and not p.preprocessors:
                return p
        return None

    def _prep_parts_ahead(self, parts: list) -> None:
        """Rounds 1 .. k-1 of a multi-round tick: their v3 preps (hash, occurrence flags,
        chunk Grams — model-independent) run on the route stream while round 0 scans, so
        each later round only scans (one prep workspace set per round, ops.linear ring)."""
        if self.device.type != "cuda" or str(self.cfg.prepAhead).lower() in ("false", "0"):
            return
        pipe = self._linear_prep_pipe()
        if pipe is None:
            return
        if self._route_stream is None:
            self._route_stream = self.lanes.prep if self.lanes is not None else \
                torch.cuda.Stream(self.device)
        ps, cur = self._route_stream, torch.cuda.current_stream(self.device)
        ps.wait_stream(cur)  # the parts' rows are cut on the compute stream
        ctx = pipe.protocol._ctx(fused=True)
        with torch.cuda.stream(ps):
            for part in parts[1:]:
                if not pipe.learner.prepare_ahead(part, ctx, ps):
                    return
                padded = part._padded[1] if part._padded is not None else None
                for b in (part, padded):
                    if b is not None:
                        for t in (b.num, b.cat, b.y):
                            t.record_stream(ps)  # read on the route stream, freed on compute

    def _round_split(self, routed: HashedBatch) -> list:
        """A tick whose spokes routed more than ``roundRows`` rows each trains in several
        Synchronous rounds: round i gives every spoke its rows [i·rr, (i+1)·rr) in stream
        order (the spoke's sequential order is kept; the model is averaged between rounds as
        for ticks of ``roundRows`` rows per spoke). Large ticks amortise the tick's host work
        (control, poll, flags, staging) over several rounds."""
        rr = int(self.cfg.roundRows)
        sh = routed.shards
        S = self.spokes
        if rr <= 0 or sh is None or len(sh) != S or max(sh) <= rr or not routed.B:
            return [routed]
        R = max(sh)
        k = -(-R // rr)
        out = []
        if len(set(sh)) == 1:  # equal shards: each round is a strided view of the block
            for i in range(k):
                lo, hi = i * rr, min(R, (i + 1) * rr)
                part = HashedBatch(routed.num.view(S, R, -1)[:, lo:hi].reshape(-1, routed.dn),
                                   routed.cat.view(S, R, -1)[:, lo:hi].reshape(-1, routed.dc),
                                   routed.y.view(S, R)[:, lo:hi].reshape(-1), None,
                                   routed.cat_span)
                part.shards = (hi - lo,) * S
                out.append(part)
            return out
        starts = np.concatenate([[0], np.cumsum(sh)[:-1]])
        for i in range(k):
            lo = i * rr
            cnt = [max(0, min(n, lo + rr) - lo) for n in sh]
            idx = np.concatenate([np.arange(a + lo, a + lo + c) for a, c in zip(starts, cnt)])
            part = routed.select(idx)
            part.shards = tuple(cnt)
            out.append(part)
        return out

    def _train_round(self, routed: HashedBatch) -> None:
        groups: dict[int, list] = {}
        # hashed-linear Synchronous pipelines without preprocessors that share a prep train
        # in ONE multi-pipeline launch (ops.linear.linear_scan3_round_multi; BASELINE config 5)
        fused = self._fused_groups(routed)
        done = set()
        for grp in fused:
            with tracing.range("round:multi"):
                ctx = grp[0].protocol._ctx(fused=True)
                for pipe in grp:
                    pipe._note_buffer(routed.B)
                type(grp[0].learner).fit_group([p.learner for p in grp], routed, ctx)
                for pipe in grp:
                    done.add(pipe.id)
                    buf = pipe.protocol.local_done()
                    if self.world > 1:
                        groups.setdefault(pipe.protocol.hubs, []).append((pipe, buf))
                if self.world == 1:  # the group's models averaged in one launch
                    Synchronous.finish_group([p.protocol for p in grp])
        rest = [pid for pid in sorted(self.pipes) if pid not in done]
        # several pipelines: each trains on its own stream (a linear pipeline's exact scan
        # occupies 16 CUs, so M of them run side by side), joined before the collectives
        streams = self._pipe_streams() if len(rest) > 1 else None
        main = torch.cuda.current_stream(self.device) if streams else None
        for i, pid in enumerate(rest):
            pipe = self.pipes[pid]
            st = streams[i % len(streams)] if streams else None
            if st is not None:
                st.wait_stream(main)
            with tracing.range(f"round:{pid}"), (torch.cuda.stream(st) if st is not None
                                                 else _nullcontext()):
                if self.world > 1 and isinstance(pipe.protocol, Synchronous):
                    groups.setdefault(pipe.protocol.hubs, []).append(
                        (pipe, pipe.train_local(routed)))
                else:
                    pipe.train(routed)
        if streams:
            for st in streams:
                main.wait_stream(st)
        for hubs, items in groups.items():
            with tracing.range("sync:coalesced"):
                if self._coll_timer is not None:
                    self._coll_timer.start()
                self.comm.all_reduce_coalesced_([b for _, b in items], tag="sync", hubs=hubs,
                                                bucket_bytes=self.cfg.bucketBytes)
                if self._coll_timer is not None:
                    self._coll_timer.stop(nbytes=sum(b.numel() * b.element_size()
                                                     for _, b in items))
            syn = [pipe.protocol for pipe, _ in items if isinstance(pipe.protocol, Synchronous)]
            Synchronous.finish_group(syn)
            for pipe, _ in items:
                if not isinstance(pipe.protocol, Synchronous):
                    pipe.protocol.finish()

    def _fused_groups(self, routed) -> list:
        """Pipelines whose rounds share one launch: ≥ 2 hashed-linear Synchronous pipelines
        without preprocessors, on a GPU, with equal ``group_key`` (same prep and rule)."""
        if self.device.type != "cuda" or len(self.pipes) < 2 or not routed.B or \
                str(self.cfg.fusePipelines).lower() in ("false", "0"):
            return []
        from omldm_amd.models.linear import LinearLearner

        by_key: dict = {}
        for pid in sorted(self.pipes):
            p = self.pipes[pid]
            if p.preprocessors or not isinstance(p.protocol, Synchronous) or \
                    not isinstance(p.learner, LinearLearner) or not p.protocol.fusable():
                continue
            k = p.learner.group_key(routed, p.protocol._ctx(fused=True))
            if k is not None:
                by_key.setdefault((k, p.protocol.hubs), []).append(p)
        return [g for g in by_key.values() if len(g) >= 2]

    def _pipe_streams(self):
        n = int(self.cfg.pipelineStreams)
        if self.device.type != "cuda" or n <= 1:
            return None
        if getattr(self, "_streams", None) is None:
            self._streams = [torch.cuda.Stream(self.device) for _ in range(n)]
        return self._streams[:n]

    # ------------------------------------------------------------------- queries
    def _answer(self, req: Request, response_id=None, write=True) -> dict:
        pipe = self.pipes[req.id]
        pipe.protocol.finalize()
        # every spoke scores its own test set (FlinkSpoke.scala:136-138,160-163)
        answers = []
        reg = pipe.learner.TASK == "regression"
        # every spoke's evaluation enqueued first, then ONE transfer of all (loss, score, n)
        # triples (a host sync per spoke cost 16 round trips per query)
        evals = [pipe.evaluate(test) for test in self.holdout.test_sets() if test.B]
        on_dev = [v for ev in evals for v in ev if torch.is_tensor(v) and v.device.type != "cpu"]
        got = iter(torch.stack([v.detach().double().reshape(()) for v in on_dev]).cpu().tolist()
                   if on_dev else [])
        for ev in evals:
            loss, score, n = (next(got) if torch.is_tensor(v) and v.device.type != "cpu"
                              else float(v) for v in ev)
            n = int(n)
            if n:
                sc = float(score) / n
                answers.append((float(loss) / n, float(np.sqrt(max(sc, 0.0))) if reg else sc, n))
        tot = pipe.learner.running_totals()
        m = ST.reduce_query_metrics(self.comm, answers, tot["fitted"], tot["loss_sum"],
                                    pipe.mean_buffer_size(), self.spokes)
        if self.rank == 0 and write:
            learner = {"name": pipe.learner.NAME,
                       "hyperParameters": pipe.learner.hyper_parameters(),
                       "parameters": pipe.learner.parameters_map(),
                       "dataStructure": pipe.learner.data_structure()}
            pre = [p.to_obj() for p in pipe.preprocessors]
            rid = req.requestId if response_id is None else response_id
            for qr in ST.build_query_responses(int(rid if rid is not None else -1), pipe.id, pre,
                                               learner, pipe.protocol_name, m,
                                               self.cfg.queryBucketSize):
                self.brokers["responses"].produce(self.cfg.responsesTopic, qr.to_json())
                self.counters["responses"] += 1
        return m

    # --------------------------------------------------------------------- tick
    def tick(self) -> None:
        if self.lanes is not None:
            with torch.cuda.stream(self.lanes.compute):
                self._tick()
        else:
            self._tick()

    def _tick(self) -> None:
        t0 = time.time()
        if self.faults:
            self.faults.on_tick(self.ticks)
        if self.watchdog is not None:
            self.watchdog.beat()
        with tracing.range("control"):
            n_ctrl, queries = self._control()
        if self.fserver is not None:
            self._forecast_fallback()
        with tracing.range("poll"):
            block = self._poll()
        if isinstance(block, TickBlock):
            n_local = block.n
        else:
            buf, offs = block
            n_local = len(offs) - 1
        if n_local:
            with tracing.range("parse"):
                if self._gpu_parser is not None:  # raw JSON → HBM → one thread per record
                    self._ready_ev = None
                    if isinstance(block, TickBlock):
                        batch, op_d, cnt = self._gpu_parser.parse_block(block, self.space)
                        if block.parsed is not None:
                            self._ready_ev = block.staged
                    else:
                        batch, op_d, cnt = self._gpu_parser.parse(buf, offs, self.space)
                    cnt = cnt if isinstance(cnt, np.ndarray) else cnt.cpu().numpy()
                    n_tr, n_fc, n_bad = (int(v) for v in cnt)
                    # the op array is only needed on the host to pick rows out
                    op = None if n_tr == n_local else op_d.cpu().numpy()
                elif isinstance(block, TickBlock):
                    batch, op, _ = parse_block(block.buf, block.offs, self.space,
                                               self.cfg.parseThreads)
                    batch.raw = block.raw()
                else:
                    batch, op, _ = parse_block(buf, offs, self.space, self.cfg.parseThreads)
                if op is not None:
                    n_tr, n_fc = int((op == OP_TRAINING).sum()), int((op == OP_FORECASTING).sum())
                    n_bad = n_local - n_tr - n_fc
            self.counters["records"] += n_tr + n_fc
            self.counters["invalid"] += n_bad
            if op is None:  # a pure, valid training block: train on it as it is
                tb = batch.without_raw()
            else:
                self._ready_ev = None  # the training rows are selected on the compute stream
                opt = torch.from_numpy(op)
                fidx = torch.nonzero(opt == OP_FORECASTING).flatten()
                tidx = torch.nonzero(opt == OP_TRAINING).flatten()
                if fidx.numel():
                    tf = time.perf_counter()
                    raw = RawRecords.from_view(batch.raw, fidx.numpy()) \
                        if batch.raw is not None else None
                    self._forecast(batch.without_raw().select(fidx).to(self.device), raw)
                    self._fc_lat.append((time.perf_counter() - tf) * 1e3)
                tb = batch.without_raw().select(tidx).to(self.device, non_blocking=True)
        else:
            tb = HashedBatch.empty(self.space, 0, device=self.device)
        spill = getattr(self, "_restored_train", None)
        if spill is not None and self.pipes:
            # holdout rows that no longer fit the merged ring after a re-scaled restore:
            # trained on directly (not routed through the holdout again)
            self._restored_train = None
            spill = spill.to(self.device)
        else:
            spill = None
        # global activity + termination flag (one tiny all-reduce per tick); every rank
        # then takes the same decisions, so the pipelines' collectives stay aligned
        self._flags[0] = float(n_local + n_ctrl)
        self._flags[1] = 0.0
        if self.rank == 0 and self.cfg.test and self.idle.expired(t0) and self.pipes:
            self._flags[1] = 1.0
        self._flags[2] = float(tb.B + (spill.B if spill is not None else 0))
        self._flags[3] = 0.0
        if self.world > 1 and self.rank == 0:
            self._ctrl_pending += self._poll_requests()
            self._flags[3] = float(len(self._ctrl_pending))
        # rank 0's clock decides checkpoints: every rank snapshots at the same tick
        self._flags[4] = 1.0 if (self.rank == 0 and self.checkpointer is not None
                                 and self.checkpointer.due()) else 0.0
        with tracing.range("flags"):
            self.comm.all_reduce_host_(self._flags, tag="heartbeat")
            active, term, n_train, n_req, ckpt = (float(v) for v in self._flags.tolist())
        self._ctrl_due = n_req > 0
        active += n_req
        self._trained_global += int(n_train)
        fs = self.fserver if (self.pipes and (n_train > 0 or queries)) else None
        if fs is not None:  # the lane's predicts see models between two rounds
            fs.begin_training()
        try:
            if self.pipes and n_train > 0:
                if self._train_timer is not None:
                    self._train_timer.start()
                self._train(tb, spill)
                if self._train_timer is not None:
                    self._train_timer.stop()
                if self._health is not None:
                    self._health.arm(self.pipes)
                if self._trace_dir:
                    self._trace_models()
            for q in queries:
                self._answer(q)
            if queries and self.device.type == "cuda":
                self._holdout_read_ev = torch.cuda.Event()
                self._holdout_read_ev.record()
        finally:
            if fs is not None:
                fs.end_training()
        with tracing.range("learning_curve"):
            for pipe in self.pipes.values():
                pipe.record_learning_curve()
        if isinstance(block, TickBlock) and block.n and self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            block.consumed = ev  # the ingest thread reuses this slot's HBM after this
        if active > 0:
            self.idle.activity(time.time())  # idle = time since the last active tick ended
        if term > 0:
            self._terminate()
        with tracing.range("catch_up"):
            behind = self.fserver is not None and not self.fserver.catch_up()
        if behind:
            print(f"[omldm] rank {self.rank}: forecast lane behind after 5 s", flush=True)
        if self.checkpointer is not None and ckpt > 0:
            if self._health is not None:
                # this tick's device words first (blocking; the snapshot's host copy syncs
                # anyway): a discarded round or a dropped update raises here, before a
                # model it touched can be snapshotted and restored by a restart
                self._health.check(block=True)
            self.egress.flush()  # outputs of the checkpointed ticks are in their topic
            self.checkpointer.save(self)
        self.ticks += 1
        if active == 0 and not self.terminated:
            time.sleep(0.001)

    def _terminate(self):
        """Final −1 query of every pipeline + JobStatistics (reference §3.7), graceful."""
        stats = []
        for pid in sorted(self.pipes):
            pipe = self.pipes[pid]
            m = self._answer(Request(id=pid, request="Query", requestId=-1), write=False)
            stats.append(ST.pipeline_statistics(pipe, m))
        self.egress.flush()
        js = ST.job_statistics(self.cfg.jobName, self.spokes * self.world,
                               self.idle.duration_ms(), stats)
        js.metrics = self._metrics(js.duration)
        self.final_stats = js
        if self.rank == 0:
            self.brokers["performance"].produce(self.cfg.performanceTopic, js.to_json())
        self.terminated = True

    def _metrics(self, duration_ms: int) -> dict:
        """Engine metrics attached to JobStatistics: node-wide training
        throughput, forecast latency percentiles (rank 0), collective traffic, stages."""
        lat = sorted(self._fc_lat)
        pct = (lambda q: round(lat[min(len(lat) - 1, int(q * len(lat)))], 3)) if lat else \
            (lambda q: None)
        cs = self.comm.stats
        fsl = self.fserver.latency_percentiles() if self.fserver is not None else None
        dev = {}
        if self._train_timer is not None:
            wall_ms = max(1e-3, (time.time() - self._t_start) * 1e3)
            for t in (self._train_timer, self._coll_timer, self.ingest.h2d_timer,
                      self.ingest.parse_timer):
                if t is not None:
                    t.settle()
            tr, co = self._train_timer, self._coll_timer
            h2d, pa = self.ingest.h2d_timer, self.ingest.parse_timer
            dev = {"trainDeviceMs": round(tr.ms, 3),
                   "collectiveDeviceMs": round(co.ms, 3), "collectiveGBps": co.gbps(),
                   "h2dMs": round(h2d.ms, 3) if h2d else None,
                   "h2dGBps": h2d.gbps() if h2d else None,
                   "parseMs": round(pa.ms, 3) if pa else None,
                   "parseGBps": pa.gbps() if pa else None,
                   # share of the job's wall time the training rounds kept the GPU busy
                   # (MFMA / VALU utilisation per kernel: rocprofv3 PMC, profiles/)
                   "trainBusyFraction": round(tr.ms / wall_ms, 4)}
        return {"ranks": self.world, "spokesPerRank": self.spokes,
                "forecastRecordLatencyUs": fsl,
                "forecastRecordLatencyUsPerLearner":
                    self.fserver.family_percentiles() if self.fserver is not None else None,
                "trainedExamples": self._trained_global,
                "examplesPerSec": round(self._trained_global / max(duration_ms, 1) * 1e3, 1),
                "forecastBatchLatencyMs": {"p50": pct(0.5), "p99": pct(0.99)},
                "collectives": cs.collectives, "collectiveBytes": cs.bytes,
                "collectiveBytesPerTag": dict(cs.per_tag), "counters": dict(self.counters),
                "stages": tracing.report(), "modelStoreMB": round(self.store.bytes() / 2**20, 2),
                "device": dev}

    def run(self) -> "Job":
        while not self.terminated and (self.cfg.maxTicks <= 0 or self.ticks < self.cfg.maxTicks):
            self.tick()
        for p in self.pipes.values():
            p.protocol.finalize()
        if self._health is not None:
            self._health.check()  # the last trained tick's words
        if self._trace_dir:
            self._trace_models(final=True)
        self.close()
        return self

    def close(self) -> None:
        """Stop what the job runs beside its ticks — the forecast lane (thread and resident
        wave), the ingest read-ahead, the egress writer, the checkpointer, the watchdog — and
        wait for the device. Idempotent; ``run`` ends with it, and a caller that drives
        ``tick`` itself (tests, embedding) calls it when done."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        if self.fserver is not None:
            self.fserver.close()
        self.ingest.close()
        self.egress.close()
        if self.checkpointer is not None:
            self.checkpointer.close()
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # --------------------------------------------------------------- checkpoint
    def state_dict(self) -> dict:
        fc_lane, fc_pending = (None, [])
        if self.fserver is not None:
            fc_lane, fc_pending = self.fserver.snapshot()
        sd = {"pipelines": {pid: p.state_dict() for pid, p in self.pipes.items()},
              "holdout": self.holdout.state_dict(),
              "consumers": {k: {"offsets": v}
                            for k, v in self.consumer_offsets(fc_lane).items()},
              "record_buffer": [r for b in self.record_buffer for r in RawView(*b)],
              # forecasting records the lane handed back, not yet predicted by a tick
              "forecast_pending": [bytes(r) for r in fc_pending],
              "ticks": self.ticks,
              "counters": dict(self.counters), "world": self.world,
              "spoke_parallelism": self.spoke_parallelism,
              "request_buffer": [list(m) for m in self.request_buffer]}
        if self.rank == 0:
            sd["pipeline_map"] = self.pmap.state_dict()
            sd["requests"] = self.req_in.state_dict()
            sd["control_pending"] = list(self._ctrl_pending)  # polled, not yet applied
        return sd

    def load_state_dict(self, sd: dict, same_world: bool = True,
                        consumer_offsets: dict | None = None, owned: list | None = None) -> None:
        """``owned`` (re-scaled restore only): the state dicts of the old ranks whose
        per-rank data this rank takes over (utils/checkpoint.py:rescale_owners); models
        and protocol state come from ``sd``."""
        for pid, psd in sd.get("pipelines", {}).items():
            req = Request.from_json(psd["request"])
            pipe = Pipeline(req, self.space, self.comm, self.device, self.spokes,
                            self.cfg.parallelism, self.cfg.maxMsgParams, store=self.store)
            pipe.load_state_dict(psd)
            self.pipes[int(pid)] = pipe
        if same_world:  # partition ownership only matches at the same world size
            spill = self.holdout.load_state_dict(sd["holdout"])  # spoke count may differ
            if spill is not None and spill.B:
                self._restored_train = spill
            self.train_in.load_state_dict(sd["consumers"]["train"])
            self.fcst_in.load_state_dict(sd["consumers"]["forecast"])
            recs = list(sd.get("record_buffer", []))
            self.counters.update(sd.get("counters", {}))
        else:
            if consumer_offsets is not None:  # Consumer keeps only the partitions it owns
                self.train_in.load_state_dict({"offsets": consumer_offsets["train"]})
                self.fcst_in.load_state_dict({"offsets": consumer_offsets["forecast"]})
            owned = list(owned or [])
            # holdout rings merged oldest-first; rows beyond the ring are trained on
            spill = self.holdout.load_merged([o["holdout"] for o in owned])
            if spill is not None and spill.B:
                self._restored_train = spill
            recs = [r for o in owned for r in o.get("record_buffer", [])]
            # running totals are per rank and summed by queries: sum the owned ranks'
            for pid, pipe in self.pipes.items():
                cums = [o["pipelines"][pid]["learner"]["cum"] for o in owned
                        if pid in o.get("pipelines", {})]
                tot = torch.stack([c.to(torch.float64) for c in cums]).sum(0) if cums else \
                    torch.zeros_like(pipe.learner.cum, device="cpu")
                pipe.learner.cum.copy_(tot.to(pipe.learner.cum.device))
            for o in owned:
                for k, v in o.get("counters", {}).items():
                    self.counters[k] = self.counters.get(k, 0) + v
        pending = list(sd.get("forecast_pending", [])) if same_world else \
            [r for o in (owned or []) for r in o.get("forecast_pending", [])]
        if pending and self.fserver is not None:
            self.fserver.fallback.extend(pending)
        elif pending:  # no lane here: the batched path predicts them with the next tick
            recs = recs + pending
        self.record_buffer = [join_block(recs)] if recs else []
        self._buffered = len(recs)
        self.ticks = int(sd.get("ticks", 0))
        # the gate's state is the same on every rank (every rank applies every Create);
        # a restore onto more spokes raises the recorded parallelism (checkParallelism)
        self.spoke_parallelism = max(self.parallelism, int(sd.get("spoke_parallelism", 0)))
        self.request_buffer = [tuple(m) for m in sd.get("request_buffer", [])]
        if self.rank == 0 and "pipeline_map" in sd:
            self.pmap.load_state_dict(sd["pipeline_map"])
            self.req_in.load_state_dict(sd.get("requests", {}))
            pending = [tuple(m) for m in sd.get("control_pending", [])]
            if self.world == 1:  # single rank: applied at the next tick's _control
                self._restored_ctrl = pending
            else:
                self._ctrl_pending = pending
