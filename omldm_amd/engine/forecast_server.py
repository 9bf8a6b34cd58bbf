"""Per-record forecasting: every forecasting record is answered as it arrives.

Reference: a forecasting point reaching a spoke is predicted at once by every pipeline
(``FlinkSpoke.processElement1`` → ``node.receiveTuple`` → ``predict``,
omldm/operators/spoke/FlinkSpoke.scala:101-105) and the Prediction is emitted right away
(omldm/network/FlinkNetwork.scala:243-257) — no batching, so the record-in →
Prediction-out latency is one predict.

Here the engine's tick batches training rows (throughput); forecasting records take a
separate low-latency lane: a host thread consumes the forecasting topic, parses each
record natively (csrc/host/ingest.cpp, the same hashing as the GPU parser) and answers
it for EVERY pipeline before taking the next one:

* hashed-linear pipelines of the HBM model store (no preprocessor) are scored together
  by the PERSISTENT serving wavefront (csrc/kernels/serving.hip: one resident wave
  polling a coherent pinned mailbox; no kernel launch, no stream synchronisation per
  request);
* every other pipeline — preprocessors in front (StandardScaler, MinMaxScaler,
  PolynomialFeatures), ORR, MultiClassPA, K-means, NN, Hoeffding tree — runs its own
  predict kernels on a one-row batch on the lane's HIP stream (one stream sync per
  record).

Consistency (the reference serialises a spoke's predict and fit in one operator,
FlinkSpoke.scala:97-105, so a prediction sees a model between two fits):

* the wave reads one of two published weight banks, never the live store rows: after a
  tick's training the engine copies the served rows into the bank no request reads
  (``publish``, on the compute stream, stream-ordered after the round's apply) and the
  lane switches its requests to that bank once the copy's event has completed — an
  answer never mixes slots of two rounds, and is at most one round stale;
* a one-row predict of a direct pipeline waits for the tick's training to finish
  (``begin_training`` / ``end_training``: the lane's stream waits on the event recorded
  after the last round), and the tick's next training starts only after the lane's
  in-flight predict has returned (the lane holds ``lock`` for a whole record) — so it reads
  the model between two rounds, never one half-way through an update.

Records wait for the tick (``take_fallback``) only while no pipeline exists yet.

Native lane (file topics, every pipeline on the wave — the engine's default linear
pipelines): the whole lane runs in a C++ thread (csrc/host/fcst_lane.cpp: pread of the
forecasting partitions → native parse → mailbox → native Prediction formatting → one
append per record), so no Python — and no GIL shared with the tick thread — sits on the
record's path. The Python thread then only supervises: it starts the resident wave when
the lane asks for one. The bank a request reads is a pinned word the GPU sets after each
publish copy (stream-ordered), the same at-most-one-round-stale guarantee. Kafka and
in-process topics, and pipelines needing one-row predicts, keep the Python lane.
"""
from __future__ import annotations

import atexit
import collections
import os
import threading
import time
import weakref

import numpy as np
import torch

from omldm_amd.io.egress import RawRecords, format_predictions
from omldm_amd.ops import native

OP_FORECASTING = 1

_LIVE: "weakref.WeakSet[ForecastServer]" = weakref.WeakSet()


@atexit.register
def _stop_all() -> None:
    """No resident wave outlives its process (a Job that was never run to the end)."""
    for fs in list(_LIVE):
        try:
            fs.close()
        except Exception:  # noqa: BLE001 — best effort at interpreter exit
            pass


class ForecastServer:
    IDLE_SLEEP_S = 20e-6
    # idle polling backs off in tiers so a quiet forecasting topic costs the training tick
    # nothing: busy-poll (sleep(0) yields the GIL) for 2 ms after a record, then 50 µs
    # sleeps, then 1 ms sleeps once the topic has been quiet for 50 ms
    SPIN_S = 2e-3
    WARM_S = 50e-3

    def __init__(self, job, lifetime_us: int = 2_000_000):
        self.job = job
        self.space = job.space
        self.consumer = job.fcst_in
        self.topic = job.cfg.predictionsTopic
        self.broker = job.brokers["predictions"]
        self.lifetime_us = int(lifetime_us)
        self.lock = threading.Lock()
        self._server = None
        self._spec = None             # (first store row, end row, bias) the wave serves
        self._served: list = []       # (pipeline id, store row, classification?) in W order
        self._direct: list = []       # (pipeline id, Pipeline): one-row predicts on the lane
        self._order: list = []        # every served pipeline id, in id order
        self._row0 = 0
        self._stream = None           # the lane's HIP stream (direct predicts)
        # published model banks of the store rows the wave serves (see the module doc)
        self._banks = None            # [bank0, bank1]: copies of store.W
        self._bank = 0                # the bank requests read
        self._pend = None             # (bank, event): a publish the lane adopts when done
        self._pub_lock = threading.Lock()
        # direct predicts: training in flight → wait for its end event
        self._trained = threading.Event()
        self._trained.set()
        self._train_ev = None
        self.family_latency: dict = {}  # learner name → deque of µs (record in → outputs out)
        self.fallback: collections.deque = collections.deque()
        self.latency_us: collections.deque = collections.deque(maxlen=1 << 16)
        self.served = 0
        self.invalid = 0
        dn, dc = self.space.dn, self.space.dc
        # one record's parse buffers (omldm_serve_request copies them into the mailbox)
        self._num = torch.zeros((1, dn), dtype=torch.float32)
        self._cat = torch.full((1, dc), -1, dtype=self.space.cat_dtype)
        # the mailbox carries int32 per field: the wide slot, or the compact uint16 value
        self._cat32 = np.full(max(dc, 1), -1, dtype=np.int32)
        self._y = torch.zeros(1, dtype=torch.float32)
        self._op = np.zeros(1, dtype=np.int8)
        self._offs = np.zeros(2, dtype=np.int64)
        self._done: dict = {}          # consumer offsets up to which every record is answered
        # held by the lane for one poll → answer / hand back → ``_done`` cycle, so a
        # checkpoint sees ``_done`` and ``fallback`` of the same instant (``snapshot``)
        self._cycle = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="omldm-forecast", daemon=True)
        self._native = None           # csrc/host/fcst_lane.cpp handle (file topics)
        self._native_parts: list = []
        self._native_fds: list = []
        self._bank_word = None        # pinned word: the bank the native lane reads
        self._nat_target = 0          # the bank of the native lane's last publish
        self._native_lat = None       # its per-record latencies (µs, sorted), last read
        self._last_native = None      # its last counters
        _LIVE.add(self)

    # ----------------------------------------------------------------- control
    def start(self) -> None:
        self._thread.start()

    def close(self) -> None:
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(5.0)
        with self.lock:
            self._stop_native()
            self._stop_wave()
            if self._bank_word is not None:
                from omldm_amd.ops.serving import _lib

                _lib().omldm_bank_word_free(self._bank_word)
                self._bank_word = None

    def _stop_wave(self) -> None:
        if self._server is not None:
            self._server.close()
            self._server = None

    def suspend(self) -> None:
        """Before the model store may move (a Create can grow its arena) or pipelines
        change: the lane stops serving until ``reconfigure``."""
        with self.lock:
            self._stop_native()
            self._stop_wave()
            self._spec = None
            self._served = []
            self._direct = []
            self._order = []

    def reconfigure(self) -> None:
        """After a Create / Delete / restore (main thread): the model-store pipelines of
        the most common bias go to the wave, every other pipeline to one-row predicts on
        the lane's stream. The wave itself starts with the first record: a resident wave
        holds one of the process's hardware queues (4 on this pool), which costs the
        training tick's copy / parse / compute overlap while no forecast arrives (engine
        end-to-end 33 → 15 M records/s with an idle resident wave)."""
        with self.lock:
            self._stop_native()
            self._stop_wave()
            self._spec = None
            self._served, self._direct, self._order = [], [], []
            pipes = [self.job.pipes[pid] for pid in sorted(self.job.pipes)]
            self._order = [p.id for p in pipes]
            store = [p for p in pipes if p.store is not None]
            if os.environ.get("OMLDM_FS_NOWAVE") or self.job.device.type != "cuda":
                store = []  # diagnostics / CPU jobs: the lane without the wave
            if store:
                by_bias: dict = {}
                for p in store:
                    by_bias.setdefault(bool(p.learner.rule.bias), []).append(p)
                bias, store = max(by_bias.items(), key=lambda kv: len(kv[1]))
                rows = [p.store_row for p in store]
                lo, hi = min(rows), max(rows) + 1
                self._spec = (lo, hi, bias)
                self._row0 = lo
                self._served = [(p.id, p.store_row, p.learner.TASK == "classification")
                                for p in store]
                # both banks start as the current models (the store may have moved)
                W = self.job.store.W
                with self._pub_lock:
                    if self._banks is None or self._banks[0].shape != W.shape:
                        self._banks = [torch.empty_like(W), torch.empty_like(W)]
                    for b in self._banks:
                        b.copy_(W)
                    torch.cuda.synchronize(self.job.device)
                    self._bank, self._pend = 0, None
            waved = {pid for pid, _, _ in self._served}
            self._direct = [(p.id, p) for p in pipes if p.id not in waved]
            if self._direct and self._stream is None and self.job.device.type == "cuda":
                self._stream = torch.cuda.Stream(self.job.device)
            if self._native_eligible():
                self._start_native()

    # ------------------------------------------------------------ native lane
    def _native_eligible(self) -> bool:
        from omldm_amd.io.transport import FileBroker

        return (os.environ.get("OMLDM_FS_NATIVE", "1") != "0"
                and self.job.device.type == "cuda" and self._spec is not None
                and not self._direct and bool(self._served) and bool(self.consumer.parts)
                and isinstance(self.consumer.broker, FileBroker)
                and isinstance(self.broker, FileBroker))

    @property
    def native(self) -> bool:
        """The lane runs in the native thread (csrc/host/fcst_lane.cpp)."""
        return self._native is not None

    def _start_native(self) -> None:
        """Under the lock, after reconfigure: the native lane from the consumer's offsets."""
        import ctypes

        from omldm_amd.ops.serving import _lib

        hl, sl = native.host(), _lib()
        if self._bank_word is None:
            self._bank_word = sl.omldm_bank_word_alloc()
        ctypes.c_uint32.from_address(self._bank_word).value = 0  # both banks = W (above)
        self._nat_target = 0
        cb, topic = self.consumer.broker, self.consumer.topic
        parts = list(self.consumer.parts)
        fds = []
        for p in parts:
            path = os.path.join(cb.root, topic, f"{p}.jsonl")
            if not os.path.exists(path):
                open(path, "ab").close()
            fds.append(os.open(path, os.O_RDONLY))
        n_out = self.broker.partitions(self.topic)
        outs = []
        for p in range(n_out):
            path = os.path.join(self.broker._dir(self.topic), f"{p}.jsonl")
            outs.append(os.open(path, os.O_WRONLY | os.O_APPEND | os.O_CREAT, 0o644))
        in_fds = np.array(fds, dtype=np.int32)
        out_fds = np.array(outs, dtype=np.int32)
        offs = np.array([self.consumer.offsets[p] for p in parts], dtype=np.int64)
        lo = self._spec[0]
        pids = np.array([pid for pid, _, _ in self._served], dtype=np.int32)
        rows = np.array([row - lo for _, row, _ in self._served], dtype=np.int32)
        cls = np.array([1 if c else 0 for _, _, c in self._served], dtype=np.int32)
        sp = self.space
        serve = ctypes.cast(sl.cdll.omldm_serve_request, ctypes.c_void_p).value
        alive = ctypes.cast(sl.cdll.omldm_serve_alive, ctypes.c_void_p).value
        h = hl.omldm_fcst_lane_start(
            in_fds.ctypes.data, offs.ctypes.data, len(parts), out_fds.ctypes.data, len(outs),
            sp.n_numerical, sp.n_discrete, sp.dc, sp.dim, sp.cat_span, serve, alive,
            self._spec[1] - lo, pids.ctypes.data, rows.ctypes.data, cls.ctypes.data, len(pids),
            self._bank_word)
        if not h:
            for fd in fds + outs:
                os.close(fd)
            return
        self._native, self._native_parts, self._native_fds = h, parts, fds + outs
        if self._server is not None:
            hl.omldm_fcst_lane_set_mailbox(h, self._server.mb)

    def _native_offsets(self) -> dict:
        offs = np.zeros(max(1, len(self._native_parts)), dtype=np.int64)
        native.host().omldm_fcst_lane_offsets(self._native, offs.ctypes.data)
        return {p: int(offs[i]) for i, p in enumerate(self._native_parts)}

    def _stop_native(self) -> None:
        """Under the lock: the native lane stops; the consumer resumes at its offsets."""
        h = self._native
        if h is None:
            return
        self.native_stats()  # (the last counters, kept for the caller)
        self.latency_percentiles()  # (and the lane's latencies)
        offs = self._native_offsets()
        native.host().omldm_fcst_lane_stop(h)
        self._native = None
        self.consumer.offsets.update(offs)
        self._done = dict(self.consumer.offsets)
        for fd in self._native_fds:
            try:
                os.close(fd)
            except OSError:
                pass
        self._native_fds = []

    def native_stats(self) -> dict | None:
        """Answered records and the mean µs per stage of the native lane (poll, parse, wave,
        format, produce, record) — None when it is not running."""
        if self._native is None:
            return self._last_native
        st = np.zeros(9, dtype=np.int64)
        native.host().omldm_fcst_lane_stats(self._native, st.ctypes.data)
        n = max(1, int(st[0]))
        names = ("poll", "parse", "wave", "format", "produce", "record")
        out = {"served": int(st[0]), "invalid": int(st[1]), "write_errors": int(st[2]),
               "stage_us": {k: round(float(st[3 + i]) / n / 1e3, 3) for i, k in enumerate(names)}}
        self._last_native = out
        return out

    def native_wait(self, count: int, timeout_s: float = 1.0) -> bool:
        """Blocks (GIL released) until the native lane has answered ``count`` records."""
        h = self._native
        return h is not None and native.host().omldm_fcst_lane_wait(
            h, int(count), int(timeout_s * 1e6)) == 0

    def native_tout(self, k: int) -> float:
        """perf_counter-clock time at which the native lane answered record k."""
        return native.host().omldm_fcst_lane_tout(self._native, int(k)) / 1e9

    @property
    def serving(self) -> bool:
        """Records are answered on the lane (else they wait in the fallback queue)."""
        return bool(self._order)

    def _ensure_wave(self):
        """Under the lock: a live wave over the configured store rows (started on the
        first record, restarted after its lifetime)."""
        from omldm_amd.ops.serving import PredictServer

        srv = self._server
        if srv is not None and srv.lib.omldm_serve_alive(srv.mb):
            return srv
        self._stop_wave()
        lo, hi, bias = self._spec
        b0, b1 = self._banks
        srv = PredictServer(b0[lo:hi], self.space.dn, self.space.dc, bias,
                            cat_span=self.space.cat_span, w1=b1[lo:hi])
        srv.start(lifetime_us=self.lifetime_us)
        self._server = srv
        return srv

    def snapshot(self) -> tuple[dict, list]:
        """Checkpoint view of the lane, taken between two of its cycles: the consumer
        offsets up to which every forecasting record is answered or handed back, and the
        handed-back records still waiting for the tick (saved with the job's state like
        the record buffer, so a restore neither skips nor repeats a forecast)."""
        with self._cycle:
            if self._native is not None:
                return self._native_offsets(), list(self.fallback)
            done = dict(self._done) if self._thread.is_alive() else dict(self.consumer.offsets)
            return done, list(self.fallback)

    # ------------------------------------------------------ model publication
    def begin_training(self) -> None:
        """Tick thread, before the round's kernels are enqueued: waits for the lane's
        in-flight record (its direct predicts read the models the round updates), then
        holds later direct predicts until ``end_training``."""
        with self.lock:
            self._trained.clear()

    def end_training(self) -> None:
        """Tick thread, after the round (and the queries that may finalize models): the
        event after the last kernel gates the lane's next direct predicts, and the served
        store rows are published into the bank no request reads."""
        try:
            if self.job.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
                self._train_ev = ev
                self.publish()
        finally:
            self._trained.set()

    def publish(self) -> None:
        """Copy the served store rows into the bank requests do not read (current stream,
        after the round's apply) and hand it to the lane with the copy's event."""
        with self._pub_lock:
            spec, banks = self._spec, self._banks
            if spec is None or banks is None:
                return
            lo, hi, _ = spec
            if self._native is not None and self._bank_word is not None:
                # the native lane reads the bank named by a pinned word the GPU sets after
                # the copy (stream order): alternate banks, the word flips when it is done
                import ctypes

                from omldm_amd.ops.serving import _lib

                # the last publish's word not written yet: the lane still reads the other
                # bank, so this copy goes to the pending bank again (never the read one)
                cur = ctypes.c_uint32.from_address(self._bank_word).value & 1
                prev = self._nat_target
                target = self._nat_target = prev if cur != prev else 1 - prev
                banks[target][lo:hi].copy_(self.job.store.W[lo:hi], non_blocking=True)
                check_rc = _lib().omldm_bank_word_set(
                    self._bank_word, target, torch.cuda.current_stream().cuda_stream)
                if check_rc != 0:
                    raise RuntimeError(f"hipStreamWriteValue32 failed ({check_rc})")
                return
            target = self._pend[0] if self._pend is not None else 1 - self._bank
            banks[target][lo:hi].copy_(self.job.store.W[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pend = (target, ev)

    def _read_bank(self) -> int:
        """The bank this request reads: the latest publish whose copy has completed."""
        with self._pub_lock:
            if self._pend is not None and self._pend[1].query():
                self._bank, self._pend = self._pend[0], None
            return self._bank

    def take_fallback(self) -> list:
        out = []
        while self.fallback:
            out.append(self.fallback.popleft())
        return out

    def latency_percentiles(self) -> dict:
        if self._native is not None:  # the native lane's own per-record times
            buf = np.zeros(1 << 16, dtype=np.int64)
            n = int(native.host().omldm_fcst_lane_latencies(self._native, buf.ctypes.data,
                                                              buf.size))
            self._native_lat = sorted((buf[:n] / 1e3).tolist())
        lat = self._native_lat if (self._native_lat and not self.latency_us) else \
            sorted(self.latency_us)
        if not lat:
            return {"p50": None, "p99": None, "n": 0}
        return {"p50": round(lat[len(lat) // 2], 2),
                "p99": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 2), "n": len(lat)}

    # --------------------------------------------------------------- data path
    def _parse(self, rec: bytes) -> bool:
        sp = self.space
        self._offs[1] = len(rec)
        self._cat.fill_(-1)
        self._num.zero_()
        native.host().omldm_parse_instances(
            rec, self._offs.ctypes.data, 1, sp.n_numerical, sp.n_discrete, sp.dc, sp.dim,
            sp.cat_span, self._num.data_ptr(), self._cat.data_ptr(), self._y.data_ptr(),
            self._op.ctypes.data, 1)
        if sp.cat_span > 0:
            self._cat32[: sp.dc] = self._cat.numpy()[0].view(np.uint16)
        else:
            self._cat32[: sp.dc] = self._cat.numpy()[0]
        return int(self._op[0]) == OP_FORECASTING

    def _predict_direct(self, pipes: list) -> list:
        """One-row predicts of the pipelines the wave does not score, on the lane's stream:
        the record moves to the device once, every pipeline's predict is enqueued, and one
        copy brings all the answers back (one stream synchronisation per record, not one per
        pipeline)."""
        from omldm_amd.api.batch import HashedBatch

        dev = self.job.device
        b = HashedBatch(self._num, self._cat, self._y, None, self.space.cat_span)
        if not self._trained.wait(60.0):
            raise RuntimeError("forecast lane: the tick's training did not end within 60 s")
        if self._stream is None:
            bd = b.to(dev)
            return [float(pipe.predict(bd)[0]) for pipe in pipes]
        with torch.cuda.stream(self._stream):
            if self._train_ev is not None:
                self._stream.wait_event(self._train_ev)  # the model between two rounds
            bd = b.to(dev, non_blocking=False)
            outs = [pipe.predict(bd).float().reshape(-1)[:1] for pipe in pipes]
            return torch.cat(outs).cpu().tolist()

    def serve_one(self, rec: bytes, t_in: float | None = None) -> bool:
        """Answers one forecasting record for every pipeline (wave + one-row predicts).
        False: no pipeline yet — the caller keeps it for the tick."""
        t_in = time.perf_counter() if t_in is None else t_in
        with self.lock:
            if not self._order:
                return False
            if not self._parse(rec):
                self.invalid += 1
                return True
            preds: dict = {}
            t_w = None
            if self._spec is not None:
                cat = self._cat32.ctypes.data
                srv = self._ensure_wave()
                bank = self._read_bank()
                try:
                    out = srv.request_raw(self._num.data_ptr(), cat, bank=bank)
                except TimeoutError:  # the wave's lifetime ended under the request
                    self._stop_wave()
                    out = self._ensure_wave().request_raw(self._num.data_ptr(), cat, bank=bank)
                for pid, row, cls in self._served:
                    s = float(out[row - self._row0])
                    preds[pid] = (1.0 if s >= 0 else -1.0) if cls else s
                t_w = time.perf_counter()
            fam_t: list = []
            if self._direct:
                t0 = time.perf_counter()
                vals = self._predict_direct([pipe for _, pipe in self._direct])
                dt = (time.perf_counter() - t0) / len(self._direct)
                for (pid, pipe), v in zip(self._direct, vals):
                    preds[pid] = v
                    fam_t.append((pipe.learner.NAME, dt))
            raw = RawRecords(np.frombuffer(rec, dtype=np.uint8),
                             np.zeros(1, dtype=np.int64), np.array([len(rec)], dtype=np.int64))
            for pid in self._order:
                block, offs = format_predictions(raw, pid, [preds[pid]])
                self.broker.produce(self.topic, block[:int(offs[1]) - 1])
            self.served += 1
        t_out = time.perf_counter()
        self.latency_us.append((t_out - t_in) * 1e6)
        # per learner family: the record's parse + wave (store learners) or parse + its
        # own one-row predict (the others), as if it were the only pipeline
        base = (t_w - t_in) if t_w is not None else 0.0
        if t_w is not None:
            for pid, _, _ in self._served:
                self._fam("linear-store", base)
        for name, dt in fam_t:
            self._fam(name, (base if t_w is None else 0.0) + dt)
        return True

    def _fam(self, name: str, seconds: float) -> None:
        q = self.family_latency.get(name)
        if q is None:
            q = self.family_latency[name] = collections.deque(maxlen=1 << 14)
        q.append(seconds * 1e6)

    def family_percentiles(self) -> dict:
        out = {}
        for name, q in list(self.family_latency.items()):
            lat = sorted(q)
            if lat:
                out[name] = {"p50": round(lat[len(lat) // 2], 2),
                             "p99": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 2),
                             "n": len(lat)}
        return out

    def catch_up(self, timeout_s: float = 5.0) -> bool:
        """Waits until every forecasting record in the topic when called is answered (or
        handed to the tick). The engine calls it at the end of a tick, so a tick's outputs
        are complete when it returns; records keep being answered one by one as they
        arrive in between."""
        if not self._thread.is_alive():
            return True
        target = {p: self.consumer.broker.end_offset(self.consumer.topic, p)
                  for p in self.consumer.parts}
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            done = self._native_offsets() if self._native is not None else self._done
            if all(done.get(p, 0) >= o for p, o in target.items()):
                return True
            time.sleep(self.IDLE_SLEEP_S)
        return False

    def _pending(self) -> bool:
        br, topic, offs = self.consumer.broker, self.consumer.topic, self.consumer.offsets
        return any(br.end_offset(topic, p) > o for p, o in offs.items())

    def _run(self) -> None:
        if self.job.device.type == "cuda":
            torch.cuda.set_device(self.job.device)
        last = 0.0
        idle_marked = False
        while not self._stop.is_set():
            if self._native is not None:  # supervise the native lane: start its wave
                h = self._native
                if native.host().omldm_fcst_lane_need_wave(h):
                    with self.lock:
                        if self._native is h:
                            srv = self._ensure_wave()
                            native.host().omldm_fcst_lane_set_mailbox(h, srv.mb)
                    continue
                time.sleep(200e-6)
                continue
            quiet = time.perf_counter() - last
            with self._cycle:
                # right after traffic the topic is polled directly; a quiet topic is looked
                # at through its end offsets first (cheap) and not polled
                recs = self.consumer.poll(64) if (quiet < self.SPIN_S or self._pending()) else []
                if recs:
                    idle_marked = False
                    last = time.perf_counter()
                    t_in = last
                    for i, rec in enumerate(recs):
                        if not self.serve_one(rec, t_in if i == 0 else None):
                            self.fallback.append(rec)
                    self._done = dict(self.consumer.offsets)
                    continue
                if not idle_marked:  # everything polled so far is answered
                    self._done = dict(self.consumer.offsets)
                    idle_marked = True
            time.sleep(0 if quiet < self.SPIN_S else (50e-6 if quiet < self.WARM_S else 1e-3))
