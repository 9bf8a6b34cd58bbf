"""Tick ingest: this rank's training ∪ forecasting records, read one tick ahead.

Reference: one Flink Kafka source subtask per partition deserialises records one at a
time and forwards them to the spokes (omldm/Job.scala:42-57,
omldm/job/FlinkLearning.scala:70,83). Here a tick's records are ONE byte block:

    topic log ──pread (no GIL, csrc/host/logio.cpp)──► pinned staging slot
              ──H2D──► HBM ──GPU JSON parser (csrc/kernels/json_ingest.hip)──► batch

Two background stages run behind the tick: a reader thread fills slot k+2 from the logs
while a staging thread moves slot k+1 to HBM and parses it on the GPU (its own copy
stream), while the tick trains on slot k. Slots are reused round-robin; a slot's host
bytes are rewritten only after its H2D copy event, its HBM buffers only after the
``consumed`` event the tick records behind its last use.

Latency: a prefetched block that came back empty is re-polled synchronously at the start
of the tick, so an idle stream's new records are picked up by the next tick, as with
synchronous polling (records that arrive while a read is in flight may land one tick
later; CPU jobs poll synchronously by default, which keeps tests tick-exact). Offsets for checkpoints are the consumers' offsets
*after* the block the job has actually processed (``TickBlock.offsets``), never the
prefetcher's read-ahead position.
"""
from __future__ import annotations

import collections
import os
import concurrent.futures as cf
from dataclasses import dataclass, field

import numpy as np
import torch


@dataclass
class TickBlock:
    slot: int
    data: torch.Tensor            # uint8 staging slot (pinned on GPU ranks)
    offs_t: torch.Tensor          # int64 record offsets (pinned), [n + 1] valid
    n: int = 0
    nbytes: int = 0
    offsets: dict = field(default_factory=dict)  # consumer offsets after this block
    event: object = None          # GPU event behind the H2D copy of this slot
    ends: np.ndarray | None = None  # true record ends where a region gap follows
    d_raw: torch.Tensor | None = None   # HBM copy of the slot (staged by the ingest thread)
    d_offs: torch.Tensor | None = None
    staged: object = None         # copy-stream event: d_raw/d_offs hold this block
    consumed: object = None       # compute-stream event: the tick is done with the slot
    parsed: tuple | None = None   # (num, cat, y, op) device views, parsed by the thread
    counts: np.ndarray | None = None  # host (training, forecasting, invalid) of `parsed`
    out: tuple | None = None      # slot-persistent parse outputs + counts buffers
    # gap-free device layout: (host start, device start, bytes) per filled region, the
    # device bytes, and the record offsets in it (pinned) — only the records cross PCIe,
    # not the regions' unused tails (a third of the slot at the 1.5x read caps)
    segs: list | None = None
    dev_nbytes: int = 0
    doffs_t: torch.Tensor | None = None
    ends_buf: np.ndarray | None = None  # native fill: the slot's record-end array

    @property
    def offs(self) -> np.ndarray:
        return self.offs_t.numpy()[: self.n + 1]

    @property
    def buf(self) -> np.ndarray:
        return self.data.numpy()[: self.nbytes]

    def raw(self):
        from omldm_amd.io.parse import RawView

        return RawView(self.buf, self.offs, self.ends)

    def to_bytes(self) -> tuple[bytes, np.ndarray]:
        """Detached, gap-free copy (records kept past this tick, e.g. the pre-Create
        buffer)."""
        if self.ends is None:
            return self.buf.tobytes(), self.offs.copy()
        from omldm_amd.io.transport import join_block

        return join_block(list(self.raw()))


class TickIngest:
    def __init__(self, consumers: list, batch_size: int, pinned: bool, prefetch: bool = True,
                 depth: int = 2, bytes_per_record: int = 1024, device=None,
                 copy_blocks: int = 128, space=None, copy_stream=None, parse_stream=None,
                 copy_method: str = "pull"):
        self.consumers = consumers
        self.space = space  # set: the ingest thread also parses each block on the GPU
        # GPU ranks: the ingest thread also moves each block to HBM on its own copy
        # stream (pull-copy kernel), so the tick only waits for an event
        self.device = torch.device(device) if device is not None else None
        self.stage = self.device is not None and self.device.type == "cuda" and pinned
        self.copy_blocks = copy_blocks
        # pull: the GPU reads the pinned slot (csrc/kernels/ingest.hip); sdma: a
        # hipMemcpyAsync on the copy stream (copy engine; enqueue stalls only hit this thread)
        assert copy_method in ("pull", "sdma"), copy_method
        self.copy_method = copy_method
        self._copy_stream = (copy_stream or torch.cuda.Stream(self.device)) if self.stage else None
        self.h2d_timer = self.parse_timer = None  # device time of the copies / GPU parses
        if self.stage:
            from omldm_amd.utils.devtimer import LaggedTimer

            self.h2d_timer, self.parse_timer = LaggedTimer(), LaggedTimer()
        self._parse_stream = parse_stream  # None: the parse follows the copy on its stream
        self.batch = max(1, int(batch_size))
        self.pinned = bool(pinned)
        self.slots: list[TickBlock] = []
        cap = self.batch * bytes_per_record
        # the tick's slot + `depth` read-ahead slots + one being recycled
        self.depth = max(1, int(depth)) if prefetch else 0
        for i in range(self.depth + 2):
            self.slots.append(TickBlock(i, self._alloc(cap, torch.uint8),
                                        self._alloc(len(consumers) * self.batch + 1, torch.int64)))
        self._k = 0
        # two pipeline stages on their own threads: host read of block k+2 ‖ H2D + GPU
        # parse of block k+1 ‖ the tick trains on block k
        self._pool = cf.ThreadPoolExecutor(1, thread_name_prefix="omldm-read-ahead") \
            if prefetch else None
        self._dev_pool = cf.ThreadPoolExecutor(1, thread_name_prefix="omldm-stage") \
            if prefetch and self.stage else None
        self._pending: collections.deque = collections.deque()
        nreg = sum(len(c.parts) for c in consumers)
        # one reader per partition region (GIL-free preads), up to 16: 8 reached 51 GB/s of
        # log reads into pinned memory on the MI355X host (scripts/read_bw_probe.py)
        nthr = int(os.environ.get("OMLDM_READERS", "16"))
        self._readers = cf.ThreadPoolExecutor(min(nthr, nreg), thread_name_prefix="omldm-read") \
            if nreg > 1 else None
        from omldm_amd.io.transport import FileBroker

        self._fds: dict = {}  # (consumer, partition) → the partition log's descriptor
        # file-log topics: one native call per block (OMLDM_NATIVE_FILL=0: the Python path)
        self._native_fill = (os.environ.get("OMLDM_NATIVE_FILL", "1") != "0" and consumers
                             and all(isinstance(c.broker, FileBroker) and hasattr(c, "read_plan")
                                     for c in consumers))

    def _alloc(self, n: int, dtype) -> torch.Tensor:
        return torch.empty(max(1, n), dtype=dtype, pin_memory=self.pinned)

    def _fill(self, blk: TickBlock) -> TickBlock:
        from omldm_amd.utils import tracing

        with tracing.range("ingest_read"):  # (reader thread) per-block cost, diagnostics
            return self._fill_block(blk)

    def _fill_block(self, blk: TickBlock) -> TickBlock:
        from omldm_amd.utils import tracing

        if blk.event is not None:
            with tracing.range("ingest_slot_wait"):
                blk.event.synchronize()  # the GPU has finished copying this slot's last use
            blk.event = None
        if self._native_fill:
            return self._fill_native(blk)
        # one region of the slot per (consumer, partition), sized from the observed
        # bytes per record; regions are read concurrently when the broker allows it
        jobs, pos = [], 0
        for c in self.consumers:
            for p, share, cap in c.read_plan(self.batch):
                cap = (cap + 15) & ~15  # 16-B aligned regions (the pull copy's vectors)
                jobs.append((c, p, share, pos, cap))
                pos += cap
        if pos > blk.data.numel():
            blk.data = self._alloc(int(pos * 1.25), torch.uint8)
        dst = blk.data.numpy()

        def read(j):
            c, p, share, start, cap = j
            return c.read_region(p, share, dst[start:start + cap])

        with tracing.range("ingest_pread"):
            if self._readers is not None and len(jobs) > 1 and \
                    all(c.broker.parallel_reads for c in self.consumers):
                results = list(self._readers.map(read, jobs))
            else:
                results = [read(j) for j in jobs]
        # Offsets: records of a region are contiguous; the first record of a region
        # starts at the region start, so the record before it also spans the unused tail
        # of its own region. Parsers stop at the record's closing brace; ``ends`` keeps
        # the true end of such records for the raw echo of forecasts.
        offs = blk.offs_t.numpy()
        offs[0] = 0
        if self.stage and (blk.doffs_t is None or blk.doffs_t.numel() < blk.offs_t.numel()):
            blk.doffs_t = self._alloc(blk.offs_t.numel(), torch.int64)
        doffs = blk.doffs_t.numpy() if self.stage else None
        n, end, gaps, segs, dpos = 0, 0, [], [], 0
        for (c, p, share, start, cap), (k, o) in zip(jobs, results):
            if not k:
                continue
            if n and start != end:
                gaps.append((n - 1, end))
            offs[n] = start
            offs[n + 1:n + k + 1] = o[1:k + 1] + start
            used = int(o[k])
            if doffs is not None:  # the same records packed (16-B aligned) for the device
                doffs[n:n + k + 1] = offs[n:n + k + 1] - (start - dpos)
                segs.append((start, dpos, used))
                dpos = (dpos + used + 15) & ~15
            n += k
            end = start + used
        blk.segs, blk.dev_nbytes = (segs, dpos) if doffs is not None else (None, 0)
        blk.ends = None
        if gaps:
            ends = offs[1:n + 1].copy()
            for i, e in gaps:
                ends[i] = e
            blk.ends = ends
        blk.n, blk.nbytes = n, end
        blk.offsets = [dict(c.offsets) for c in self.consumers]
        return blk

    def _fill_native(self, blk: TickBlock) -> TickBlock:
        """File-log topics: the whole block in one GIL-free call — the region reads on
        native threads and the block's record index assembled there
        (csrc/host/logio.cpp: omldm_fill_regions); same layout as the Python path."""
        from omldm_amd.ops import native
        from omldm_amd.utils import tracing

        rows, owners, pos = [], [], 0
        fds = self._fds
        for ci, c in enumerate(self.consumers):
            for p, share, cap in c.read_plan(self.batch):
                cap = (cap + 15) & ~15
                fd = fds.get((ci, p), -1)
                if fd < 0:  # a partition log opened once it exists
                    path = os.path.join(c.broker.root, c.topic, f"{p}.jsonl")
                    if os.path.exists(path):
                        fd = fds[(ci, p)] = c.broker._fd(path)
                rows.append((fd, c.offsets[p], pos, cap, share if fd >= 0 else 0,
                             int(share * c._avg_len * 1.02) + 4096))
                owners.append((c, p))
                pos += cap
        if pos > blk.data.numel():
            blk.data = self._alloc(int(pos * 1.25), torch.uint8)
        nj = len(rows)
        jobs = np.asarray(rows, dtype=np.int64).reshape(-1)
        if self.stage and (blk.doffs_t is None or blk.doffs_t.numel() < blk.offs_t.numel()):
            blk.doffs_t = self._alloc(blk.offs_t.numel(), torch.int64)
        if blk.ends_buf is None or blk.ends_buf.shape[0] < blk.offs_t.numel():
            blk.ends_buf = np.empty(blk.offs_t.numel(), dtype=np.int64)
        res, segs, meta = (np.zeros(2 * max(1, nj), dtype=np.int64),
                           np.zeros(3 * max(1, nj), dtype=np.int64), np.zeros(5, dtype=np.int64))
        doffs = blk.doffs_t.numpy() if self.stage else None
        with tracing.range("ingest_pread"):
            n = native.host().omldm_fill_regions(
                nj, jobs.ctypes.data, blk.data.data_ptr(), blk.offs_t.data_ptr(),
                blk.ends_buf.ctypes.data, 0 if doffs is None else doffs.ctypes.data,
                res.ctypes.data, segs.ctypes.data, meta.ctypes.data,
                max(1, int(os.environ.get("OMLDM_READERS", "16"))))
        if n < 0:
            raise OSError(-int(n), "reading the topic logs")
        for j, (c, p) in enumerate(owners):  # consumer positions + bytes-per-record estimate
            k, used = int(res[2 * j]), int(res[2 * j + 1])
            nxt = int(rows[j][1]) + used
            c.offsets[p] = nxt
            if k:
                c._avg_len = 0.8 * c._avg_len + 0.2 * (used / k)
            elif rows[j][0] >= 0 and c.broker.end_offset(c.topic, p) > nxt:
                c._avg_len *= 2
        n, end, dpos, nsegs, ngaps = (int(v) for v in meta)
        blk.segs = [tuple(int(v) for v in segs[3 * i:3 * i + 3]) for i in range(nsegs)] \
            if self.stage else None
        blk.dev_nbytes = dpos if self.stage else 0
        blk.ends = blk.ends_buf[:n] if ngaps else None
        blk.n, blk.nbytes = n, end
        blk.offsets = [dict(c.offsets) for c in self.consumers]
        return blk

    def _finish(self, blk: TickBlock) -> TickBlock:
        if self.stage and blk.n:
            from omldm_amd.utils import tracing

            with tracing.range("ingest_stage"):  # (staging thread) copy + parse + counts
                self._to_device(blk)
        return blk

    def _to_device(self, blk: TickBlock) -> None:
        from omldm_amd.ops.ingest import pull_copy_segs

        n = blk.n
        nbytes = blk.dev_nbytes if blk.segs is not None else blk.nbytes
        with torch.cuda.device(self.device):
            grow = (blk.d_raw is None or blk.d_raw.numel() < nbytes + 16 or
                    blk.d_offs is None or blk.d_offs.numel() < n + 1)
            if grow and blk.consumed is not None:
                blk.consumed.synchronize()  # old buffers are freed: nothing may read them
            if blk.d_raw is None or blk.d_raw.numel() < nbytes + 16:
                blk.d_raw = torch.empty(int((nbytes + 16) * 1.25), dtype=torch.uint8,
                                        device=self.device)
            if blk.d_offs is None or blk.d_offs.numel() < n + 1:
                blk.d_offs = torch.empty(blk.offs_t.numel(), dtype=torch.int64,
                                         device=self.device)
            cs = self._copy_stream
            if blk.consumed is not None:
                cs.wait_event(blk.consumed)  # the parser of this slot's last use is done
                blk.consumed = None
            self.h2d_timer.start(cs)
            segs = blk.segs if blk.segs is not None else [(0, 0, nbytes)]
            offs_src = blk.doffs_t if blk.segs is not None else blk.offs_t
            if self.copy_method == "sdma":
                with torch.cuda.stream(cs):
                    for h, d, ln in segs:
                        blk.d_raw[d:d + ln].copy_(blk.data[h:h + ln], non_blocking=True)
                    blk.d_offs[:n + 1].copy_(offs_src[:n + 1], non_blocking=True)
            else:  # the regions and the offsets in one launch
                hb, db = blk.data.data_ptr(), blk.d_raw.data_ptr()
                pull_copy_segs([(hb + h, db + d, ln) for h, d, ln in segs] +
                               [(offs_src.data_ptr(), blk.d_offs.data_ptr(), 8 * (n + 1))],
                               self.copy_blocks, cs.cuda_stream)
            self.h2d_timer.stop(cs, sum(ln for _, _, ln in segs) + 8 * (n + 1))
            blk.parsed = None
            if self.space is not None:
                ps = cs
                if self._parse_stream is not None:
                    copied = torch.cuda.Event()
                    copied.record(cs)
                    ps = self._parse_stream
                    ps.wait_event(copied)
                self.parse_timer.start(ps)
                self._parse(blk, ps)
                self.parse_timer.stop(ps, nbytes)
                cs = ps
            ev = torch.cuda.Event()
            ev.record(cs)
            blk.staged = ev
            blk.event = ev  # the host slot may be rewritten once this copy is done
            # the host-side counts are read by the tick (ops.ingest.parse_block) once the
            # event is done: this thread goes on to the next block's copy at once
            blk.counts = None

    def _parse(self, blk: TickBlock, cs) -> None:
        """JSON parse of the staged block into slot-persistent device outputs, plus the
        (training, forecasting, invalid) counts read back to pinned memory."""
        from omldm_amd.ops.ingest import json_parse

        sp, dev = self.space, self.device
        cap = self.batch * len(self.consumers)
        if blk.out is None:
            blk.out = (torch.empty((cap, sp.dn), dtype=torch.float32, device=dev),
                       torch.empty((cap, sp.dc), dtype=sp.cat_dtype, device=dev),
                       torch.empty(cap, dtype=torch.float32, device=dev),
                       torch.empty(cap, dtype=torch.int8, device=dev),
                       torch.zeros(3, dtype=torch.int32, device=dev),
                       torch.zeros(3, dtype=torch.int32, pin_memory=True))
        num, cat, y, op, cnt_d, cnt_h = blk.out
        with torch.cuda.stream(cs):
            cnt_d.zero_()
            json_parse(blk.d_raw, blk.d_offs, blk.n, sp, num, cat, y, op, cnt_d, cs.cuda_stream)
            cnt_h.copy_(cnt_d, non_blocking=True)
        blk.parsed = (num, cat, y, op)

    def _next_slot(self) -> TickBlock:
        blk = self.slots[self._k % len(self.slots)]
        self._k += 1
        return blk

    def _submit(self) -> None:
        blk = self._next_slot()
        f = self._pool.submit(self._fill, blk)
        if self._dev_pool is not None:
            f = self._dev_pool.submit(lambda fut=f: self._finish(fut.result()))
        self._pending.append(f)

    def next(self) -> TickBlock:
        """This tick's block; keeps ``depth`` blocks reading / staging behind it."""
        if self._pool is None:
            return self._finish(self._fill(self._next_slot()))
        if not self._pending:
            self._submit()
        blk = self._pending.popleft().result()
        if blk.n == 0:
            # idle stream: skip empty read-aheads, then poll once more now so that new
            # records are picked up by this tick (empty reads moved no offsets)
            while self._pending and blk.n == 0:
                blk = self._pending.popleft().result()
            if blk.n == 0:
                blk = self._finish(self._fill(blk))
        while len(self._pending) < self.depth:
            self._submit()
        return blk

    def drain(self) -> None:
        """Waits for the in-flight read-aheads (before reading/restoring offsets)."""
        for f in self._pending:
            f.result()

    def close(self) -> None:
        self.drain()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None
        if self._dev_pool is not None:
            self._dev_pool.shutdown(wait=True)
            self._dev_pool = None
        if self._readers is not None:
            self._readers.shutdown(wait=True)
            self._readers = None
