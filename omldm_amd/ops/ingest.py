"""Host→HBM ingest engines (csrc/kernels/copy_engine.hip, csrc/kernels/ingest.hip).

* ``CopyEngine`` — a native host thread submits SDMA copies (split over several streams)
  so the training thread never blocks on PCIe; GPU-side events order buffer reuse and
  consumption.
* ``pull_copy`` — a copy kernel reading the pinned host buffer over PCIe.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from omldm_amd.ops import native


def copy_cu_bits(total: int, ncu: int, layout: int) -> set[int]:
    """CU-mask bits of the ingest lane (same choice as omldm_stream_create_cumask_ex)."""
    if ncu <= 0 or ncu >= total:
        return set(range(total))
    if layout == 1:
        return set(range(ncu))
    step = total // ncu
    return {total - 1 - i * step for i in range(ncu)}


def reserve_cu_bits(total: int, n: int, taken: set[int], nxcd: int = 8) -> set[int]:
    """n CU-mask bits outside ``taken``, spread evenly over the XCDs. The bit → XCD map
    (round-robin c % nxcd, or blocked c // (total / nxcd)) is measured by
    scripts/cumask_probe.py; a bit c = per·x + x + nxcd·j is on XCD x under both, so the
    choice does not depend on which one the runtime uses."""
    if n <= 0:
        return set()
    if total % nxcd:
        nxcd = 1
    per = total // nxcd
    quota = -(-n // nxcd)
    out: set[int] = set()
    for x in range(nxcd):
        got = 0
        for j in range(per // nxcd):
            c = per * x + x + nxcd * j
            if c < total and c not in taken and got < quota and len(out) < n:
                out.add(c)
                got += 1
    return out


def cumask_stream(bits: set[int], total: int, device=None):
    """A torch ExternalStream restricted to the CUs in ``bits`` (returns (stream, raw))."""
    words = (total + 31) // 32
    arr = (native.u32 * words)()
    for c in bits:
        arr[c >> 5] |= 1 << (c & 31)
    raw = native.hip().omldm_stream_create_cumask_words(arr, words)
    if not raw:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    return torch.cuda.ExternalStream(raw, device=device), raw


class CopyEngine:
    def __init__(self, nstreams: int = 2):
        self.lib = native.hip()
        self.h = self.lib.omldm_copy_engine_create(int(nstreams))
        if not self.h:
            raise RuntimeError("omldm_copy_engine_create failed")

    def event(self):
        ev = self.lib.omldm_event_create()
        if not ev:
            raise RuntimeError("hipEventCreate failed")
        return ev

    def record(self, ev, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        native.check(self.lib.omldm_event_record(ev, s), "hipEventRecord")

    def submit(self, dst: torch.Tensor, src: torch.Tensor, wait_ev, done_ev) -> int:
        n = src.numel() * src.element_size()
        assert dst.numel() * dst.element_size() >= n and src.is_pinned() and dst.is_cuda
        return int(self.lib.omldm_copy_engine_submit(self.h, dst.data_ptr(), src.data_ptr(), n,
                                                     wait_ev, done_ev))

    def stream_wait(self, ticket: int, done_ev, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        native.check(self.lib.omldm_copy_engine_stream_wait(self.h, ticket, done_ev, s),
                     "copy_engine_stream_wait")

    def close(self) -> None:
        if self.h:
            self.lib.omldm_copy_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class XcdLanes:
    """CU-masked streams: ``copy`` on a contiguous block of ``ingest_cus`` CUs (inside
    one XCD) for host→HBM pull copies; ``compute`` and ``aux`` on every other CU. A pull
    copy spread over the chip lets its long-latency PCIe reads occupy every XCD's L2 and
    slows training; confined to one XCD it runs at the PCIe peak next to training
    (profiles/round1_ablation.md, "XCD-local ingest"). The streams are blocking
    (hipExtStreamCreateWithCUMask): nothing may run on the legacy default stream
    meanwhile, so the user switches all its GPU work to ``compute``.

    One set per (device, ingest_cus) for the whole process (``XcdLanes.get``): events and
    pinned-memory bookkeeping recorded on a stream must never outlive it, so the streams
    are never destroyed while the process runs."""

    _cache: dict = {}

    def __init__(self, device, ingest_cus: int = 16):
        lib = native.hip()
        self.device = torch.device(device)
        with torch.cuda.device(self.device):
            raw = [lib.omldm_stream_create_cumask_ex(int(ingest_cus), 0, 1),
                   lib.omldm_stream_create_cumask_ex(int(ingest_cus), 1, 1),
                   lib.omldm_stream_create_cumask_ex(int(ingest_cus), 1, 1),
                   lib.omldm_stream_create_cumask_ex(int(ingest_cus), 1, 1)]
        if not all(raw):
            raise RuntimeError("hipExtStreamCreateWithCUMask failed")
        self.copy = torch.cuda.ExternalStream(raw[0], device=self.device)
        self.compute = torch.cuda.ExternalStream(raw[1], device=self.device)
        # a second stream on the compute CUs for work the ingest thread issues after a
        # copy (the JSON parse), so it neither queues behind training nor runs on the
        # ingest CUs
        self.aux = torch.cuda.ExternalStream(raw[2], device=self.device)
        # the engine's route / prep-ahead stream (engine/job.py), also off the ingest CUs
        self.prep = torch.cuda.ExternalStream(raw[3], device=self.device)

    @classmethod
    def get(cls, device, ingest_cus: int = 16) -> "XcdLanes":
        dev = torch.device(device)
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), ingest_cus)
        if key not in cls._cache:
            cls._cache[key] = cls(dev, ingest_cus)
        return cls._cache[key]


def pull_copy(dst: torch.Tensor, src: torch.Tensor, blocks: int = 16, stream=None) -> None:
    s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    native.check(native.hip().omldm_pull_copy(src.data_ptr(), dst.data_ptr(),
                                              src.numel() * src.element_size(), blocks, s),
                 "omldm_pull_copy")


def pull_copy_segs(segs: list, blocks: int = 128, stream=None) -> None:
    """One launch for several (host src ptr, device dst ptr, bytes) copies
    (csrc/kernels/ingest.hip: pull_copy_segs_kernel); pointers 16-B aligned."""
    if not segs:
        return
    s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    arr = np.asarray(segs, dtype=np.int64).reshape(-1)
    native.check(native.hip().omldm_pull_copy_segs(arr.ctypes.data, len(segs), blocks, s),
                 "omldm_pull_copy_segs")


def json_parse(dbuf, doffs, n: int, space, num, cat, y, op, counts, stream) -> None:
    """Launches csrc/kernels/json_ingest.hip on HBM-resident records (one thread each);
    ``counts`` (3 × int32, accumulated) receives training / forecasting / invalid."""
    assert num.shape[0] >= n and cat.shape[0] >= n and y.shape[0] >= n and op.shape[0] >= n
    assert doffs.numel() >= n + 1 and counts.numel() >= 3
    native.check(native.hip().omldm_json_parse(
        dbuf.data_ptr(), doffs.data_ptr(), n, space.n_numerical, space.n_discrete, space.dc,
        space.dim, space.cat_span, num.data_ptr(), cat.data_ptr(), y.data_ptr(), op.data_ptr(),
        counts.data_ptr(), stream), "omldm_json_parse")


class GpuJsonParser:
    """Parses a block of DataInstance JSON records on the GPU
    (csrc/kernels/json_ingest.hip): the raw bytes go to HBM through a pinned staging ring
    and one thread per record produces the columnar hashed batch in place — the host
    only indexes record boundaries."""

    def __init__(self, device, slots: int = 2):
        self.device = torch.device(device)
        self.slots = [None] * slots
        self.events = [None] * slots
        self.k = 0

    def _stage(self, buf: bytes) -> torch.Tensor:
        import numpy as np

        i = self.k % len(self.slots)
        self.k += 1
        if self.events[i] is not None:
            self.events[i].synchronize()  # staging slot reused only after its copy finished
        n = max(1, len(buf))
        if self.slots[i] is None or self.slots[i].numel() < n:
            self.slots[i] = torch.empty(max(n, 1 << 20), dtype=torch.uint8, pin_memory=True)
        st = self.slots[i]
        if buf:
            st.numpy()[: len(buf)] = np.frombuffer(buf, dtype=np.uint8)
        d = st[:n].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev
        return d

    def _dev(self, key: str, n: int, dtype) -> torch.Tensor:
        t = getattr(self, key, None)
        if t is None or t.numel() < n:
            t = torch.empty(max(n, 1 << 16), dtype=dtype, device=self.device)
            setattr(self, key, t)
        return t

    def parse_block(self, blk, space, copy_blocks: int = 32):
        """Parses a pinned ``engine.ingest.TickBlock``. Returns (device batch with a lazy
        raw view, device int8 op, counts) where counts = (training, forecasting,
        invalid) — a host ndarray when the ingest thread already parsed the block
        (``blk.parsed``: this stream only waits for its event), else a device tensor.
        Otherwise the bytes and offsets move to HBM with the pull-copy kernel
        (non-blocking for the host) and the parse kernel follows on this stream."""
        from omldm_amd.api.batch import HashedBatch

        n, nbytes = blk.n, blk.nbytes
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        if blk.parsed is not None:
            cur.wait_event(blk.staged)
            if blk.counts is None:  # staged a tick ahead: normally done by now
                from omldm_amd.utils import tracing

                with tracing.range("ingest_counts_wait"):
                    blk.staged.synchronize()
                blk.counts = blk.out[5].numpy().copy()
            num, cat, y, op = (t[:n] for t in blk.parsed)
            return HashedBatch(num, cat, y, blk.raw(), space.cat_span), op, blk.counts.copy()
        num = torch.empty((n, space.dn), dtype=torch.float32, device=dev)
        cat = torch.empty((n, space.dc), dtype=space.cat_dtype, device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        op = torch.empty(n, dtype=torch.int8, device=dev)
        counts = torch.zeros(3, dtype=torch.int32, device=dev)
        if n > 0:
            s = cur.cuda_stream
            if blk.staged is not None:  # moved to HBM by the ingest thread
                cur.wait_event(blk.staged)
                dbuf, doffs = blk.d_raw, blk.d_offs
            else:
                assert blk.data.is_pinned() and blk.offs_t.is_pinned()
                dbuf = self._dev("_raw", nbytes + 16, torch.uint8)
                doffs = self._dev("_offs", n + 1, torch.int64)
                pull_copy(dbuf, blk.data[:nbytes], copy_blocks, s)
                pull_copy(doffs, blk.offs_t[: n + 1], copy_blocks, s)
                ev = torch.cuda.Event()
                ev.record()
                blk.event = ev
            assert dbuf.numel() >= nbytes and doffs.numel() >= n + 1
            json_parse(dbuf, doffs, n, space, num, cat, y, op, counts, s)
        return HashedBatch(num, cat, y, blk.raw(), space.cat_span), op, counts

    def parse(self, buf: bytes, offs, space):
        """Returns (device HashedBatch with a lazy raw view, device int8 op, device int32
        counts: training, forecasting, invalid)."""
        import numpy as np

        from omldm_amd.api.batch import HashedBatch
        from omldm_amd.io.parse import RawView

        n = len(offs) - 1
        dev = self.device
        num = torch.empty((n, space.dn), dtype=torch.float32, device=dev)
        cat = torch.empty((n, space.dc), dtype=space.cat_dtype, device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        op = torch.empty(n, dtype=torch.int8, device=dev)
        counts = torch.zeros(3, dtype=torch.int32, device=dev)
        if n > 0:
            dbuf = self._stage(buf)
            offs64 = np.ascontiguousarray(offs, dtype=np.int64)
            doffs = torch.from_numpy(offs64).to(dev, non_blocking=False)
            json_parse(dbuf, doffs, n, space, num, cat, y, op, counts,
                       torch.cuda.current_stream(dev).cuda_stream)
        return HashedBatch(num, cat, y, RawView(buf, offs), space.cat_span), op, counts


def hash_raw(tok: torch.Tensor, space) -> torch.Tensor:
    """Raw token ids [B, dc] → wide hashed slots [B, dc] int32 (sign in bit 31, -1 =
    absent), the csrc/host/hashing.h function on CPU and on the device."""
    assert tok.dtype == torch.int32 and tok.is_contiguous()
    out = torch.empty_like(tok)
    B, dc = tok.shape
    if tok.is_cuda:
        native.check(native.hip().omldm_hash_raw(native.ptr(tok), B, dc, space.dn, space.dim,
                                                 native.ptr(out), native.stream_of(tok)),
                     "omldm_hash_raw")
    else:
        native.host().omldm_cpu_hash_raw(native.ptr(tok), B, dc, space.dn, space.dim,
                                     native.ptr(out), min(16, os.cpu_count() or 1))
    return out
