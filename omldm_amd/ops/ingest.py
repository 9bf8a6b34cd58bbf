"""Host→HBM ingest engines (csrc/kernels/copy_engine.hip, csrc/kernels/ingest.hip).

* ``CopyEngine`` — a native host thread submits SDMA copies (split over several streams)
  so the training thread never blocks on PCIe; GPU-side events order buffer reuse and
  consumption.
* ``pull_copy`` — a copy kernel reading the pinned host buffer over PCIe.
"""
from __future__ import annotations

import torch

from omldm_amd.ops import native


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


def pull_copy(dst: torch.Tensor, src: torch.Tensor, blocks: int = 16, stream=None) -> None:
    s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    native.check(native.hip().omldm_pull_copy(src.data_ptr(), dst.data_ptr(),
                                              src.numel() * src.element_size(), blocks, s),
                 "omldm_pull_copy")


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

    def parse(self, buf: bytes, offs, space):
        """Returns (device HashedBatch with a lazy raw view, device int8 op, device int32
        valid count)."""
        import numpy as np

        from omldm_amd.api.batch import HashedBatch
        from omldm_amd.io.parse import RawView

        n = len(offs) - 1
        dev = self.device
        num = torch.empty((n, space.dn), dtype=torch.float32, device=dev)
        cat = torch.empty((n, space.dc), dtype=space.cat_dtype, device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        op = torch.empty(n, dtype=torch.int8, device=dev)
        nvalid = torch.zeros(1, dtype=torch.int32, device=dev)
        if n > 0:
            dbuf = self._stage(buf)
            offs64 = np.ascontiguousarray(offs, dtype=np.int64)
            doffs = torch.from_numpy(offs64).to(dev, non_blocking=False)
            native.check(native.hip().omldm_json_parse(
                dbuf.data_ptr(), doffs.data_ptr(), n, space.n_numerical, space.n_discrete,
                space.dc, space.dim, space.cat_span, num.data_ptr(), cat.data_ptr(),
                y.data_ptr(), op.data_ptr(), nvalid.data_ptr(),
                torch.cuda.current_stream(dev).cuda_stream), "omldm_json_parse")
        return HashedBatch(num, cat, y, RawView(buf, offs), space.cat_span), op, nvalid
