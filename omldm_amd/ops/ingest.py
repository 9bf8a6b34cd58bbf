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
