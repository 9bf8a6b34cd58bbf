"""Persistent low-latency predict server (csrc/kernels/serving.hip).

One resident wavefront polls a coherent pinned host mailbox; a request is a host write
+ sequence bump, the answer comes back through the same mailbox — no kernel launch or
stream synchronisation on the request path. The wave exits on ``stop()`` or after its
lifetime. It reads one of two weight banks (``w`` / ``w1``), chosen per request: a
publisher writes new models into the bank no request reads and switches requests over
once the copy is complete (engine/forecast_server.py), so an answer never mixes versions.
"""
from __future__ import annotations

import ctypes as C

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.ops import native
from omldm_amd.ops.native import check, ptr

SIGS = [
    ("omldm_mailbox_alloc", C.c_void_p, []),
    ("omldm_mailbox_free", None, [C.c_void_p]),
    ("omldm_serve_start", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_longlong, C.c_int,
                                    C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                    C.c_longlong, C.c_void_p]),
    ("omldm_serve_request", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                      C.c_int, C.c_void_p, C.c_longlong, C.c_int]),
    ("omldm_serve_stop", None, [C.c_void_p]),
    ("omldm_serve_alive", C.c_int, [C.c_void_p]),
    ("omldm_serve_exit_reason", C.c_int, [C.c_void_p]),
    ("omldm_bank_word_alloc", C.c_void_p, []),
    ("omldm_bank_word_free", None, [C.c_void_p]),
    ("omldm_bank_word_set", C.c_int, [C.c_void_p, C.c_uint, C.c_void_p]),
]


def _lib():
    lib = native.hip()
    if not hasattr(lib, "omldm_serve_start"):
        for name, res, args in SIGS:
            fn = getattr(lib.cdll, name)
            fn.restype, fn.argtypes = res, args
            setattr(lib, name, fn)
    return lib


class PredictServer:
    def __init__(self, w: torch.Tensor, dn: int, dc: int, bias: bool = True, cat_span: int = 0,
                 w1: torch.Tensor | None = None):
        assert w.is_cuda
        self.lib = _lib()
        self.W = w if w.dim() == 2 else w.unsqueeze(0)
        self.W1 = None if w1 is None else (w1 if w1.dim() == 2 else w1.unsqueeze(0))
        assert self.W1 is None or (self.W1.shape == self.W.shape and
                                   self.W1.stride() == self.W.stride() and
                                   self.W1.dtype == self.W.dtype)
        self.M, self.dim = int(self.W.shape[0]), int(self.W.shape[1])
        self.dn, self.dc, self.bias, self.cspan = dn, dc, bias, cat_span
        self.mb = self.lib.omldm_mailbox_alloc()
        if not self.mb:
            raise RuntimeError("hipHostMalloc(coherent) failed for the serving mailbox")
        # The resident wave must not block other work queued on the device: a blocking
        # stream (e.g. hipExtStreamCreateWithCUMask's) serialises with the legacy default
        # stream, and a normal-priority pool stream can share a hardware queue with the
        # training streams. Measured (scripts/diag_serve_queue.py): a high-priority,
        # non-blocking stream never delays work on other streams.
        self._raw_stream = None
        self.stream = torch.cuda.Stream(w.device, priority=-1)
        self.out = (C.c_float * self.M)()

    def start(self, lifetime_us: int = 10_000_000) -> None:
        check(self.lib.omldm_serve_start(ptr(self.W), ptr(self.W1),
                                         int(self.W.dtype == torch.bfloat16),
                                         self.W.stride(0), self.M, self.dn, self.dc, self.dim,
                                         int(self.bias), self.cspan, self.mb, int(lifetime_us),
                                         self.stream.cuda_stream), "omldm_serve_start")
        import time

        t = time.time()
        while not self.lib.omldm_serve_alive(self.mb):
            if time.time() - t > 10:
                raise RuntimeError("serving wave did not start")
            time.sleep(1e-4)

    def request_raw(self, num_ptr: int, cat_ptr: int, timeout_us: int = 1_000_000,
                    bank: int = 0) -> list[float]:
        rc = self.lib.omldm_serve_request(self.mb, num_ptr, self.dn, cat_ptr, self.dc, self.M,
                                          self.out, timeout_us, int(bank))
        if rc:
            raise TimeoutError("serving wave did not answer")
        return list(self.out)

    def request(self, point: HashedBatch, bank: int = 0) -> list[float]:
        """Scores of one point (row 0 of a host batch) against the M models."""
        num = point.num[0].float().contiguous()
        cat = point.cat[0].to(torch.int64)
        if point.cat_span:
            cat = cat & 0xFFFF
        cat = cat.to(torch.int32).contiguous()
        return self.request_raw(num.data_ptr(), cat.data_ptr(), bank=bank)

    def stop(self) -> None:
        self.lib.omldm_serve_stop(self.mb)
        self.stream.synchronize()

    def close(self) -> None:
        if self.mb:
            self.stop()
            self.lib.omldm_mailbox_free(self.mb)
            self.mb = None
        if getattr(self, "_raw_stream", None):
            native.hip().omldm_stream_destroy(self._raw_stream)
            self._raw_stream = None
