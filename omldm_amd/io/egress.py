"""Prediction egress: a forecast batch becomes one block of Prediction JSON lines.

Reference: each forecast is a ``Prediction`` sunk to the predictions topic with
``toString`` (omldm/network/FlinkNetwork.scala:243-257, omldm/Job.scala:99-105), echoing
the forecasting DataInstance (omldm/utils/parsers/dataStream/DataPointParser.scala:38-46).
Here the native formatter (csrc/host/egress.cpp) copies each record's raw bytes from
the tick's staging block and prints the number like ``json.dumps`` — no per-record
Python objects; brokers append the block in one call where they can.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from omldm_amd.ops import native


@dataclass
class RawRecords:
    """Byte ranges [starts[i], ends[i]) of selected records inside one buffer."""

    buf: np.ndarray      # uint8
    starts: np.ndarray   # int64
    ends: np.ndarray     # int64

    @staticmethod
    def from_view(view, idx: np.ndarray | None = None) -> "RawRecords":
        """From an ``io.parse.RawView`` or a list of records (optionally a subset)."""
        if isinstance(view, (list, tuple)):
            from omldm_amd.io.parse import RawView
            from omldm_amd.io.transport import join_block

            view = RawView(*join_block([r if isinstance(r, (bytes, bytearray)) else
                                        str(r).encode() for r in view]))
        buf = view.buf
        if isinstance(buf, (bytes, bytearray)):
            buf = np.frombuffer(buf, dtype=np.uint8)
        offs = np.asarray(view.offs, dtype=np.int64)
        starts = offs[:-1]
        ends = offs[1:] if view.ends is None else np.asarray(view.ends, dtype=np.int64)
        if idx is not None:
            starts, ends = starts[idx], ends[idx]
        return RawRecords(buf, np.ascontiguousarray(starts), np.ascontiguousarray(ends))

    def __len__(self) -> int:
        return int(self.starts.shape[0])


def _format(raw: RawRecords, lo: int, hi: int, mlp_id: int, p: np.ndarray):
    n = hi - lo
    offs = np.zeros(n + 1, dtype=np.int64)
    if n == 0:
        return np.empty(0, dtype=np.uint8), offs
    starts, ends = raw.starts[lo:hi], raw.ends[lo:hi]
    cap = int((ends - starts).sum()) + n * 128
    for _ in range(2):
        out = np.empty(cap, dtype=np.uint8)
        got = native.host().omldm_format_predictions(
            raw.buf.ctypes.data, starts.ctypes.data, ends.ctypes.data, n, int(mlp_id),
            p[lo:hi].ctypes.data, out.ctypes.data, cap, offs.ctypes.data)
        if got >= 0:
            return out[:got], offs
        cap = -got
    raise RuntimeError("omldm_format_predictions: output sizing failed")


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        import concurrent.futures as cf
        import os

        _POOL = cf.ThreadPoolExecutor(min(8, os.cpu_count() or 1),
                                      thread_name_prefix="omldm-egress-fmt")
    return _POOL


def format_predictions_chunks(raw: RawRecords, mlp_id: int, preds,
                              chunk: int = 16384) -> list[tuple[np.ndarray, np.ndarray]]:
    """Like ``format_predictions`` but formats chunks of records on a thread pool (the
    native formatter runs without the GIL); returns the blocks in record order."""
    p = np.ascontiguousarray(np.asarray(preds, dtype=np.float32))
    n = len(raw)
    assert p.shape[0] == n
    raw = RawRecords(np.ascontiguousarray(raw.buf), np.ascontiguousarray(raw.starts),
                     np.ascontiguousarray(raw.ends))
    bounds = [(lo, min(n, lo + chunk)) for lo in range(0, n, chunk)]
    if len(bounds) <= 1:
        return [_format(raw, 0, n, mlp_id, p)] if n else []
    return list(_pool().map(lambda b: _format(raw, b[0], b[1], mlp_id, p), bounds))


def format_predictions(raw: RawRecords, mlp_id: int, preds) -> tuple[bytes, np.ndarray]:
    """Prediction JSON lines for ``preds[i]`` of record i → (block, line offsets[n+1])."""
    p = np.ascontiguousarray(np.asarray(preds, dtype=np.float32))
    assert p.shape[0] == len(raw)
    raw = RawRecords(np.ascontiguousarray(raw.buf), np.ascontiguousarray(raw.starts),
                     np.ascontiguousarray(raw.ends))
    out, offs = _format(raw, 0, len(raw), mlp_id, p)
    return out.tobytes(), offs


class EgressWriter:
    """Producer thread for output topics (a Kafka producer's send thread): the tick hands
    over formatted blocks and moves on; blocks are appended in submission order.
    ``flush()`` waits until everything submitted is in the broker."""

    def __init__(self, broker, enabled: bool = True):
        import concurrent.futures as cf

        self.broker = broker
        self._ex = cf.ThreadPoolExecutor(1, thread_name_prefix="omldm-egress") if enabled else None
        self._futs: list = []

    def submit(self, topic: str, block, offs: np.ndarray) -> None:
        if self._ex is None:
            self.broker.produce_lines(topic, block, offs)
            return
        self._futs = [f for f in self._futs if not f.done()]
        for f in self._futs:  # surface producer errors on the tick thread
            if f.done():
                f.result()
        self._futs.append(self._ex.submit(self.broker.produce_lines, topic, block, offs))

    def flush(self) -> None:
        futs, self._futs = self._futs, []
        for f in futs:
            f.result()

    def close(self) -> None:
        self.flush()
        if self._ex is not None:
            self._ex.shutdown(wait=True)
            self._ex = None
