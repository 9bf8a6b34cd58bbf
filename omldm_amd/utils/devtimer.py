"""Device-time accounting without host synchronisation (SURVEY §5.5 metrics).

A ``LaggedTimer`` records a pair of timing events around GPU work on a stream and adds
the pair's elapsed time once both events have completed, polled with ``Event.query()``
— the tick never waits for its own work to be timed (the readings trail by a tick or
two). Used for the H2D copy bandwidth and the parse time of the ingest lane, the training
rounds' device time and the collectives' device time (engine/job.py: ``_metrics``).
"""
from __future__ import annotations

import collections

import torch


class LaggedTimer:
    def __init__(self, max_pending: int = 64):
        self.ms = 0.0
        self.count = 0
        self.bytes = 0
        self._pending: collections.deque = collections.deque()
        self._open = None
        self.max_pending = max_pending

    def start(self, stream=None) -> None:
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self._open = e

    def stop(self, stream=None, nbytes: int = 0) -> None:
        if self._open is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self._pending.append((self._open, e, int(nbytes)))
        self._open = None
        self.poll()
        while len(self._pending) > self.max_pending:  # bounded: settle the oldest
            a, b, n = self._pending.popleft()
            b.synchronize()
            self._add(a, b, n)

    def _add(self, a, b, n) -> None:
        self.ms += a.elapsed_time(b)
        self.count += 1
        self.bytes += n

    def poll(self) -> None:
        while self._pending and self._pending[0][1].query():
            a, b, n = self._pending.popleft()
            self._add(a, b, n)

    def settle(self) -> None:
        """Waits for every recorded pair (end of job)."""
        while self._pending:
            a, b, n = self._pending.popleft()
            b.synchronize()
            self._add(a, b, n)

    def gbps(self) -> float | None:
        return round(self.bytes / (self.ms * 1e6), 2) if self.ms > 0 and self.bytes else None
