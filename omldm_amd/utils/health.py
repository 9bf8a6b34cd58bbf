"""Device-side failure detection that never stalls a tick (failure detection).

Two conditions must stop the job instead of silently degrading the model:

* a dropped update — a spoke learner's round could not place a key even in its HBM spill
  (csrc/kernels/spoke_table.h; the learners' running ``overflow`` counter, cum[5]);
* a combiner timeout of the v3 scan — an in-launch combiner workgroup gave up waiting for
  its spoke's granules (csrc/kernels/linear_scan3.hip: g_s3_comb_err), so part of that
  spoke's update never reached the round accumulator.

Both live on the device. ``arm()`` (end of a tick) enqueues their copy into a pinned host
block on the compute stream and records an event; ``check()`` (the next tick) reads the
block once that event has completed — one tick late, no host synchronisation on the hot
path — and raises :class:`DeviceHealthError`.
"""
from __future__ import annotations

import torch


class DeviceHealthError(RuntimeError):
    pass


class DeviceHealth:
    MAXP = 64  # pipelines whose overflow counters fit the block

    def __init__(self, device):
        self.device = torch.device(device)
        self.host = torch.zeros(2 + self.MAXP, dtype=torch.float64, pin_memory=True)
        self.flag = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        self.stage = torch.zeros(self.MAXP, dtype=torch.float64, device=self.device)
        self.event = None
        self.pids: list = []

    def arm(self, pipes: dict) -> None:
        """Enqueue the copies of this tick's health words (current stream)."""
        from omldm_amd.ops import native

        h = native.hip()
        self.check(block=False)
        if getattr(h, "omldm_scan3_comb_err_drain", None) is not None:
            native.check(h.omldm_scan3_comb_err_drain(native.dptr(self.flag), native.stream_of(
                self.stage)), "omldm_scan3_comb_err_drain")
        pids = [pid for pid in sorted(pipes) if getattr(pipes[pid].learner, "cum", None) is not None]
        pids = pids[: self.MAXP]
        for i, pid in enumerate(pids):
            self.stage[i : i + 1].copy_(pipes[pid].learner.cum[5:6])
        if pids:
            self.host[2 : 2 + len(pids)].copy_(self.stage[: len(pids)], non_blocking=True)
        self.pids = pids
        self.event = torch.cuda.Event()
        self.event.record()

    def check(self, block: bool = True) -> None:
        """Raise if the last armed tick saw a dropped update or a combiner timeout."""
        ev = self.event
        if ev is None:
            return
        if not ev.query():
            if not block:
                return  # still in flight: checked at the next arm / check
            ev.synchronize()
        self.event = None
        code = int(self.flag[0])
        if code:
            self.flag[0] = 0
            what = {1: "an in-launch combiner timed out waiting for its spoke's granules",
                    2: "a helper workgroup's bounded spin gave up",
                    3: "the round's prep never set its ready word (the round waited for a "
                       "prep that did not run)"}
            raise DeviceHealthError(
                f"v3 scan: {what.get(code, 'a bounded in-launch wait failed')} "
                f"(linear_scan3.hip g_s3_comb_err = {code}); the round was discarded")
        bad = {pid: int(self.host[2 + i]) for i, pid in enumerate(self.pids)
               if float(self.host[2 + i]) != 0.0}
        if bad:
            raise DeviceHealthError(f"dropped spoke updates (overflow counter) in pipelines {bad}")
