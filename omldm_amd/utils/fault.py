"""Failure detection and fault injection.

Reference: failure detection is left to the Flink JobManager with no restart strategy
(``RestartStrategies`` imported, unused: omldm/Job.scala:14); liveness is only the
idle-timeout detector fed by spoke heartbeats (omldm/utils/statistics/
StatisticsOperator.scala:87-91,135-142; FlinkSpoke.scala:83-89); there is no fault
injection.

Here:
* ``Watchdog`` — a rank-level heartbeat monitor. The job beats it once per tick (every
  tick already carries a global heartbeat all-reduce, so a dead or hung peer stalls
  every rank inside a collective). When no beat arrives for ``timeout`` the watchdog
  aborts the communicator (so RCCL/gloo calls of the other threads return) and exits
  the process with ``EXIT_WATCHDOG`` — the supervisor (omldm_amd/launch.py) then
  restarts the job from its last checkpoint, possibly on fewer ranks.
* ``FaultPlan`` — deterministic fault injection for tests, from ``--faults`` or the
  ``OMLDM_FAULTS`` env var, ``;``-separated specs:
      kill:rank=1:tick=20            exit abruptly (code EXIT_INJECTED) at that tick
      hang:rank=0:tick=5             stop making progress (watchdog test)
      delay:rank=1:ms=50[:every=1]   slow rank (straggler / SSP staleness tests)
      drop:rank=0:tag=push[:every=3] lose this rank's contribution to a collective
                                     (the message is zeroed, the rank still joins so
                                     the collective stays aligned)
  Faults apply only to supervisor attempt 0 unless ``attempt=N`` is given.
"""
from __future__ import annotations

import os
import sys
import threading
import time

EXIT_WATCHDOG = 75
EXIT_INJECTED = 17


class FaultPlan:
    def __init__(self, spec: str = "", rank: int = 0, attempt: int | None = None):
        self.rank = rank
        self.attempt = int(os.environ.get("OMLDM_ATTEMPT", "0")) if attempt is None else attempt
        self.rules: list[dict] = []
        for part in (spec or "").split(";"):
            part = part.strip()
            if not part:
                continue
            kind, *kvs = part.split(":")
            r = {"kind": kind}
            for kv in kvs:
                k, _, v = kv.partition("=")
                r[k] = v
            if int(r.get("rank", rank)) != rank or int(r.get("attempt", 0)) != self.attempt:
                continue
            self.rules.append(r)
        self._drops: dict[str, int] = {}

    @staticmethod
    def from_config(cfg, rank: int) -> "FaultPlan":
        spec = cfg.extra.get("faults") or os.environ.get("OMLDM_FAULTS", "")
        return FaultPlan(spec, rank)

    def __bool__(self):
        return bool(self.rules)

    def on_tick(self, tick: int) -> None:
        for r in self.rules:
            k = r["kind"]
            if k == "kill" and tick == int(r.get("tick", 0)):
                sys.stderr.write(f"[fault] rank {self.rank}: injected kill at tick {tick}\n")
                sys.stderr.flush()
                os._exit(EXIT_INJECTED)
            if k == "hang" and tick == int(r.get("tick", 0)):
                sys.stderr.write(f"[fault] rank {self.rank}: injected hang at tick {tick}\n")
                sys.stderr.flush()
                while True:
                    time.sleep(3600)
            if k == "delay" and tick % max(1, int(r.get("every", 1))) == 0:
                time.sleep(float(r.get("ms", 10)) / 1000.0)

    def drop(self, tag: str) -> bool:
        for r in self.rules:
            if r["kind"] == "drop" and r.get("tag", tag) == tag:
                n = self._drops.get(tag, 0) + 1
                self._drops[tag] = n
                if n % max(1, int(r.get("every", 1))) == 0:
                    return True
        return False


class Watchdog:
    """Exits the process if ``beat()`` is not called for ``timeout_s`` seconds."""

    def __init__(self, timeout_s: float, rank: int = 0, on_expire=None):
        self.timeout = float(timeout_s)
        self.rank = rank
        self.last = time.monotonic()
        self.on_expire = on_expire
        self.expired = False
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="omldm-watchdog", daemon=True)
        if self.timeout > 0:
            self._t.start()

    def beat(self) -> None:
        self.last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()

    def _run(self):
        period = min(1.0, self.timeout / 4)
        while not self._stop.wait(period):
            if time.monotonic() - self.last > self.timeout:
                self.expired = True
                sys.stderr.write(f"[watchdog] rank {self.rank}: no progress for "
                                 f"{self.timeout:.1f}s — aborting\n")
                sys.stderr.flush()
                try:  # where every thread is stuck: the first thing a hang report needs
                    import faulthandler
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                except Exception:
                    pass
                if self.on_expire is not None:
                    self.on_expire()
                    return
                abort_communicator()
                os._exit(EXIT_WATCHDOG)


def abort_communicator() -> None:
    """Best effort: abort the default process group so blocked collectives return
    (ncclCommAbort on RCCL)."""
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            pg = dist.distributed_c10d._get_default_group()
            for dev in ("cuda", "cpu"):
                try:
                    pg._get_backend(__import__("torch").device(dev)).abort()
                except Exception:  # noqa: BLE001 - backend may not exist / support abort
                    pass
    except Exception:  # noqa: BLE001
        pass
