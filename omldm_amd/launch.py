"""Single-node supervisor: one process per GPU, restart-from-checkpoint on failure,
optionally on fewer ranks (SURVEY.md §5.3 elastic recovery).

    python -m omldm_amd.launch --nproc 8 [--max-restarts 3] [--min-nproc 4]
                               [--shrink-on-failure] [--master-port 29533] -- <job flags>

Reference: a Flink job with no restart strategy simply fails (omldm/Job.scala:14);
Flink's own JobManager would restore operator state from the FsStateBackend.

Here every attempt spawns ``nproc`` ranks of ``python -m omldm_amd`` (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in the environment — the torchrun
contract). When any rank exits non-zero (crash, injected fault, watchdog abort) the
remaining ranks are terminated, and the job is relaunched with ``--restore true``: the
checkpoint manifest is world-size independent (utils/checkpoint.py), so with
``--shrink-on-failure`` the next attempt may run on one rank fewer (down to
``--min-nproc``), e.g. after losing a GPU. Children are started as ordinary child
processes (never exec'd over a GPU-initialised process) and killed by their own PIDs.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def _spawn(nproc: int, port: int, attempt: int, job_args: list[str], restore: bool):
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc),
                    "LOCAL_WORLD_SIZE": str(nproc), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "OMLDM_ATTEMPT": str(attempt)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        args = [sys.executable, "-m", "omldm_amd", *job_args]
        if restore:
            args += ["--restore", "true"]
        procs.append(subprocess.Popen(args, env=env, start_new_session=True))
    return procs


def _stop(procs, grace: float = 5.0) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < t:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def supervise(nproc: int, job_args: list[str], max_restarts: int = 3, min_nproc: int = 1,
              shrink: bool = False, port: int = 29533, poll_s: float = 0.05,
              log=print) -> int:
    attempt = 0
    while True:
        procs = _spawn(nproc, port + attempt, attempt, job_args, restore=attempt > 0)
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
        if failed is None:
            log(f"[launch] attempt {attempt}: {nproc} ranks finished")
            return 0
        _stop(procs)
        log(f"[launch] attempt {attempt}: rank {failed[0]} exited with {failed[1]}")
        if attempt >= max_restarts:
            return failed[1] if failed[1] > 0 else 1
        attempt += 1
        if shrink and nproc > min_nproc:
            nproc -= 1
        log(f"[launch] restarting from the last checkpoint on {nproc} rank(s)")


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        i = argv.index("--")
        own, job_args = argv[:i], argv[i + 1:]
    else:
        own, job_args = argv, []
    ap = argparse.ArgumentParser(prog="python -m omldm_amd.launch")
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--min-nproc", type=int, default=1)
    ap.add_argument("--shrink-on-failure", action="store_true")
    ap.add_argument("--master-port", type=int, default=29533)
    a = ap.parse_args(own)
    return supervise(a.nproc, job_args, a.max_restarts, a.min_nproc, a.shrink_on_failure,
                     a.master_port)


if __name__ == "__main__":
    sys.exit(main())
