"""Checkpoint / resume.

Reference (omldm/utils/Checkpointing.scala:11-23, omldm/operators/spoke/
FlinkSpoke.scala:233-334): Flink checkpoints every ``checkInterval`` ms into an
FsStateBackend — spoke state (test set, pipelines, record/request buffers), hub state,
the PipelineMap and Kafka offsets; restore merges list state but loses the spoke
pipelines.

Here every rank writes ``<stateBackend>/ckpt-<n>/rank-<r>.pt`` (tensors moved to host
first, so the GPU stream is not held), and rank 0 writes ``manifest.json`` after a
barrier (so a manifest only exists for complete checkpoints). Everything is restored,
including the pipelines (Q1 fixed). A checkpoint taken with G ranks restores on G' ranks
(``rescale_owners``): new rank r OWNS old ranks {o : o mod G' = r} and takes over exactly
their per-rank data — record buffers concatenated, holdout rings merged in FIFO order
(rows beyond the ring are trained on, as the reference's restore does,
FlinkSpoke.scala:307-317), running counters summed — so no record is trained twice or
lost and Σ-over-ranks metrics are preserved. Models and protocol state come from old
rank r mod G (replicas agree after a sync; GM/FGM estimates are identical everywhere).
Files are loaded with ``weights_only=True``.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import time

import torch


def _root(state_backend: str) -> str:
    if state_backend.startswith("file://"):
        return state_backend[len("file://"):]
    if "://" in state_backend:
        raise ValueError(f"unsupported state backend {state_backend!r} (use file://)")
    return state_backend


def rescale_owners(old_world: int, new_world: int, rank: int) -> list[int]:
    """Old ranks whose per-rank data (record buffer, holdout, counters) new rank ``rank``
    takes over on a restore at a different world size: every old rank has exactly one
    new owner (o mod new_world), so shrinking merges and growing leaves the extra new
    ranks empty."""
    return [o for o in range(old_world) if o % new_world == rank]


class Checkpointer:
    KEEP = 3

    def __init__(self, cfg, rank: int, world: int):
        self.root = _root(cfg.stateBackend)
        self.interval = cfg.checkInterval / 1000.0
        self.rank, self.world = rank, world
        self.last = time.time()
        os.makedirs(self.root, exist_ok=True)
        self.n = self._latest_index() + 1

    def _latest_index(self) -> int:
        best = -1
        for m in glob.glob(os.path.join(self.root, "ckpt-*", "manifest.json")):
            try:
                best = max(best, int(os.path.basename(os.path.dirname(m)).split("-")[1]))
            except ValueError:
                pass
        return best

    def due(self) -> bool:
        return time.time() - self.last >= self.interval

    def save(self, job) -> str:
        d = os.path.join(self.root, f"ckpt-{self.n:06d}")
        os.makedirs(d, exist_ok=True)
        sd = job.state_dict()
        tmp = os.path.join(d, f".rank-{self.rank}.pt.tmp")
        torch.save(sd, tmp)
        os.replace(tmp, os.path.join(d, f"rank-{self.rank}.pt"))
        job.comm.barrier()
        if self.rank == 0:
            with open(os.path.join(d, "manifest.json"), "w") as f:
                json.dump({"index": self.n, "world": self.world, "time": time.time(),
                           "ticks": job.ticks, "pipelines": sorted(job.pipes)}, f)
            old = sorted(glob.glob(os.path.join(self.root, "ckpt-*")))[:-self.KEEP]
            for o in old:
                shutil.rmtree(o, ignore_errors=True)
        job.comm.barrier()
        self.n += 1
        self.last = time.time()
        return d

    def restore(self, job) -> bool:
        idx = self._latest_index()
        if idx < 0:
            return False
        d = os.path.join(self.root, f"ckpt-{idx:06d}")
        with open(os.path.join(d, "manifest.json")) as f:
            man = json.load(f)
        old_world = int(man["world"])
        src = self.rank % old_world

        def load(r):
            return torch.load(os.path.join(d, f"rank-{r}.pt"), map_location="cpu",
                              weights_only=True)

        sd = load(src)
        if old_world == self.world:
            job.load_state_dict(sd, same_world=True)
        else:
            # Re-scaled restore: partition ownership changes, so gather every old rank's
            # consumer offsets (each partition had exactly one owner) and let the new
            # owners resume from them; the per-rank data of the old ranks this rank owns
            # (buffers, holdout, counters) moves here and nowhere else.
            offsets = {"train": {}, "forecast": {}}
            owned = []
            mine = set(rescale_owners(old_world, self.world, self.rank))
            for r in range(old_world):
                o = sd if r == src else load(r)
                for k in offsets:
                    offsets[k].update(o["consumers"][k].get("offsets", {}))
                if r in mine:
                    owned.append(o)
            job.load_state_dict(sd, same_world=False, consumer_offsets=offsets, owned=owned)
        self.n = idx + 1
        return True
