"""Checkpoint / resume.

Reference (omldm/utils/Checkpointing.scala:11-23, omldm/operators/spoke/
FlinkSpoke.scala:233-334): Flink checkpoints every ``checkInterval`` ms into an
FsStateBackend — spoke state (test set, pipelines, record/request buffers), hub state,
the PipelineMap and Kafka offsets; restore merges list state but loses the spoke
pipelines.

Here every rank snapshots its state at the same tick (rank 0's clock decides, carried in
the tick's control flags), copies it to host and hands it to a writer thread: the tick
goes on while ``<stateBackend>/ckpt-<n>/rank-<r>.pt`` is written, then a ``rank-<r>.done``
marker. Rank 0's writer also exports every pipeline in the reference's portable model
format (``models.json``: one Create request per pipeline whose ``learner.parameters`` are
the QueryResponse learner map — what ``python -m omldm_amd.tools import-models`` replays
into any job) and writes ``manifest.json`` — versioned (``format``/``version``) — only
once every rank's marker exists, so a manifest only exists for complete checkpoints. No
barrier or file I/O sits in the tick. Everything is restored, including the pipelines
(Q1 fixed). A checkpoint taken with G ranks restores on G' ranks
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
import threading
import time
import uuid

import torch

FORMAT = "omldm-amd-checkpoint"
VERSION = 2  # 1: round-2 manifests (no format field); 2: + models.json export, done markers


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
    WAIT_S = 600.0  # rank 0's writer waits this long for the other ranks' files

    def __init__(self, cfg, rank: int, world: int, nonce: str | None = None):
        self.root = _root(cfg.stateBackend)
        # one value per job run (rank 0's, broadcast by the Job): a done marker an earlier
        # process left at the same index and tick can never match this run's attempt tag
        self.nonce = nonce or uuid.uuid4().hex
        self.interval = cfg.checkInterval / 1000.0
        self.rank, self.world = rank, world
        self.export = bool(getattr(cfg, "checkpointExport", True))
        self.last = time.time()
        os.makedirs(self.root, exist_ok=True)
        self.n = self._latest_index() + 1
        self._writer: threading.Thread | None = None
        self.errors: list = []
        self.completed = 0  # manifests this rank's writer published (rank 0)

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
        """Snapshot now (host copies), write in the background. At most one write per
        rank is in flight: a new snapshot first waits for the previous write."""
        d = os.path.join(self.root, f"ckpt-{self.n:06d}")
        # host copies taken HERE, on the tick's thread: live tensors (scaler statistics,
        # the holdout ring, models) keep changing in place after this returns
        sd = host_copy(job.state_dict())
        models = export_models(job) if (self.rank == 0 and self.export) else None
        meta = {"format": FORMAT, "version": VERSION, "index": self.n, "world": self.world,
                "time": time.time(), "ticks": job.ticks, "pipelines": sorted(job.pipes),
                "files": [f"rank-{r}.pt" for r in range(self.world)],
                "models": "models.json" if models is not None else None}
        # every rank saves at the same tick (rank 0's clock, carried in the tick flags):
        # the marker names the attempt, so files a crashed earlier attempt left in this
        # directory never complete the manifest
        meta["attempt"] = f"{self.nonce}:{self.n}:{job.ticks}"
        self.wait()
        self._writer = threading.Thread(target=self._write, args=(d, sd, models, meta),
                                         name=f"omldm-ckpt-{self.n}", daemon=True)
        self._writer.start()
        self.n += 1
        self.last = time.time()
        return d

    def _write(self, d: str, sd: dict, models, meta: dict) -> None:
        try:
            os.makedirs(d, exist_ok=True)
            done = os.path.join(d, f"rank-{self.rank}.done")
            if os.path.exists(done):  # left by a crashed attempt at this index
                os.remove(done)
            tmp = os.path.join(d, f".rank-{self.rank}.pt.tmp")
            torch.save(sd, tmp)
            os.replace(tmp, os.path.join(d, f"rank-{self.rank}.pt"))
            _atomic_text(done, meta["attempt"])
            if self.rank != 0:
                return
            if models is not None:
                _atomic_json(os.path.join(d, "models.json"), models)
            t0 = time.time()
            while not all(_read_text(os.path.join(d, f"rank-{r}.done")) == meta["attempt"]
                          for r in range(self.world)):
                if time.time() - t0 > self.WAIT_S:
                    raise TimeoutError(f"checkpoint {d}: ranks did not finish their files")
                time.sleep(0.01)
            _atomic_json(os.path.join(d, "manifest.json"), meta)
            self.completed += 1
            done = sorted(os.path.dirname(m) for m in
                          glob.glob(os.path.join(self.root, "ckpt-*", "manifest.json")))
            for o in done[:-self.KEEP]:
                shutil.rmtree(o, ignore_errors=True)
        except Exception as e:  # surfaced by wait() / close()
            self.errors.append(e)

    def wait(self) -> None:
        if self._writer is not None:
            self._writer.join()
            self._writer = None
        if self.errors:
            e, self.errors = self.errors[0], []
            raise RuntimeError(f"checkpoint write failed: {e}") from e

    def close(self) -> None:
        self.wait()

    def restore(self, job) -> bool:
        idx = self._latest_index()
        if idx < 0:
            return False
        d = os.path.join(self.root, f"ckpt-{idx:06d}")
        with open(os.path.join(d, "manifest.json")) as f:
            man = json.load(f)
        check_manifest(man)
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


def check_manifest(man: dict) -> int:
    """Version of a checkpoint manifest this build can restore (round-2 manifests carry
    no format field: version 1); anything else is refused with a clear error."""
    fmt = man.get("format", FORMAT)
    ver = int(man.get("version", 1))
    if fmt != FORMAT:
        raise ValueError(f"not an {FORMAT} manifest: format={fmt!r}")
    if ver > VERSION:
        raise ValueError(f"checkpoint version {ver} is newer than this build ({VERSION})")
    for k in ("index", "world"):
        if k not in man:
            raise ValueError(f"checkpoint manifest lacks {k!r}")
    return ver


def host_copy(obj):
    """Deep copy of a state tree with every tensor in fresh host memory."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: host_copy(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [host_copy(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(host_copy(v) for v in obj)
    return obj


def _atomic_text(path: str, text: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


def _read_text(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _atomic_json(path: str, obj) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def export_models(job) -> dict:
    """Every pipeline as the Create request that re-creates it from the reference's
    portable model format: learner {name, hyperParameters, parameters} (the QueryResponse
    learner map, FlinkNetwork.scala:196-230), preprocessors with their parameters, and the
    training configuration. Replayed by ``tools import-models``."""
    out = []
    for pid in sorted(job.pipes):
        p = job.pipes[pid]
        req = p.request.to_obj()
        lrn = p.learner
        hyper = {k: v for k, v in lrn.hyper_parameters().items() if not k.startswith("_")}
        req.update({"id": pid, "request": "Create",
                    "learner": {"name": lrn.NAME, "hyperParameters": hyper,
                                "parameters": lrn.parameters_map()},
                    "preProcessors": [pp.to_obj() for pp in p.preprocessors]})
        out.append({"request": req, "protocol": p.protocol_name,
                    "dataFitted": lrn.running_totals()["fitted"]})
    return {"format": "omldm-amd-models", "version": 1, "pipelines": out}


def import_requests(path: str) -> list[dict]:
    """The Create requests of a ``models.json`` export (see export_models)."""
    with open(path) as f:
        obj = json.load(f)
    if obj.get("format") != "omldm-amd-models":
        raise ValueError(f"{path}: not a model export")
    return [p["request"] for p in obj["pipelines"]]
