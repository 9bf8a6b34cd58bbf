"""The eight worker↔parameter-server synchronisation protocols, on RCCL collectives.

Reference: MLNodeGenerator maps ``trainingConfiguration.protocol`` to a (worker, PS) pair —
CentralizedTraining, SingleLearner, Asynchronous, Synchronous, SSP, EASGD, GM, FGM —
falling back to Asynchronous when missing/unknown
(omldm/utils/generators/MLNodeGenerator.scala:20-76; algorithms: SURVEY.md Appendix E).

MI355X mapping. A *worker* is one GPU rank; inside a rank the learner's virtual spokes
are merged every round on the GPU (cheap, in HBM), so only the rank-level model crosses
xGMI. Every protocol is written so that all ranks issue the same collectives in the same
order (the decision logic of the "hub" is replicated on every rank from reduced values),
which is what lets a PS be a collective instead of a server process:

* Synchronous — BSP round: the round delta (fused into the learner's kernel accumulator
  when the learner supports it) is summed by one all-reduce (H>1) or reduce+bcast (H=1).
* Asynchronous — point-to-point, no barrier: a worker pushes its local progress δ to
  the hub shard owners (non-blocking isend) and installs the hub's unicast reply when it
  arrives; a slow worker never stops a fast one (parallel/p2p.py).
* SSP — the same channels; the hub withholds a worker's reply while its clock leads the
  slowest worker's by more than ``staleness``.
* EASGD — elastic averaging toward a centre variable every ``tau`` rounds.
* GM — geometric monitoring: sync only when some local drift ‖w_i − E‖² leaves the safe
  zone (an 8-byte max-reduction per round decides, on the device).
* FGM — functional geometric monitoring with rounds/subrounds: a 16-byte sum-reduction of
  (counter increment, φ) per local round, worker and hub logic on the device; a full
  model sync only at round end. GM/FGM read their decision one round late (no host sync
  inside a round).
* CentralizedTraining — one worker, no communication.
* SingleLearner — workers forward their points to the hub rank (0), which alone trains
  (HT, K-means); the hub model is broadcast back for serving.

``merge_mode`` of the learner selects averaging ("mean") or summing ("sum") of worker
increments — additive sufficient statistics (ORR, K-means) must be summed.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.models.base import Learner, RoundContext
from omldm_amd.ops import merge as M
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.p2p import AsyncPS


@dataclass
class ProtocolStatistics:
    protocol: str
    models_shipped: int = 0
    bytes_shipped: int = 0
    num_of_blocks: int = 0
    syncs: int = 0
    rounds: int = 0
    small_messages: int = 0
    # per hub shard [models, bytes, blocks] — what each of the H hubs of the reference
    # counts for its own shard (FlinkHub.scala:118-127), merged by the reference rule
    hubs: list | None = None

    def as_dict(self) -> dict:
        return {"protocol": self.protocol, "modelsShipped": self.models_shipped,
                "bytesShipped": self.bytes_shipped, "numOfBlocks": self.num_of_blocks,
                "syncs": self.syncs, "rounds": self.rounds, "smallMessages": self.small_messages}


def _cfg_int(cfg, k, d):
    try:
        return int(cfg.get(k, d))
    except (TypeError, ValueError):
        return d


def _cfg_float(cfg, k, d):
    try:
        return float(cfg.get(k, d))
    except (TypeError, ValueError):
        return d


class Protocol:
    NAME = "Protocol"

    def __init__(self, comm: Comm, learner: Learner, cfg: dict | None = None,
                 spokes: int = 1, max_msg_params: int = 10000):
        self.comm = comm
        self.learner = learner
        self.cfg = dict(cfg or {})
        self.spokes = max(1, int(self.cfg.get("virtualSpokes", spokes)))
        self.hubs = _cfg_int(self.cfg, "HubParallelism", 0 if comm.world > 1 else 1)
        self.max_msg_params = max(1, int(max_msg_params))
        self.stats = ProtocolStatistics(self.NAME)
        self.G = comm.world

    # --------------------------------------------------------------- helpers
    def _ctx(self, fused: bool = False) -> RoundContext:
        return RoundContext(spokes=self.spokes, inv_p=1.0, fused_delta=fused)

    def n_hubs(self) -> int:
        """Parameter-server shards of this pipeline: HubParallelism, every rank when 0."""
        return max(1, min(self.G, self.hubs if self.hubs > 0 else self.G))

    def _account_model_sync(self, nparams: int, nbytes: int) -> None:
        """Every worker pushes one model to the hub(s) and pulls one back: hub h of H sees
        2G messages of its shard, in ⌈shard/maxMsgParams⌉ blocks each."""
        g, H = self.G, self.n_hubs()
        self.stats.syncs += 1
        self.stats.models_shipped += 2 * g
        self.stats.bytes_shipped += 2 * g * nbytes
        self.stats.num_of_blocks += 2 * g * max(1, math.ceil(nparams / self.max_msg_params))
        if self.stats.hubs is None or len(self.stats.hubs) != H:
            self.stats.hubs = [[0, 0, 0] for _ in range(H)]
        step = -(-max(1, nparams) // H)
        for h in range(H):
            shard = max(0, min(nparams, (h + 1) * step) - h * step)
            hs = self.stats.hubs[h]
            hs[0] += 2 * g
            hs[1] += 2 * g * (nbytes * shard // max(1, nparams))
            hs[2] += 2 * g * max(1, math.ceil(shard / self.max_msg_params))

    def hub_statistics(self) -> list[dict]:
        """One statistics record per hub shard (models, bytes, blocks)."""
        if not self.stats.hubs:
            return [{"modelsShipped": self.stats.models_shipped,
                     "bytesShipped": self.stats.bytes_shipped,
                     "numOfBlocks": self.stats.num_of_blocks}]
        return [{"modelsShipped": m, "bytesShipped": b, "numOfBlocks": k}
                for m, b, k in self.stats.hubs]

    def _small(self, vals: list) -> torch.Tensor:
        """A few fp32 scalars for a small collective, on the device the backend reduces
        (RCCL: the learner's GPU; gloo: host)."""
        dev = self.learner.device if self.comm.backend == "nccl" else "cpu"
        return torch.tensor(vals, dtype=torch.float32, device=dev)

    def _account_small(self, n_msgs: int, nbytes: int) -> None:
        self.stats.small_messages += n_msgs
        self.stats.bytes_shipped += n_msgs * nbytes

    def _scale(self) -> float:
        """Factor turning the reduced SUM of worker increments into the global increment."""
        return 1.0 if self.learner.merge_mode == "sum" else 1.0 / self.G

    # --------------------------------------------------------------- API
    def round(self, batch: HashedBatch) -> None:
        raise NotImplementedError

    def finalize(self) -> None:
        """Drain in-flight communication (end of stream / before a query or checkpoint)."""

    def state_dict(self) -> dict:
        return {"stats": self.stats.__dict__.copy()}

    def load_state_dict(self, sd: dict) -> None:
        for k, v in sd.get("stats", {}).items():
            setattr(self.stats, k, v)


class CentralizedTraining(Protocol):
    NAME = "CentralizedTraining"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if "virtualSpokes" not in self.cfg:
            self.spokes = 1  # P == 1: one exact sequential learner

    def round(self, batch):
        self.learner.fit(batch, self._ctx())
        self.stats.rounds += 1


class Synchronous(Protocol):
    NAME = "Synchronous"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._E = None
        # > 1: pipelined sync — the learner's delta reduce runs in that many key-range
        # launches and each range's all-reduce starts as soon as its launch is enqueued
        # (RCCL works on range k while the GPU reduces range k+1). Same sums, same
        # collectives on every rank; only with every rank a hub (all-reduce).
        self.reduce_parts = max(1, _cfg_int(self.cfg, "reduceParts", 1))
        # benchmarks: CUDA events around every round's collective (collective_time_ms)
        self.time_collectives = False
        self._coll_events: list = []

    # The round is split in two so the engine can coalesce the collectives of several
    # pipelines into one bucket: local() trains and returns the buffer to
    # sum over ranks, finish() consumes the reduced buffer.
    def local(self, batch) -> torch.Tensor:
        L = self.learner
        if L.supports_fused_delta:
            # Fast path: the kernel leaves Σ σ·Δ (+ counters) of every local spoke in the
            # learner's accumulator; one collective sums it over ranks; apply averages.
            L.fit(batch, self._ctx(fused=True))
            self._buf = L.delta_buffer()
        else:
            if self._E is None:
                self._E = L.state_vector().detach().clone()
            if getattr(self, "_d", None) is None or self._d.shape != self._E.shape:
                self._d = torch.empty_like(self._E)  # also after a restore (E loaded)
            L.fit(batch, self._ctx())
            self._buf = torch.sub(L.state_vector(), self._E, out=self._d)
        return self._buf

    def local_done(self) -> torch.Tensor:
        """Phase 1 when the learner's round already ran (a fused multi-pipeline launch,
        engine/job.py): the buffer to sum over ranks."""
        assert self.learner.supports_fused_delta
        self._buf = self.learner.delta_buffer()
        return self._buf

    def fusable(self) -> bool:
        """This round may run inside a multi-pipeline launch (a v3 launch: its accumulator is
        final only at the round end, so a reduceParts split never applies there)."""
        return self.learner.supports_fused_delta

    def finish(self, applied: bool = False) -> None:
        """Phase 2: the summed buffer into the model (``applied``: ``finish_group`` already
        averaged this learner's delta in its shared launch)."""
        L, buf = self.learner, self._buf
        if L.supports_fused_delta:
            if not applied:
                L.apply_delta()
        else:
            M.fold_reload(self._E, buf, self._scale(), L.state_vector())  # E += s·Σd ; x = E
            L.on_state_loaded()
        self._account_model_sync(L.num_params(), buf.numel() * buf.element_size())
        self._buf = None
        self.stats.rounds += 1

    @staticmethod
    def finish_group(protos: list) -> None:
        """``finish`` of several Synchronous pipelines; the hashed-linear models among them
        are averaged in ONE launch (ops.linear.linear_apply_multi; BASELINE config 5: 16
        apply launches and their gaps were ~85 µs of a 16-pipeline step)."""
        from omldm_amd.models.linear import LinearLearner

        lin = [p for p in protos if isinstance(p.learner, LinearLearner)
               and p.learner.supports_fused_delta]
        if len(lin) > 1:
            LinearLearner.apply_delta_group([p.learner for p in lin])
        done = {id(p) for p in lin} if len(lin) > 1 else set()
        for p in protos:
            p.finish(applied=id(p) in done)

    def _pipelined(self, batch) -> bool:
        L = self.learner
        return (self.reduce_parts > 1 and self.G > 1 and L.supports_fused_delta
                and L.supports_reduce_parts and (self.hubs == 0 or self.hubs >= self.G)
                and L.reduce_parts_apply(batch, self._ctx(fused=True)))

    def round(self, batch):
        if self._pipelined(batch):
            L, works = self.learner, []
            buf = L.delta_buffer()

            def on_part(k: int, lo: int, hi: int) -> None:
                if hi > lo:
                    works.append(self.comm.all_reduce_(buf[lo:hi], "sync", async_op=True))

            ctx = self._ctx(fused=True)
            ctx.reduce_parts, ctx.on_reduce_part = self.reduce_parts, on_part
            L.fit(batch, ctx)
            for w in works:
                if w is not None:
                    w.wait()  # the compute stream waits for RCCL; the host does not block
            self._buf = buf
            self.finish()
            return
        buf = self.local(batch)
        if self.time_collectives and buf.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.comm.hub_reduce_(buf, self.hubs, tag="sync")
            e1.record()
            self._coll_events.append((e0, e1))
        else:
            self.comm.hub_reduce_(buf, self.hubs, tag="sync")
        self.finish()

    def collective_time_ms(self) -> float:
        """Device time of the collectives timed since the last call (synchronises)."""
        if not self._coll_events:
            return 0.0
        self._coll_events[-1][1].synchronize()
        t = sum(a.elapsed_time(b) for a, b in self._coll_events)
        self._coll_events.clear()
        return t

    def state_dict(self):
        sd = super().state_dict()
        sd["E"] = None if self._E is None else self._E.cpu()
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        if sd.get("E") is not None:
            self._E = sd["E"].to(self.learner.device)


class _PointToPoint(Protocol):
    """Shared machinery of Asynchronous and SSP: every worker's round ends with a
    non-blocking push of its local progress to the hub shard owners and the install of
    whatever reply has arrived (parallel/p2p.py: AsyncPS). No collective per round."""

    staleness: int | None = None

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._ps = None
        self.tag = _cfg_int(self.cfg, "_tag", 0)

    def _make(self):
        x = self.learner.state_vector()
        hubs = self.hubs if self.hubs > 0 else 1
        self._ps = AsyncPS(self.comm, x.numel(), x.dtype, hubs, self.tag, self.staleness,
                           self._scale())
        self._ps.init(x)

    def round(self, batch):
        L = self.learner
        if self.comm.world > 1 and self._ps is None:
            self._make()  # every rank starts from the same (initial / restored) model
        L.fit(batch, self._ctx())
        self.stats.rounds += 1
        if self._ps is None:
            return  # one worker: its local model IS the global model
        x = L.state_vector()
        installs = self._ps.installs
        pushed = self._ps.step(x)
        if pushed:
            self._count_pushes(1, x)
        # the signal plane decides installs on the device (pushed is None): derived state
        # is refreshed every round
        if pushed is None or self._ps.installs != installs:
            L.on_state_loaded()

    def _count_pushes(self, k: int, x) -> None:
        nbytes = x.numel() * x.element_size()
        self.stats.syncs += k
        self.stats.models_shipped += 2 * k  # one push, one reply (unicast)
        self.stats.bytes_shipped += 2 * k * nbytes
        self.stats.num_of_blocks += 2 * k * max(1, math.ceil(x.numel() / self.max_msg_params))

    @property
    def max_lead(self) -> int:
        return self._ps.max_lead if self._ps is not None else 0

    def finalize(self):
        if self._ps is not None and self.comm.world > 1:
            x = self.learner.state_vector()
            self._ps.finalize(x)
            self._count_pushes(self._ps.take_unreported_pushes(), x)
            self.learner.on_state_loaded()

    def state_dict(self):
        self.finalize()
        return super().state_dict()

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        if self._ps is not None:
            self._ps.close()
        self._ps = None  # re-seeded from the restored model at the next round


class Asynchronous(_PointToPoint):
    NAME = "Asynchronous"
    staleness = None


class SSP(_PointToPoint):
    NAME = "SSP"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.staleness = max(0, _cfg_int(self.cfg, "staleness", 2))


class EASGD(Protocol):
    NAME = "EASGD"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.tau = max(1, _cfg_int(self.cfg, "tau", 1))
        self.alpha = _cfg_float(self.cfg, "alpha", 0.9 / max(1, self.G))
        self._c = None
        self._diff = self._s = None
        self._k = 0

    def round(self, batch):
        L = self.learner
        if self._c is None:
            self._c = L.state_vector().detach().clone()
        if self._s is None or self._s.shape != self._c.shape:  # also after a restore
            self._diff, self._s = torch.empty_like(self._c), torch.empty_like(self._c)
        L.fit(batch, self._ctx())
        self._k += 1
        if self._k % self.tau == 0:
            x = L.state_vector()
            s = self._s
            M.elastic_pre(x, self._c, self._diff, s)        # diff = s = x_i − c
            self.comm.all_reduce_(s, tag="elastic")
            # x_i ← x_i − α(x_i − c) ; c ← c + α Σ_i (x_i − c)
            M.elastic_post(x, self._c, self._diff, s, self.alpha)
            L.on_state_loaded()
            self._account_model_sync(L.num_params(), s.numel() * s.element_size())
        self.stats.rounds += 1

    def state_dict(self):
        sd = super().state_dict()
        sd["center"] = None if self._c is None else self._c.cpu()
        sd["k"] = self._k
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        if sd.get("center") is not None:
            self._c = sd["center"].to(self.learner.device)
        self._k = int(sd.get("k", 0))


def _model_sync(p: Protocol) -> None:
    """Full model sync of GM / FGM: every worker ships its drift (×G for additive state),
    the sum is folded into the estimate E and every worker reloads E."""
    L = p.learner
    x = L.state_vector()
    if getattr(p, "_d", None) is None or p._d.shape != x.shape:
        p._d = torch.empty_like(x)
    d = torch.sub(x, p._E, out=p._d)
    if L.merge_mode == "sum":
        d.mul_(p.G)
    p.comm.all_reduce_(d, tag="sync")
    M.fold_reload(p._E, d, 1.0 / p.G, x)
    L.on_state_loaded()
    p._account_model_sync(L.num_params(), d.numel() * d.element_size())


class _LaggedDecision:
    """A device-computed sync decision read by the host one round later.

    The monitor writes its (reduced) decision into a device scalar and ``post`` starts a
    non-blocking copy into pinned host memory behind it. ``take`` — called after the next
    round's training kernels are enqueued — waits only for that copy, so the GPU always
    has the next round queued while the host decides: no drain of the stream inside a
    round. Every rank reduces the same flag, so every rank takes the same decision at the
    same round and issues the same collectives."""

    def __init__(self, device):
        self.dev = torch.zeros(1, dtype=torch.float64, device=device)
        cuda = self.dev.is_cuda
        self.host = torch.zeros(1, dtype=torch.float64, pin_memory=cuda)
        self._event = None
        self.pending: float | None = None  # a decision restored from a checkpoint

    def post(self) -> None:
        if self.dev.is_cuda:
            self.host.copy_(self.dev, non_blocking=True)
            self._event = torch.cuda.Event()
            self._event.record()
        else:
            self.host.copy_(self.dev)
            self._event = True

    def take(self) -> float | None:
        if self.pending is not None:
            v, self.pending = self.pending, None
            return v
        if self._event is None:
            return None
        if self._event is not True:
            self._event.synchronize()
        self._event = None
        return float(self.host[0])

    def peek_for_checkpoint(self) -> float | None:
        """The outstanding decision, kept outstanding (a checkpoint must not change the
        trajectory)."""
        v = self.take()
        self.pending = v
        return v


class _Monitored(Protocol):
    """GM / FGM machinery: the estimate E, the lagged decision and the reduction of the
    per-round monitoring message (RCCL on the device; over gloo through host memory)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._E = None
        self._lag = None
        self._nrm = None
        self._msg = None

    def _buffers(self, nmsg: int):
        if self._lag is None:
            dev = self.learner.device
            self._lag = _LaggedDecision(dev)
            self._nrm = torch.zeros(2, dtype=torch.float32, device=dev)
            self._msg = torch.zeros(nmsg, dtype=torch.float64, device=dev)

    def _reduce_msg(self, tag: str, op=None) -> None:
        if self.G > 1:
            m = self._msg
            if self.comm.backend == "nccl" or not m.is_cuda:
                self.comm.all_reduce_(m, tag=tag, op=op)
            else:  # gloo rehearsal with device tensors: through host memory
                h = m.cpu()
                self.comm.all_reduce_(h, tag=tag, op=op)
                m.copy_(h)
        self._account_small(self.G, self._msg.numel() * self._msg.element_size())

    def _full_sync(self):
        _model_sync(self)

    def finalize(self):
        """End of stream / query / checkpoint: a sync that is due is carried out now."""
        if self._lag is not None and self._E is not None:
            v = self._lag.take()
            if v:
                self._full_sync()
                self._after_sync()

    def _after_sync(self) -> None:
        pass

    # E is identical on every rank (it only changes in a full sync) while the local
    # models differ by their unsynced drifts: E must be checkpointed, or a restored rank
    # would re-seed it from its own model and the replicas would never agree again.
    def state_dict(self):
        sd = super().state_dict()
        sd["E"] = None if self._E is None else self._E.cpu()
        sd["pending"] = None if self._lag is None else self._lag.peek_for_checkpoint()
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        if sd.get("E") is not None:
            self._E = sd["E"].to(self.learner.device)
        self._lag = None
        if sd.get("pending") is not None:
            self._buffers(self.NMSG)
            self._lag.pending = float(sd["pending"])


class GM(_Monitored):
    """Geometric monitoring: a worker leaves the safe zone when ‖X_i‖² > θ·‖E‖²; one
    8-byte max-reduction per round; the decision is taken on the device and read by the
    host one round later (the sync happens after the round following the violation)."""

    NAME = "GM"
    NMSG = 1

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.threshold = _cfg_float(self.cfg, "threshold", 0.05)

    def round(self, batch):
        L = self.learner
        if self._E is None:
            self._E = L.state_vector().detach().clone()
        self._buffers(self.NMSG)
        L.fit(batch, self._ctx())
        if self._lag.take():
            self._full_sync()  # x = E: no drift left to monitor this round
        else:
            x = L.state_vector()
            scale = self.G if L.merge_mode == "sum" else 1.0
            M.drift_norms(x, self._E, scale, out=self._nrm)   # [‖X_i‖², ‖E‖²], one pass
            M.gm_local(self._nrm, self.threshold, self._msg)   # safe-zone test, on device
            self._reduce_msg("gm-flag", op=torch.distributed.ReduceOp.MAX)
            self._lag.dev.copy_(self._msg[:1])
            self._lag.post()
        self.stats.rounds += 1


class FGM(_Monitored):
    """Functional Geometric Monitoring (variance safe function).

    Safe function on a worker's drift X_i (state − E, scaled by G for additive state):
        φ(X) = ‖X‖² − ε‖E‖²          (φ(0) = −ε‖E‖² < 0 while E ≠ 0)
    round start: ψ = G·φ(0), quantum θ = −ψ / (2G);
    subround: worker counter c_i = ⌊(φ(X_i) − φ(0)) / θ⌋, the hub sums increments;
    when Σ c_i > G the hub collects ψ = Σ φ(X_i): if ψ ≥ ε_ψ·G·φ(0) the round ends with
    a full model sync, otherwise a new subround starts with θ = −ψ / (2G).
    The worker and the (replicated) hub logic run on the device (merge.hip fgm_*_kernel)
    around one 16-byte all-reduce per local round ((Δc_i, φ_i)); only the full-sync
    decision reaches the host, one round late (_LaggedDecision), so only round ends move
    models over xGMI and no round drains the stream.
    """

    NAME = "FGM"
    NMSG = 2

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.eps = _cfg_float(self.cfg, "epsilon", 0.05)
        self.eps_psi = _cfg_float(self.cfg, "epsilonPsi", 0.01)
        self._st = None
        self.fgm_rounds = 0

    def _begin_round(self):
        L = self.learner
        x = L.state_vector()
        if self._E is None:
            self._E = x.detach().clone()
        M.drift_norms(x, self._E, 1.0, out=self._nrm)  # [·, ‖E‖²]
        M.fgm_begin(self._nrm, self._st, self.eps)
        self.fgm_rounds += 1

    def _after_sync(self):
        self._begin_round()

    @property
    def subrounds(self) -> int:
        return 0 if self._st is None else int(self._st[6].item())

    def round(self, batch):
        L = self.learner
        self._buffers(self.NMSG)
        if self._st is None:
            self._st = torch.zeros(8, dtype=torch.float64, device=L.device)
            self._begin_round()
        L.fit(batch, self._ctx())
        if self._lag.take():
            self._full_sync()
            self._begin_round()
        else:
            x = L.state_vector()
            scale = self.G if L.merge_mode == "sum" else 1.0
            M.drift_norms(x, self._E, scale, out=self._nrm)
            M.fgm_local(self._nrm, self._st, self.eps, self._msg)
            self._reduce_msg("fgm-counters")
            M.fgm_hub(self._st, self._msg, self.eps_psi, self.G, self._lag.dev)
            self._lag.post()
        self.stats.rounds += 1

    def state_dict(self):
        """The round/subround state is the hub's (identical on every rank) plus this
        worker's counter; E is the estimate every local drift is measured against."""
        sd = super().state_dict()
        sd["fgm"] = {"state": None if self._st is None else self._st.cpu(),
                     "fgm_rounds": self.fgm_rounds}
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        f = sd.get("fgm")
        if f and f.get("state") is not None:
            self._buffers(self.NMSG)
            self._st = f["state"].to(self.learner.device)
            self.fgm_rounds = int(f["fgm_rounds"])


class SingleLearner(Protocol):
    """Workers forward training points to the hub rank, which alone trains (HT, K-means);
    reference: ForwardingWorker + CentralizedMLServer (MLNodeGenerator.scala:27,56).

    The other ranks keep a replica only to serve forecasts and queries: the hub model is
    broadcast every ``broadcastEvery`` rounds (default 8) and whenever the replicas are
    read collectively — before a query, a checkpoint or the end of the stream
    (``finalize``) — instead of G× the model bytes every round. Forecasts on a non-hub
    rank may therefore lag the hub by up to ``broadcastEvery`` − 1 rounds."""

    NAME = "SingleLearner"
    HUB = 0

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.every = max(1, _cfg_int(self.cfg, "broadcastEvery", 8))
        self._stale = 0  # rounds since the replicas last received the hub model

    def _broadcast(self) -> None:
        L = self.learner
        v = L.state_vector()
        self.comm.broadcast_(v, src=self.HUB)
        L.on_state_loaded()
        self._account_model_sync(L.num_params(), v.numel() * v.element_size())
        self._stale = 0

    def finalize(self) -> None:
        if self.G > 1 and self._stale:
            self._broadcast()

    def state_dict(self):
        self.finalize()
        return super().state_dict()

    def round(self, batch):
        L = self.learner
        parts = {}
        for name in ("num", "cat", "y"):
            parts[name] = self.comm.gather_tensor(getattr(batch, name).contiguous(), dst=self.HUB)
        if self.comm.rank == self.HUB:
            # same batch kind and wire as the local one (cat_span, a fused PolyBatch's pairs)
            merged = batch._like(torch.cat(parts["num"]), torch.cat(parts["cat"]),
                                 torch.cat(parts["y"]), None)
            L.fit(merged, RoundContext(spokes=1))
        self._account_small(self.G, batch.B)  # forwarded points
        self.stats.rounds += 1
        if self.G > 1:  # hub → replicas, every `every` rounds (finalize: on demand)
            self._stale += 1
            if self._stale >= self.every:
                self._broadcast()


PROTOCOLS = {c.NAME: c for c in (CentralizedTraining, Synchronous, Asynchronous, SSP, EASGD, GM,
                                 FGM, SingleLearner)}


def make_protocol(name: str | None, comm: Comm, learner: Learner, cfg: dict | None = None,
                  spokes: int = 1, max_msg_params: int = 10000) -> Protocol:
    """Reference fallback rule: unknown or missing protocol → Asynchronous
    (omldm/utils/generators/MLNodeGenerator.scala:26-38)."""
    cls = PROTOCOLS.get(name or "", Asynchronous)
    return cls(comm, learner, cfg, spokes=spokes, max_msg_params=max_msg_params)
