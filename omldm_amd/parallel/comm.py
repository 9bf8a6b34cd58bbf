"""Communication layer: the worker↔hub transport of the reference, on RCCL.

Reference: spokes push model blocks to the hub through a Flink shuffle and the hub
answers through the Kafka ``psMessages`` topic (omldm/network/FlinkNetwork.scala:242-293,
omldm/Job.scala:77-87,136-142) — two network hops plus a broker per sync.
Here one process drives one GPU and the hub is a collective:

* hub parallelism H > 1 (sharded PS)  → ``all_reduce`` (= reduce-scatter + all-gather, RCCL
  ring/direct algorithms over the 7 xGMI links per GPU);
* H == 1 (single hub)                 → ``reduce`` to rank 0 + ``broadcast`` from it;
* many pipelines due in the same round are coalesced into one flat bucket (one launch,
  ≥ MBs, so the collective is bandwidth- rather than latency-bound).

Works with backend ``nccl`` (RCCL on ROCm) on GPUs and ``gloo`` on CPU (tests). The byte
and message counters feed the reference's ``modelsShipped/bytesShipped/numOfBlocks``
statistics (omldm/operators/hub/FlinkHub.scala:118-127).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


# element types RCCL / gloo collectives do not carry (sent as raw bytes instead)
_BYTE_WIRE = (torch.int16, torch.uint16, torch.bool) if hasattr(torch, "uint16") else \
    (torch.int16, torch.bool)


@dataclass
class CommStats:
    collectives: int = 0
    bytes: int = 0
    small_collectives: int = 0
    per_tag: dict = field(default_factory=dict)
    # when a list: every call is appended as (kind, tag, bytes) — the exact per-round
    # communication schedule (tests pin it per protocol)
    trace: list | None = None

    def add(self, tag: str, nbytes: int, small: bool = False, kind: str = "all_reduce"):
        if self.trace is not None:
            self.trace.append((kind, tag, int(nbytes)))
        self.collectives += 1
        self.bytes += nbytes
        if small:
            self.small_collectives += 1
        self.per_tag[tag] = self.per_tag.get(tag, 0) + nbytes


class Comm:
    """World communicator (one rank per GPU)."""

    @classmethod
    def local(cls) -> "Comm":
        """A one-rank communicator even inside a multi-rank job (a rank-local engine,
        e.g. a benchmark's side measurement): no collective ever leaves the process."""
        c = cls.__new__(cls)
        c.group, c.enabled, c.rank, c.world = None, False, 0, 1
        c.stats, c.backend, c.fault, c.placement = CommStats(), "none", None, {}
        c.ctrl_group = None
        return c

    def __init__(self, group=None):
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.stats = CommStats()
        self.backend = dist.get_backend(group) if self.enabled else "none"
        self.fault = None  # utils.fault.FaultPlan (tests): may drop this rank's messages
        self.placement: dict = {}  # NUMA binding of this rank (utils/topology.py)
        # host control plane: tiny per-tick decisions (flags, counters) reduce over gloo on
        # host tensors, so reading them back never waits for the GPU stream (an RCCL
        # all-reduce of a device tensor + .tolist() would drain every queued kernel)
        self.ctrl_group = group
        if self.enabled and self.world > 1 and self.backend != "gloo":
            self.ctrl_group = dist.new_group(backend="gloo")

    # ------------------------------------------------------------ collectives
    def all_reduce_(self, t: torch.Tensor, tag: str = "sync", op=None, async_op=False):
        self.stats.add(tag, t.numel() * t.element_size(), t.numel() <= 64)
        if self.fault is not None and self.fault.drop(tag):
            t.zero_()  # lost message: the rank still joins, its contribution is gone
        if self.world == 1:
            return None
        return dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def all_reduce_host_(self, t: torch.Tensor, tag: str = "heartbeat", op=None):
        """SUM (or ``op``) of a small HOST tensor over the control group (gloo): no device
        synchronisation."""
        assert not t.is_cuda
        self.stats.add(tag, t.numel() * t.element_size(), True, kind="host_all_reduce")
        if self.world == 1:
            return
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.ctrl_group)

    def reduce_bcast_(self, t: torch.Tensor, root: int = 0, tag: str = "sync"):
        """Single-hub semantics (HubParallelism == 1): reduce to root, root broadcasts."""
        self.stats.add(tag, 2 * t.numel() * t.element_size(), kind="reduce+bcast")
        if self.world == 1:
            return
        dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, group=self.group)
        dist.broadcast(t, src=root, group=self.group)

    def hub_reduce_(self, t: torch.Tensor, hubs: int = 0, tag: str = "sync"):
        """Sum ``t`` over workers through ``hubs`` parameter-server shards.
        hubs == 1: one hub (rank 0) — reduce + broadcast;
        1 < hubs < world: hub h (rank h) owns the h-th contiguous slice — every worker pushes
        each slice to its hub and pulls the summed slice back, point-to-point (the
        reference's sharded PS, FlinkHub keyed ``net_hubIdx``; _sharded_ps_);
        hubs == 0 or ≥ world: every rank is a hub — all-reduce (reduce-scatter +
        all-gather inside RCCL)."""
        if self.world == 1:
            self.all_reduce_(t, tag)
        elif hubs == 1:
            self.reduce_bcast_(t, 0, tag)
        elif 1 < hubs < self.world:
            self._sharded_ps_(t, hubs, tag)
        else:
            self.all_reduce_(t, tag)

    def _sharded_ps_(self, t: torch.Tensor, hubs: int, tag: str) -> None:
        """1 < H < G parameter-server shards over point-to-point channels: phase 1 every
        rank sends slice h to hub h (all sends/receives of the phase are posted at once,
        so on a node they run concurrently over the direct xGMI links — a hub receives
        its G−1 slices on G−1 different links), the hub sums them in rank order; phase 2
        each hub sends its summed slice back to every rank. Per rank ≈ 2·n elements cross
        the wire, the same as a ring all-reduce, in two latency steps instead of the 2H
        serialised reduce/broadcast collectives."""
        flat = t.view(-1)
        n = flat.numel()
        step = -(-n // hubs)
        sl = [flat[h * step:min(n, (h + 1) * step)] for h in range(hubs)]
        me, G = self.rank, self.world
        self.stats.add(tag, 2 * n * t.element_size(), kind="p2p_shards")
        bufs = {}
        ops = []
        for h in range(hubs):
            if h != me and sl[h].numel():
                ops.append(dist.P2POp(dist.isend, sl[h], h, group=self.group))
        if me < hubs and sl[me].numel():
            for r in range(G):
                if r != me:
                    bufs[r] = self._p2p_buf(r, sl[me])
                    ops.append(dist.P2POp(dist.irecv, bufs[r], r, group=self.group))
        self._run_p2p(ops)
        if bufs:
            acc = sl[me]
            parts = [acc.clone() if r == me else bufs[r] for r in range(G)]
            acc.copy_(torch.stack(parts).sum(0))
        ops = []
        if me < hubs and sl[me].numel():
            for r in range(G):
                if r != me:
                    ops.append(dist.P2POp(dist.isend, sl[me], r, group=self.group))
        for h in range(hubs):
            if h != me and sl[h].numel():
                ops.append(dist.P2POp(dist.irecv, sl[h], h, group=self.group))
        self._run_p2p(ops)

    def _p2p_buf(self, r: int, like: torch.Tensor) -> torch.Tensor:
        cache = self.__dict__.setdefault("_p2p_bufs", {})
        key = (r, like.numel(), like.dtype, like.device)
        b = cache.get(key)
        if b is None:
            b = cache[key] = torch.empty_like(like)
        return b

    @staticmethod
    def _run_p2p(ops) -> None:
        if not ops:
            return
        for w in dist.batch_isend_irecv(ops):
            w.wait()

    def all_reduce_coalesced_(self, ts: list[torch.Tensor], tag: str = "sync", hubs: int = 0,
                              bucket_bytes: int = 64 << 20):
        """Sums several buffers over ranks with as few collectives as possible: they are
        packed into flat buckets of ≤ ``bucket_bytes`` (≥ 4–8 MB keeps
        a ring all-reduce bandwidth-bound on the 7 xGMI links, the cap bounds the staging
        memory); a buffer larger than the cap is reduced in cap-sized slices. With every
        rank a hub the buckets are issued back to back as asynchronous all-reduces so
        RCCL pipelines them, then waited for."""
        ts = [t for t in ts if t is not None and t.numel()]
        if not ts:
            return
        if len(ts) == 1 and ts[0].numel() * ts[0].element_size() <= bucket_bytes:
            self.hub_reduce_(ts[0], hubs, tag)
            return
        # plan: groups of whole tensors (same dtype) up to the cap; big tensors sliced
        groups: list[list[torch.Tensor]] = []
        cur, cur_bytes = [], 0
        for t in ts:
            flat = t.view(-1)
            nb = flat.numel() * flat.element_size()
            if nb > bucket_bytes:
                step = max(1, bucket_bytes // flat.element_size())
                for a in range(0, flat.numel(), step):
                    groups.append([flat[a:a + step]])
                continue
            if cur and (cur_bytes + nb > bucket_bytes or cur[0].dtype != flat.dtype):
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.append(flat)
            cur_bytes += nb
        if cur:
            groups.append(cur)
        every_rank_hub = self.world == 1 or hubs == 0 or hubs >= self.world
        pending = []
        for g in groups:
            flat = g[0] if len(g) == 1 else torch.cat(g)
            if every_rank_hub:
                work = self.all_reduce_(flat, tag, async_op=True)
            else:
                self.hub_reduce_(flat, hubs, tag)
                work = None
            pending.append((g, flat, work))
        for g, flat, work in pending:
            if work is not None:
                work.wait()
            if len(g) > 1:
                o = 0
                for t in g:
                    n = t.numel()
                    t.copy_(flat[o:o + n])
                    o += n

    def broadcast_(self, t: torch.Tensor, src: int = 0, tag: str = "bcast"):
        if self.world > 1:
            self.stats.add(tag, t.numel() * t.element_size(), kind="broadcast")
            dist.broadcast(t, src=src, group=self.group)

    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        box = [obj if self.rank == src else None]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    def all_gather_object(self, obj) -> list:
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather_tensor(self, t: torch.Tensor, dst: int = 0) -> list[torch.Tensor] | None:
        """Variable-length gather along dim 0 to ``dst`` only: the row counts travel over
        the host control group (no device sync), then every worker sends its rows to the
        hub point-to-point (RCCL send/recv over the xGMI link to the hub on GPUs) — the
        hub alone receives, nothing is padded or all-gathered (the reference's
        ForwardingWorker → CentralizedMLServer, MLNodeGenerator.scala:27,56)."""
        if self.world == 1:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64)
        ns_t = [torch.zeros_like(n) for _ in range(self.world)] if self.rank == dst else None
        dist.gather(n, ns_t, dst=dst, group=self.ctrl_group)
        wire_dtype = t.dtype
        src = t.contiguous()
        if wire_dtype in _BYTE_WIRE:
            # int16 (the compact categorical slots), bool, …: neither RCCL nor gloo has the
            # type, so the rows travel as their bytes and are viewed back on arrival
            src = src.view(torch.uint8)
        row_shape = tuple(src.shape[1:])
        if self.rank != dst:
            if t.shape[0]:
                self.stats.add("gather", src.numel() * src.element_size(), kind="p2p_send")
                dist.send(src, dst=dst, group=self.group)
            return None
        ns = [int(x[0]) for x in ns_t]
        outs, works = [], []
        for r, k in enumerate(ns):
            if r == dst:
                outs.append(src)
                continue
            buf = torch.empty((k,) + row_shape, dtype=src.dtype, device=src.device)
            outs.append(buf)
            if k:
                works.append(dist.irecv(buf, src=r, group=self.group))
        for w in works:
            w.wait()
        if wire_dtype in _BYTE_WIRE:
            outs = [o.view(wire_dtype) for o in outs]
        return outs

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)


def init_distributed(device_type: str = "auto", timeout_s: float = 600.0) -> tuple[Comm, torch.device]:
    """Initialise torch.distributed from torchrun env vars (RANK/WORLD_SIZE/MASTER_*).
    One process per GPU, backend nccl (= RCCL) on GPUs, gloo on CPU."""
    import datetime

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() if device_type == "auto" else device_type != "cpu"
    # OMLDM_DIST_BACKEND=gloo rehearses several ranks on fewer GPUs (ranks share a device
    # round-robin); production is one rank per GPU over RCCL.
    backend = os.environ.get("OMLDM_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    ndev = torch.cuda.device_count() if use_gpu else 0
    device = torch.device("cuda", local_rank % max(1, ndev)) if use_gpu else torch.device("cpu")
    placement = {}
    if use_gpu:
        torch.cuda.set_device(device)
        # host thread + pinned pages on the GPU's socket (utils/topology.py)
        from omldm_amd.utils.topology import bind_to_device

        placement = bind_to_device(device)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        kw = {}
        if use_gpu and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    comm = Comm()
    comm.placement = placement
    return comm, device
