"""Message-passing node programs of the bipartite topology — the protocol golden model.

Reference surface: ``Node.receiveTuple / receiveMsg / receiveQuery /
toggle / merge``; ``BufferingWrapper`` (spoke wrapper that buffers tuples while its
worker waits on the parameter server — dispatch via reflection in the reference,
hs_err_pid77107.log:112-113); ``GenericWrapper`` (hub wrapper; the reference's FlinkHub
caches messages that arrive before Create and drains them on the *next* message,
omldm/operators/hub/FlinkHub.scala:70-87 — fixed here: drained on Create);
8 worker and 8 PS state machines behind ``MLNodeGenerator``
(omldm/utils/generators/MLNodeGenerator.scala:20-76).

Role in this framework. Production training runs the protocols as SPMD collectives
(omldm_amd/parallel/protocols.py). This module runs the *same* protocols in their
original form — workers and hubs exchanging PUSH/REPLY/UPDATE messages — on
``LocalNetwork`` with seeded delivery interleavings. It is the golden oracle for the
protocol tests (SSP staleness bound, BSP = averaging, asynchronous convergence, EASGD
fixed point, message/byte accounting) and a readable specification of each protocol.
Models are NumPy vectors; the learner is any ``fit(w, point) -> w`` function.
"""
from __future__ import annotations

from typing import Any, Callable

import numpy as np

from omldm_amd.engine.network import RPC, LocalNetwork, NetworkDescriptor, NodeId, NodeType
from omldm_amd.utils.dataset import DataSet

FitFn = Callable[[np.ndarray, Any], np.ndarray]


class Node:
    """Base node (NodeInstance): everything arrives through these four entry points."""

    def __init__(self, nid: NodeId, network: LocalNetwork):
        self.nid = nid
        self.network = network

    def receive_tuple(self, point) -> None:
        pass

    def receive_msg(self, source: NodeId, rpc: RPC, data) -> None:
        pass

    def receive_query(self, query_id: int, payload) -> None:
        pass

    def toggle(self) -> None:
        pass

    def merge(self, others: list["Node"]) -> "Node":
        return self


class BufferingWrapper(Node):
    """Spoke wrapper: while the worker is blocked on the hub, incoming tuples are buffered
    (bounded, like the reference's record buffer) and replayed in order on unblock."""

    def __init__(self, nid, network, worker: "Worker", max_buffer: int = 100_000):
        super().__init__(nid, network)
        self.worker = worker
        self.buffer: DataSet = DataSet(max_buffer)
        self.dropped = 0

    def receive_tuple(self, point):
        if self.worker.blocked:
            if self.buffer.append(point) is not None:
                self.dropped += 1
        else:
            self.worker.receive_tuple(point)

    def receive_msg(self, source, rpc, data):
        self.worker.receive_msg(source, rpc, data)
        self._drain()

    def _drain(self):
        while not self.worker.blocked and self.buffer.non_empty():
            self.worker.receive_tuple(self.buffer.pop())

    def toggle(self):
        self._drain()

    def receive_query(self, query_id, payload):
        return self.worker.receive_query(query_id, payload)


class GenericWrapper(Node):
    """Hub wrapper with a cache for messages that arrive before the hub node exists."""

    def __init__(self, nid, network, cache_size: int = 20_000):
        super().__init__(nid, network)
        self.node: Node | None = None
        self.cache: DataSet = DataSet(cache_size)

    def create(self, node: Node):
        self.node = node
        while self.cache.non_empty():
            src, rpc, data = self.cache.pop()
            node.receive_msg(src, rpc, data)

    def receive_msg(self, source, rpc, data):
        if self.node is None:
            self.cache.append((source, rpc, data))
        else:
            self.node.receive_msg(source, rpc, data)


# ------------------------------------------------------------------------ workers
class Worker(Node):
    """Generic worker: trains on tuples; every ``batch`` tuples it runs ``on_round``."""

    def __init__(self, nid, network, w0: np.ndarray, fit: FitFn, batch: int = 8,
                 hub: NodeId | None = None):
        super().__init__(nid, network)
        self.w = w0.astype(np.float64).copy()
        self.fit = fit
        self.batch = batch
        self.hub = hub or NodeId(NodeType.HUB, 0)
        self.blocked = False
        self.seen = 0
        self.clock = 0

    def receive_tuple(self, point):
        self.w = self.fit(self.w, point)
        self.seen += 1
        if self.seen % self.batch == 0:
            self.on_round()

    def on_round(self):
        pass

    def send(self, rpc, data):
        self.network.send(self.nid, self.hub, rpc, data)


class SynchronousWorker(Worker):
    """BSP: push the local model, block until the averaged model comes back."""

    def on_round(self):
        self.blocked = True
        self.send(RPC.PUSH, self.w.copy())

    def receive_msg(self, source, rpc, data):
        if rpc == RPC.UPDATE:
            self.w = data.copy()
            self.blocked = False


class AsynchronousWorker(Worker):
    """Push the local progress since the last pull (with the clock), block until the
    hub's reply to *this* worker (no barrier across workers); SSP shares this worker."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.base = self.w.copy()

    def on_round(self):
        self.blocked = True
        self.clock += 1
        self.send(RPC.PUSH, (self.clock, self.w - self.base))

    def receive_msg(self, source, rpc, data):
        if rpc == RPC.REPLY:
            self.w = data.copy()
            self.base = self.w.copy()
            self.blocked = False


class EASGDWorker(Worker):
    """Every τ local steps: send x_i, receive the centre x̃ (pre-update), move
    x_i ← x_i − α(x_i − x̃)."""

    def __init__(self, *a, alpha: float = 0.1, **k):
        super().__init__(*a, **k)
        self.alpha = alpha

    def on_round(self):
        self.blocked = True
        self.send(RPC.PUSH, self.w.copy())

    def receive_msg(self, source, rpc, data):
        if rpc == RPC.REPLY:
            self.w = self.w - self.alpha * (self.w - data)
            self.blocked = False


# ------------------------------------------------------------------------ hubs
class Hub(Node):
    def __init__(self, nid, network, w0: np.ndarray, n_workers: int):
        super().__init__(nid, network)
        self.w = w0.astype(np.float64).copy()
        self.P = n_workers
        self.pushes = 0

    def spokes(self):
        return [NodeId(NodeType.SPOKE, i) for i in range(self.P)]


class SynchronousPS(Hub):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.pending: dict = {}

    def receive_msg(self, source, rpc, data):
        if rpc != RPC.PUSH:
            return
        self.pushes += 1
        self.pending[source] = data
        if len(self.pending) == self.P:
            self.w = np.mean(list(self.pending.values()), axis=0)
            self.pending.clear()
            self.network.broadcast(self.nid, {s: RPC.UPDATE for s in self.spokes()}, self.w.copy())


class AsynchronousPS(Hub):
    """Adds each worker's progress (scaled by 1/P) and replies to it immediately.
    With ``staleness`` s (SSP) a reply to a worker whose clock is more than s ahead of
    the slowest worker is withheld until the slowest catches up."""

    def __init__(self, *a, staleness: int | None = None, **k):
        super().__init__(*a, **k)
        self.s = staleness
        self.clocks = {s: 0 for s in self.spokes()}
        self.withheld: list = []
        self.max_gap = 0

    def receive_msg(self, source, rpc, data):
        if rpc != RPC.PUSH:
            return
        clock, delta = data
        self.pushes += 1
        self.w = self.w + delta / self.P
        self.clocks[source] = clock
        self.withheld.append(source)
        self._release()

    def _release(self):
        lo = min(self.clocks.values())
        keep = []
        for src in self.withheld:
            if self.s is not None and self.clocks[src] > lo + self.s:
                keep.append(src)
            else:
                self.max_gap = max(self.max_gap, self.clocks[src] - lo)
                self.network.send(self.nid, src, RPC.REPLY, self.w.copy())
        self.withheld = keep


class EASGDPS(Hub):
    def __init__(self, *a, alpha: float = 0.1, **k):
        super().__init__(*a, **k)
        self.alpha = alpha

    def receive_msg(self, source, rpc, data):
        if rpc != RPC.PUSH:
            return
        self.pushes += 1
        centre = self.w.copy()
        self.w = self.w + self.alpha * (data - centre)
        self.network.send(self.nid, source, RPC.REPLY, centre)


_PAIRS = {
    "Synchronous": (SynchronousWorker, SynchronousPS, {}),
    "Asynchronous": (AsynchronousWorker, AsynchronousPS, {}),
    "SSP": (AsynchronousWorker, AsynchronousPS, {"staleness": 2}),
    "EASGD": (EASGDWorker, EASGDPS, {"alpha": 0.1}),
}


def build_topology(protocol: str, n_workers: int, w0: np.ndarray, fit: FitFn, batch: int = 8,
                   seed: int = 0, **kw):
    """A LocalNetwork with ``n_workers`` BufferingWrapper spokes and one hub."""
    wcls, hcls, defaults = _PAIRS[protocol]
    opts = {**defaults, **kw}
    net = LocalNetwork(NetworkDescriptor(0, n_workers, 1), seed=seed)
    hub_kw = {k: v for k, v in opts.items() if k in ("staleness", "alpha")}
    hub = GenericWrapper(NodeId(NodeType.HUB, 0), net)
    hub.create(hcls(hub.nid, net, w0, n_workers, **hub_kw))
    net.register(hub.nid, hub)
    spokes = []
    for i in range(n_workers):
        nid = NodeId(NodeType.SPOKE, i)
        wk = {"alpha": opts["alpha"]} if wcls is EASGDWorker else {}
        wrapper = BufferingWrapper(nid, net, wcls(nid, net, w0, fit, batch, **wk))
        net.register(nid, wrapper)
        spokes.append(wrapper)
    return net, hub, spokes


def run_stream(net: LocalNetwork, spokes: list, points: list, shard: Callable[[int], int],
               deliver_every: int = 1) -> None:
    """Feed points to spokes (``shard(i)`` picks the spoke) while the network delivers
    messages in seeded random order; drains everything at the end."""
    for i, p in enumerate(points):
        spokes[shard(i)].receive_tuple(p)
        if i % deliver_every == 0:
            net.step()
    while net.step():
        pass
    for s in spokes:
        s.toggle()
