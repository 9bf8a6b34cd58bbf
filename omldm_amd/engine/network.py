"""Bipartite (spoke ↔ hub) topology: node addressing, RPC identifiers, the three message
types with byte accounting, and the ``Network`` interface with two implementations.

Reference surface:
* ``NodeId(NodeType∈{SPOKE,HUB}|null, id)``, ``NetworkDescriptor(networkId, #spokes,
  #hubs)`` — omldm/job/FlinkLearning.scala:70, omldm/network/FlinkNetwork.scala:295;
* ``RemoteCallIdentifier`` (RPC opcode) — omldm/messages/ControlMessage.scala:19;
* ControlMessage / SpokeMessage / HubMessage (6 fields each; HubMessage carries arrays
  of operations and destinations, its default form is the termination signal) —
  omldm/messages/{ControlMessage,SpokeMessage,HubMessage}.scala;
* ``FlinkMessage.getSize = 4 + op + src + dst + data + request`` feeds ``bytesShipped``
  (omldm/messages/FlinkMessage.scala:16-23); ``HubMessage.getSize`` multiplies
  ``length × Σsize`` (quadratic) — we report true bytes and keep the
  legacy value available as ``legacy_size``;
* ``Network.send / broadcast / describe`` (omldm/network/FlinkNetwork.scala:242-295);
  the hub-message fan-out of FlinkLearning (omldm/job/FlinkLearning.scala:65-75).

MI355X mapping. The training hot path never materialises these messages — the
protocols in ``omldm_amd.parallel.protocols`` are collectives over RCCL, and the
point-to-point parameter-server channels of Asynchronous / SSP live in
``omldm_amd.parallel.p2p``. The message layer exists for (a) the control plane and
statistics (byte accounting identical for every protocol) and (b) ``LocalNetwork``: a
deterministic in-process network with a seeded scheduler that permutes deliveries — the
fake transport the protocol golden tests run on.
"""
from __future__ import annotations

import enum
import json
import random
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Callable


class NodeType(enum.IntEnum):
    SPOKE = 0
    HUB = 1


@dataclass(frozen=True)
class NodeId:
    node_type: NodeType | None
    node_id: int

    def get_size(self) -> int:
        return 8  # type tag + id

    def __str__(self):
        t = "null" if self.node_type is None else self.node_type.name
        return f"{t}:{self.node_id}"


@dataclass(frozen=True)
class NetworkDescriptor:
    network_id: int
    num_spokes: int
    num_hubs: int


class RPC(enum.IntEnum):
    """RemoteCallIdentifier: the opcode of a remote call between nodes."""
    CREATE = 0
    PUSH = 1            # worker → hub: model / delta / gradient block
    PULL = 2            # worker → hub: request the global model
    REPLY = 3           # hub → worker: global model (unicast reply)
    UPDATE = 4          # hub → workers: new global model (broadcast)
    QUERY = 5
    TERMINATE = 6
    HEARTBEAT = 7
    COUNTER = 8         # FGM subround counter increment
    ZONE = 9            # GM/FGM: safe-zone violation / φ report
    FORWARD = 10        # SingleLearner: forwarded data points

    def get_size(self) -> int:
        return 4


def payload_size(data: Any) -> int:
    """Bytes of a message payload (tensors/arrays by storage, containers recursively)."""
    if data is None:
        return 0
    if hasattr(data, "element_size") and hasattr(data, "numel"):
        return int(data.numel() * data.element_size())
    if hasattr(data, "nbytes"):
        return int(data.nbytes)
    if isinstance(data, (bytes, bytearray, memoryview)):
        return len(data)
    if isinstance(data, str):
        return len(data.encode())
    if isinstance(data, bool):
        return 1
    if isinstance(data, (int, float)):
        return 8
    if isinstance(data, (list, tuple)):
        return sum(payload_size(x) for x in data)
    if isinstance(data, dict):
        return len(json.dumps(data, default=str).encode())
    if hasattr(data, "get_size"):
        return int(data.get_size())
    if hasattr(data, "to_json"):
        return len(data.to_json().encode())
    return 0


def _req_size(req) -> int:
    if req is None:
        return 0
    if hasattr(req, "to_json"):
        return len(req.to_json().encode())
    return payload_size(req)


@dataclass
class ControlMessage:
    """Message into a spoke (requests from PipelineMap, expanded hub messages)."""
    network_id: int
    operation: RPC | None
    source: NodeId | None
    destination: NodeId | None
    data: Any = None
    request: Any = None

    def get_size(self) -> int:
        return (4 + (4 if self.operation is not None else 0)
                + (self.source.get_size() if self.source else 0)
                + (self.destination.get_size() if self.destination else 0)
                + payload_size(self.data) + _req_size(self.request))


@dataclass
class SpokeMessage(ControlMessage):
    """Spoke → hub; ``network_id == -1`` is a heartbeat (FlinkSpoke.scala:83-89)."""

    @property
    def is_heartbeat(self) -> bool:
        return self.network_id == -1


@dataclass
class HubMessage:
    """Hub → spokes. Multi-destination form = broadcast; the default-constructed
    message (network -1, no destinations) is the termination signal."""
    network_id: int = -1
    operations: list = field(default_factory=list)
    source: NodeId | None = None
    destinations: list = field(default_factory=list)
    data: Any = None
    request: Any = None

    @property
    def is_termination(self) -> bool:
        return self.network_id == -1 and not self.destinations

    def get_size(self) -> int:
        return (4 + 4 * len(self.operations) + (self.source.get_size() if self.source else 0)
                + 8 * len(self.destinations) + payload_size(self.data) + _req_size(self.request))

    def legacy_size(self) -> int:
        """The reference's quadratic accounting (length × Σsize, HubMessage.scala:48-55)."""
        return max(1, len(self.destinations)) * self.get_size()

    def fan_out(self, n_workers: int) -> list[ControlMessage]:
        """FlinkLearning hub-message expansion (omldm/job/FlinkLearning.scala:65-75):
        termination → one ControlMessage per worker; otherwise one per (op, dest)."""
        if self.is_termination:
            return [ControlMessage(-1, RPC.TERMINATE, self.source, NodeId(NodeType.SPOKE, i))
                    for i in range(n_workers)]
        return [ControlMessage(self.network_id, op, self.source, dst, self.data, self.request)
                for op, dst in zip(self.operations, self.destinations)]


class Network:
    """Transport between the nodes of one pipeline's bipartite graph."""

    def __init__(self, descriptor: NetworkDescriptor):
        self.descriptor = descriptor
        self.bytes_shipped = 0
        self.messages = 0

    def describe(self) -> NetworkDescriptor:
        return self.descriptor

    def _account(self, msg) -> None:
        self.messages += 1
        self.bytes_shipped += msg.get_size()

    def send(self, source: NodeId, destination: NodeId | None, rpc: RPC, data: Any) -> None:
        raise NotImplementedError

    def broadcast(self, source: NodeId, destinations: dict, data: Any) -> None:
        raise NotImplementedError


class LocalNetwork(Network):
    """Deterministic in-process network: messages wait in per-link FIFO queues and a
    seeded scheduler picks which link delivers next, emulating the arbitrary (but
    per-link ordered) interleavings of Flink shuffles and Kafka partitions."""

    def __init__(self, descriptor: NetworkDescriptor, seed: int = 0):
        super().__init__(descriptor)
        self.nodes: dict[NodeId, Any] = {}
        self.links: dict[tuple, deque] = {}
        self.rng = random.Random(seed)
        self.outputs: list = []      # destination None: user-facing output (side output)
        self.log: list = []

    def register(self, nid: NodeId, node) -> None:
        self.nodes[nid] = node

    def _enqueue(self, src, dst, msg):
        self.links.setdefault((src, dst), deque()).append(msg)

    def send(self, source, destination, rpc, data):
        if destination is None:
            self.outputs.append(data)
            return
        if source is not None and source.node_type == NodeType.HUB:
            msg = HubMessage(self.descriptor.network_id, [rpc], source, [destination], data)
        else:
            msg = SpokeMessage(self.descriptor.network_id, rpc, source, destination, data)
        self._account(msg)
        self._enqueue(source, destination, msg)

    def broadcast(self, source, destinations, data):
        dests = list(destinations)
        msg = HubMessage(self.descriptor.network_id, [destinations[d] for d in dests], source,
                         dests, data)
        self._account(msg)
        for cm in msg.fan_out(self.descriptor.num_spokes):
            self._enqueue(source, cm.destination, cm)

    def pending(self) -> int:
        return sum(len(q) for q in self.links.values())

    def step(self) -> bool:
        """Deliver one message from a randomly chosen non-empty link."""
        live = [k for k, q in self.links.items() if q]
        if not live:
            return False
        k = live[self.rng.randrange(len(live))]
        msg = self.links[k].popleft()
        src, dst = k
        op = msg.operation if hasattr(msg, "operation") else msg.operations[0]
        self.log.append((str(src), str(dst), RPC(op).name))
        self.nodes[dst].receive_msg(src, RPC(op), msg.data)
        return True

    def run(self, max_steps: int = 1_000_000) -> int:
        n = 0
        while n < max_steps and self.step():
            n += 1
        return n


def hub_message_round_robin(counter: list, n_partitions: int) -> int:
    """Reference HubMessagePartitioner (dead code, HubMessagePartitioner.scala:15-27): it
    computes ``dest % n``, discards it and round-robins. Kept for completeness."""
    counter[0] = (counter[0] + 1) % n_partitions
    return counter[0]


def fan_out_all(msgs: list[HubMessage], n_workers: int) -> list[ControlMessage]:
    out: list[ControlMessage] = []
    for m in msgs:
        out.extend(m.fan_out(n_workers))
    return out


Handler = Callable[[NodeId, RPC, Any], None]
