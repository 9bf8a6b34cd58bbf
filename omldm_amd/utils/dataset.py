"""Bounded FIFO buffer — the reference's ``mlAPI.dataBuffers.DataSet[T](maxSize)``.

Used by the reference for the spoke's holdout test set (FIFO of ``testSetSize``,
omldm/operators/spoke/FlinkSpoke.scala:41,96-99), the record/request buffers
(omldm/operators/spoke/SpokeLogic.scala:32-35, caps 100000 / 10000) and the hub's
message cache (omldm/state/StateAccumulators.scala:38,136-144, cap 20000); restore
merges the buffers of several old subtasks (FlinkSpoke.scala:309-330,
SpokeLogic.scala:37-50). API: ``append → Option[evicted]``, ``pop``,
``merge``, ``data_buffer``, ``length``, ``max_size``, ``is_empty``/``non_empty``,
``clear``. The device-resident holdout ring (engine/holdout.py) implements the same
FIFO semantics on HBM for tensors; this class holds host objects (requests, raw records).
"""
from __future__ import annotations

from collections import deque
from typing import Generic, Iterable, TypeVar

T = TypeVar("T")


class DataSet(Generic[T]):
    def __init__(self, max_size: int = 500_000, items: Iterable[T] | None = None):
        if max_size < 0:
            raise ValueError("max_size must be >= 0")
        self.max_size = int(max_size)
        self._q: deque = deque()
        for x in items or ():
            self.append(x)

    # reference names ---------------------------------------------------------
    def append(self, item: T) -> T | None:
        """Append; when full, the oldest element is evicted and returned."""
        if self.max_size == 0:
            return item
        self._q.append(item)
        if len(self._q) > self.max_size:
            return self._q.popleft()
        return None

    def pop(self) -> T | None:
        return self._q.popleft() if self._q else None

    def merge(self, others: Iterable["DataSet[T]"]) -> "DataSet[T]":
        """Concatenate other buffers after this one (restore of several old subtasks);
        capacity grows to hold them all, like the reference's restore-merge."""
        for o in others:
            self.max_size = max(self.max_size, len(self._q) + len(o))
            self._q.extend(o._q)
        return self

    @property
    def data_buffer(self) -> list[T]:
        return list(self._q)

    @property
    def length(self) -> int:
        return len(self._q)

    def get_max_size(self) -> int:
        return self.max_size

    def is_empty(self) -> bool:
        return not self._q

    def non_empty(self) -> bool:
        return bool(self._q)

    def clear(self) -> None:
        self._q.clear()

    # python protocol -----------------------------------------------------------
    def extend(self, items: Iterable[T]) -> list[T]:
        """Append many; returns the evicted elements in order."""
        out = []
        for x in items:
            e = self.append(x)
            if e is not None:
                out.append(e)
        return out

    def take(self, n: int) -> list[T]:
        n = min(n, len(self._q))
        return [self._q.popleft() for _ in range(n)]

    def room(self) -> int:
        return self.max_size - len(self._q)

    def __len__(self):
        return len(self._q)

    def __iter__(self):
        return iter(self._q)

    def state_dict(self) -> dict:
        return {"max_size": self.max_size, "items": list(self._q)}

    @staticmethod
    def from_state(sd: dict) -> "DataSet":
        d = DataSet(sd.get("max_size", 500_000))
        d._q.extend(sd.get("items", []))
        return d


class IntWrapper:
    """Mutable boxed int shared by reference between a spoke and its networks
    (mlAPI.protocols.IntWrapper; FlinkSpoke.scala:31,69,346-347)."""

    def __init__(self, v: int = 0):
        self.v = int(v)

    def get_int(self) -> int:
        return self.v

    def set_int(self, v: int) -> None:
        self.v = int(v)


def integer_parsing(m: dict | None, key: str, default: int) -> int:
    """mlAPI.utils.Parsing.IntegerParsing(map, key, default): lenient int lookup
    (FlinkSpoke.scala:184, FlinkHub.scala:177) — numbers, numeric strings, else default."""
    if not m or key not in m or m[key] is None:
        return default
    v = m[key]
    try:
        if isinstance(v, str):
            return int(float(v.strip()))
        return int(v)
    except (TypeError, ValueError):
        return default
