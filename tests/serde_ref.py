"""Record (de)serialisers kept for API completeness.

The reference carries several serialisation helpers that its job never wires in
(SURVEY.md §2.1 dead-code check): Kafka deserialisers that attach record metadata
(omldm/utils/deserializers/DataInstanceDeserializer.scala:18-40, RequestDeserializer.scala:
17-37), a Jackson ``GenericSerializer`` (omldm/utils/serializers/GenericSerializer.scala:
8-11) and a CSV → ``Array[Double]`` parser (omldm/utils/parsers/StringToArrayDoublesParser
.scala:3-4). They are small pure functions here; the engine's hot path parses with the
C++ scanner (csrc/host/ingest.cpp) instead.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Any

from omldm_amd.api.schemas import DataInstance, Request


@dataclasses.dataclass
class RecordMetadata:
    topic: str
    partition: int
    key: int | None
    offset: int
    timestamp: int


def _metadata_obj(md: RecordMetadata) -> dict:
    return {"topic": md.topic, "partition": md.partition, "key": md.key, "offset": md.offset,
            "timestamp": md.timestamp}


def deserialize_data_instance(value: bytes | str, md: RecordMetadata | None = None
                              ) -> DataInstance | None:
    """JSON → DataInstance with ``metadata`` attached; None for invalid / EOS records."""
    try:
        di = DataInstance.from_json(value)
    except (ValueError, TypeError):
        return None
    if not di.is_valid():
        return None
    if md is not None:
        di.metadata = _metadata_obj(md)  # type: ignore[attr-defined]
    return di


def deserialize_request(value: bytes | str, md: RecordMetadata | None = None) -> Request | None:
    try:
        req = Request.from_json(value)
    except (ValueError, TypeError, AttributeError):
        return None
    if not req.is_valid():
        return None
    if md is not None:
        req.metadata = _metadata_obj(md)  # type: ignore[attr-defined]
    return req


def serialize(obj: Any) -> bytes:
    """Generic JSON serialiser: schema objects via ``to_obj``/``to_json``, dataclasses,
    and plain containers."""
    if hasattr(obj, "to_json"):
        return obj.to_json().encode()
    if hasattr(obj, "to_obj"):
        return json.dumps(obj.to_obj()).encode()
    if dataclasses.is_dataclass(obj):
        return json.dumps(dataclasses.asdict(obj)).encode()
    return json.dumps(obj).encode()


def string_to_doubles(s: str, sep: str = ",") -> list[float]:
    """CSV line → list of doubles (empty fields skipped)."""
    return [float(t) for t in s.strip().split(sep) if t.strip()]
