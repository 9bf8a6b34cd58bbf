"""DIB: the binary DataInstance record (format: csrc/host/dib.h).

A topic may carry DIB records instead of (or mixed with) DataInstance JSON: the same
fields — numerical / discrete features as fp32, categorical features as the 32-bit
murmur3 hash the JSON parser takes of each string, target, operation — in ≈ 162 bytes
for 13 numerical + 26 categorical features instead of ≈ 507 bytes of JSON text. Records
stay newline-framed (the payload is SLIP-stuffed), so every broker, the log reader and
the engine's ingest take both kinds unchanged; the host parser (csrc/host/ingest.cpp)
and the GPU parser (csrc/kernels/json_ingest.hip) decode a record by its first byte. A
forecast of a DIB record echoes it as DataInstance JSON with the categorical features
written as their hashes ("#%08x", csrc/host/egress.cpp).

Reference: the topics carry Jackson-serialised DataInstance JSON
(omldm/utils/parsers/DataInstanceParser.scala:12-22); DIB is this framework's compact
wire for the same objects (the JSON path is unchanged).
"""
from __future__ import annotations

import math
import os
import struct

import numpy as np

from omldm_amd.ops import native

MAGIC = 0xB1
SEED_BASE = 0x9747B28C  # csrc/host/hashing.h: kSeedBase


def is_dib(record: bytes) -> bool:
    return len(record) > 0 and record[0] == MAGIC


def _stuff(payload: bytes) -> bytes:
    return payload.replace(b"\xdb", b"\xdb\xdd").replace(b"\n", b"\xdb\xdc")


def encode(numerical=None, discrete=None, categorical=None, target=None,
           operation: str = "training") -> bytes:
    """One DIB record (without the log's newline) from DataInstance fields."""
    op = {"training": 0, "forecasting": 1}.get(operation, 0xFF)
    num = [float(v) for v in (numerical or [])]
    disc = [float(v) for v in (discrete or [])]
    cats = [str(c).encode() for c in (categorical or [])]
    any_f = numerical is not None or discrete is not None or categorical is not None
    has_y = target is not None and not math.isnan(float(target))
    h = native.host()
    hashes = [int(h.omldm_murmur3_32(c, len(c), (SEED_BASE + j) & 0xFFFFFFFF))
              for j, c in enumerate(cats)]
    assert max(len(num), len(disc), len(cats)) < 256
    body = struct.pack("<5B", op, (1 if has_y else 0) | (2 if any_f else 0), len(num),
                       len(disc), len(cats))
    if has_y:
        body += struct.pack("<f", float(target))
    body += struct.pack(f"<{len(num)}f{len(disc)}f{len(cats)}I", *num, *disc, *hashes)
    return bytes([MAGIC]) + _stuff(body)


def json_to_dib(buf, offs: np.ndarray, n_numerical: int, n_discrete: int, n_categorical: int,
                threads: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """DataInstance JSON records buf[offs[i], offs[i+1]) → (DIB block, record offsets),
    every record newline-terminated (csrc/host/ingest.cpp: omldm_json_to_dib, threaded).
    Records the JSON parser rejects become invalid DIB records (counted the same)."""
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = len(offs) - 1
    src = np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) \
        else np.ascontiguousarray(buf)
    per = 16 + 2 * 4 * (n_numerical + n_discrete + n_categorical + 1)
    out = np.empty(max(1, n * per), dtype=np.uint8)
    out_offs = np.empty(n + 1, dtype=np.int64)
    threads = threads or min(16, os.cpu_count() or 1)
    got = native.host().omldm_json_to_dib(src.ctypes.data, offs.ctypes.data, n, n_numerical,
                                          n_discrete, n_categorical, out.ctypes.data,
                                          out.size, out_offs.ctypes.data, threads)
    if got < 0:
        raise RuntimeError("omldm_json_to_dib: output buffer too small")
    return out[:got], out_offs


def records_to_dib(records: list, n_numerical: int, n_discrete: int,
                   n_categorical: int) -> list[bytes]:
    """JSON records (str / bytes) → DIB records (bytes, no newline)."""
    from omldm_amd.io.transport import join_block

    enc = [r if isinstance(r, (bytes, bytearray)) else str(r).encode() for r in records]
    buf, offs = join_block(enc)
    out, oo = json_to_dib(buf, offs, n_numerical, n_discrete, n_categorical)
    return [out[oo[i]:oo[i + 1] - 1].tobytes() for i in range(len(enc))]


__all__ = ["MAGIC", "encode", "is_dib", "json_to_dib", "records_to_dib"]
