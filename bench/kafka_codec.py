#!/usr/bin/env python3
"""Kafka record-set throughput on the host: decoding a Fetch response's record set into
a staging buffer (Python reference decoder vs the native one, csrc/host/kafka_wire.cpp)
and encoding a tick's output lines, per codec. DataInstance-shaped JSON records.

    python bench/kafka_codec.py [--records 200000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.io import kafka as K  # noqa: E402


def _best(fn, reps=3):
    t = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t = min(t, time.perf_counter() - t0)
    return t


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=200000)
    ap.add_argument("--batch", type=int, default=2000, help="records per RecordBatch")
    a = ap.parse_args(argv)
    rng = np.random.default_rng(25)
    vals = [json.dumps({"numericalFeatures": [round(float(v), 4) for v in rng.normal(size=13)],
                        "categoricalFeatures": [f"{int(c):08x}" for c in
                                                rng.integers(0, 1 << 30, 26)],
                        "target": float(rng.choice([-1.0, 1.0])),
                        "operation": "training"}).encode() for _ in range(a.records)]
    raw = sum(len(v) for v in vals)
    block = b"".join(v + b"\n" for v in vals)
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    np.cumsum([len(v) + 1 for v in vals], out=offs[1:])
    buf = np.frombuffer(block, dtype=np.uint8)
    dst = np.empty(len(block) + 1024, dtype=np.uint8)
    res = {}
    for codec in ["none", "gzip", "snappy", "lz4", "zstd"]:
        if not K.codec_available(codec):
            continue
        sets = []

        def enc():
            sets.clear()
            for i in range(0, len(vals), a.batch):
                j = min(len(vals), i + a.batch)
                sets.append(K.encode_lines(buf, offs[i:j + 1], codec, base_offset=i))

        t_enc = _best(enc)
        data = b"".join(sets)
        t_nat = _best(lambda: K.KafkaBroker._decode_into(data, 0, len(vals), dst, len(dst)))
        n, _o, _nx = K.KafkaBroker._decode_into(data, 0, len(vals), dst, len(dst))
        assert n == len(vals)
        t_py = _best(lambda: K.decode_batches(data), reps=1)
        res[codec] = {"wire_bytes_per_record": round(len(data) / len(vals), 1),
                      "encode_M_records_per_s": round(len(vals) / t_enc / 1e6, 2),
                      "decode_native_M_records_per_s": round(len(vals) / t_nat / 1e6, 2),
                      "decode_native_GB_per_s": round(raw / t_nat / 1e9, 2),
                      "decode_python_M_records_per_s": round(len(vals) / t_py / 1e6, 3)}
    print(json.dumps({"metric": "Kafka record-set encode/decode on one host thread",
                      "records": len(vals), "record_bytes": round(raw / len(vals), 1),
                      "records_per_batch": a.batch, "codecs": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
