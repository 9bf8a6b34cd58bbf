"""Operator tools (the reference's deployment recipe, README.md:20-41: create the Kafka
topics, then ``flink run``):

    python -m omldm_amd.tools topics  --bootstrap host:9092 [--data-partitions 36]
    python -m omldm_amd.tools produce --bootstrap host:9092 --topic requests --file reqs.jsonl
    python -m omldm_amd.tools tail    --bootstrap host:9092 --topic responses [-n 20]
    python -m omldm_amd.tools synth   --bootstrap host:9092 --topic trainingData --n 100000
    python -m omldm_amd.tools import-models --bootstrap host:9092 --file ckpt-000003/models.json
        (re-creates every pipeline of a checkpoint's model export, warm-started, through
         the requests topic — any world size, any job)

``--bootstrap`` also accepts ``file:///dir`` (FileBroker) for single-node runs.
"""
from __future__ import annotations

import argparse
import sys

from omldm_amd.io.transport import Consumer, broker_for

# Partition counts of the reference deployment (README.md:21-26); psMessages is not
# needed (RCCL replaces the feedback topic).
TOPICS = {"requests": 1, "responses": 1, "trainingData": 36, "forecastingData": 36,
          "predictions": 36, "performance": 1}


def _produce_all(br, topic: str, recs: list) -> None:
    """Records spread round-robin over the topic's partitions, one block per partition
    (a Kafka RecordBatch per ≤ 900 KiB instead of one Produce request per record)."""
    import numpy as np

    n = br.partitions(topic)
    for p in range(n):
        chunk = recs[p::n]
        if not chunk:
            continue
        block = b"".join(r + b"\n" for r in chunk)
        offs = np.zeros(len(chunk) + 1, dtype=np.int64)
        np.cumsum([len(r) + 1 for r in chunk], out=offs[1:])
        br.produce_lines(topic, block, offs, partition=p)


def _tail(br, topic: str, n: int) -> list:
    """The last ``n`` records of every partition (Kafka: read from end − n; file topics,
    whose offsets are bytes, are read whole)."""
    c = Consumer(br, topic, all_partitions=True)
    from omldm_amd.io.kafka import KafkaBroker

    if isinstance(br, KafkaBroker):
        for p in c.parts:
            c.offsets[p] = max(0, br.end_offset(topic, p) - n)
    out = []
    while True:
        got = c.poll(10**6)
        if not got:
            return out[-n:] if n else out
        out += got


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m omldm_amd.tools")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("topics")
    t.add_argument("--bootstrap", required=True)
    t.add_argument("--data-partitions", type=int, default=36)
    p = sub.add_parser("produce")
    p.add_argument("--bootstrap", required=True)
    p.add_argument("--topic", required=True)
    p.add_argument("--file", required=True)
    tl = sub.add_parser("tail")
    tl.add_argument("--bootstrap", required=True)
    tl.add_argument("--topic", required=True)
    tl.add_argument("-n", type=int, default=20)
    s = sub.add_parser("synth")
    s.add_argument("--bootstrap", required=True)
    s.add_argument("--topic", default="trainingData")
    s.add_argument("--n", type=int, default=10000)
    s.add_argument("--operation", default="training")
    s.add_argument("--hash-dim", type=int, default=1 << 20)
    im = sub.add_parser("import-models")
    im.add_argument("--bootstrap", required=True)
    im.add_argument("--file", required=True)
    im.add_argument("--topic", default="requests")
    im.add_argument("--id-offset", type=int, default=0, help="added to every pipeline id")
    a = ap.parse_args(argv)
    br = broker_for(a.bootstrap)
    if a.cmd == "topics":
        for name, n in TOPICS.items():
            n = a.data_partitions if n == 36 else n
            br.create_topic(name, n)
            print(f"{name}: {n} partition(s)")
    elif a.cmd == "produce":
        with open(a.file, "rb") as f:
            recs = [line.rstrip(b"\n") for line in f if line.strip()]
        if br.partitions(a.topic) == 1:
            for r in recs:  # single-partition control topics keep the file's order
                br.produce(a.topic, r)
        else:
            _produce_all(br, a.topic, recs)
        br.flush()
        print(f"produced {len(recs)} record(s) to {a.topic}")
    elif a.cmd == "tail":
        for rec in _tail(br, a.topic, a.n):
            sys.stdout.write(rec.decode(errors="replace") + "\n")
    elif a.cmd == "import-models":
        import json

        from omldm_amd.utils.checkpoint import import_requests

        reqs = import_requests(a.file)
        for r in reqs:
            r["id"] = int(r["id"]) + a.id_offset
            br.produce(a.topic, json.dumps(r))
        br.flush()
        print(f"produced {len(reqs)} Create request(s) to {a.topic}")
    elif a.cmd == "synth":
        from omldm_amd.api.batch import FeatureSpace
        from omldm_amd.io.synthetic import synth_json_records

        _produce_all(br, a.topic, [r.encode() for r in synth_json_records(
            a.n, FeatureSpace(13, 0, 26, a.hash_dim), operation=a.operation)])
        br.flush()
        print(f"produced {a.n} synthetic record(s) to {a.topic}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
