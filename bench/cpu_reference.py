#!/usr/bin/env python3
"""Reference-class CPU baseline for the headline metric (the reference
publishes no numbers and no JVM exists here, so we measure a faithful CPU equivalent).

Reference semantics: P spokes, each a strictly sequential online PA-I learner over its
shard with a full model replica, synchronised by model averaging (OMLDM's Synchronous
protocol, default parallelism 16). Here: the same data shapes as bench.py (13 numerical
+ 26 hashed categorical features into 2^20 slots), P = --threads spokes, one host thread
per spoke running a C++ sequential learner, averaged every round — no JVM/Kryo/Kafka
overheads, so this is an UPPER bound on the reference's throughput on this CPU:

* ``--wire raw`` (default): the headline's raw wire (32-bit tokens hashed inline) on the
  golden oracle csrc/host/rawwire.cpp — dense per-thread delta arrays, no hash maps;
* ``--wire hashed``: pre-hashed slots on csrc/host/linear_cpu.cpp (sparse deltas).

    python bench/cpu_reference.py [--threads 16 --rows 8192 --steps 10 --wire raw]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch, synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--rows", type=int, default=8192, help="rows per spoke per round")
    ap.add_argument("--wire", default="raw", choices=["raw", "hashed"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--dim-log2", type=int, default=20)
    a = ap.parse_args(argv)
    os.environ["OMLDM_CPU_THREADS"] = str(a.threads)
    space = FeatureSpace(13, 0, 26, 1 << a.dim_log2)
    S, R = a.threads, a.rows
    B = S * R
    w = torch.zeros(space.dim)
    dacc = torch.zeros(space.dim + 2)
    rule = L.LinearRule(rule=L.RULE_HINGE, variant=L.PA1, C=1.0)
    if a.wire == "raw":
        pool = [synth_raw(space, B, start=k * B, seed=25) for k in range(3)]

        def rnd(b):
            L.linear_seq_round(w, b, R, S, dacc, rule, 1.0 / S)
    else:
        pool = [synth_batch(space, B, start=k * B, seed=25) for k in range(3)]

        def rnd(b):
            L.linear_round(w, b, R, S, dacc, None, rule, 1.0 / S)
    rnd(pool[0])
    L.linear_apply(w, None, dacc)
    t0 = time.perf_counter()
    for k in range(a.steps):
        rnd(pool[k % 3])
        L.linear_apply(w, None, dacc)
    el = time.perf_counter() - t0
    if a.wire == "raw":
        test = synth_raw(space, 20000, start=10**12, seed=25).hashed(space)
    else:
        test = synth_batch(space, 20000, start=10**9, seed=25)
    acc = float(((L.linear_predict(w, test) >= 0).float() * 2 - 1 == test.y).float().mean())
    print(json.dumps({"metric": "training examples/s, reference-class CPU (sequential PA-I "
                                "spokes + model averaging)",
                      "value": round(a.steps * B / el, 1), "unit": "examples/s",
                      "threads": a.threads, "cpu_count": os.cpu_count(), "wire": a.wire,
                      "rows_per_spoke_per_round": R, "holdout_accuracy": round(acc, 4)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
