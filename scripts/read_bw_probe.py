#!/usr/bin/env python3
"""Host read bandwidth of the FileBroker log reader (csrc/host/logio.cpp) from a file in
/tmp and in /dev/shm, 1..32 reader threads, into a pinned buffer (diagnostics)."""
import concurrent.futures as cf
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_json_records  # noqa: E402
from omldm_amd.io.transport import FileBroker  # noqa: E402

sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
recs = synth_json_records(20000, sp, seed=3)
block = ("\n".join(recs) + "\n").encode()
per_part = 64 << 20
out = {}
for base in ("/tmp", "/dev/shm"):
    if not os.path.isdir(base):
        continue
    with tempfile.TemporaryDirectory(dir=base) as root:
        br = FileBroker(root)
        P = 32
        br.create_topic("t", P)
        for p in range(P):
            n = 0
            while n < per_part:
                br.produce_block("t", p, block)
                n += len(block)
        dst = torch.empty(P * (per_part + (1 << 20)), dtype=torch.uint8).pin_memory().numpy()
        for nt in (1, 8, 32):
            ex = cf.ThreadPoolExecutor(nt)
            t = time.perf_counter()
            res = list(ex.map(lambda p: br.consume_into("t", p, 0, 10**7, dst[p * (per_part + (1 << 20)):], per_part + (1 << 20)), range(P)))
            dt = time.perf_counter() - t
            nbytes = sum(int(o[k]) for k, o, _ in res)
            out[f"{base}_{nt}thr_GBps"] = round(nbytes / dt / 1e9, 1)
            ex.shutdown()
print(json.dumps(out))
