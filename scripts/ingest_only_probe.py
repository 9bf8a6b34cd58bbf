#!/usr/bin/env python3
"""Host ingest alone (engine/ingest.py TickIngest over a FileBroker topic, GPU staging on or
off): blocks/s and GB/s of the read-ahead pipeline with no training — separates the host
read ceiling from the engine's other per-tick work (diagnostics)."""
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.engine.ingest import TickIngest  # noqa: E402
from omldm_amd.io.synthetic import synth_json_records  # noqa: E402
from omldm_amd.io.transport import Consumer, FileBroker  # noqa: E402

sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
uniq = synth_json_records(20000, sp, seed=3)
res = {}
for parts in (8, 32):
    with tempfile.TemporaryDirectory() as root:
        br = FileBroker(root)
        br.create_topic("trainingData", parts)
        recs_per_part = 4_000_000 // parts
        for p in range(parts):
            recs = [uniq[(i * parts + p) % len(uniq)] for i in range(recs_per_part)]
            br.produce_block("trainingData", p, ("\n".join(recs) + "\n").encode())
        for stage in (False, True):
            c = Consumer(br, "trainingData", 0, 1)
            dev = torch.device("cuda", 0) if stage and torch.cuda.is_available() else None
            ing = TickIngest([c], 131072, pinned=True, device=dev, space=sp if dev else None)
            for _ in range(3):
                ing.next()
            t = time.perf_counter()
            n = nb = 0
            while True:
                blk = ing.next()
                if blk.n == 0:
                    break
                n += blk.n
                nb += blk.nbytes
            dt = time.perf_counter() - t
            ing.close()
            res[f"p{parts}_{'stage' if stage else 'read'}"] = {
                "Mrec_s": round(n / dt / 1e6, 1), "GB_s": round(nb / dt / 1e9, 1)}
print(json.dumps(res))
