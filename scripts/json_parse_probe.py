"""GPU JSON parser timing: wave-staged (LDS) kernel vs the one-thread-per-record global
kernel (selected by a misaligned base pointer) on the same HBM-resident block."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_json_records  # noqa: E402
from omldm_amd.io.transport import join_block  # noqa: E402
from omldm_amd.ops.ingest import json_parse  # noqa: E402

dev = torch.device("cuda", 0)
sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
out = {}
for n in (65536, 131072):
    recs = [r.encode() for r in synth_json_records(min(n, 32768), sp, seed=3)]
    recs = (recs * (n // len(recs) + 1))[:n]
    buf, offs = join_block(recs)
    raw = torch.zeros(len(buf) + 64, dtype=torch.uint8, device=dev)
    raw[16:16 + len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    o = torch.from_numpy(offs).to(dev)
    res = {}
    for name, base in (("staged", 16), ("global", 17)):
        # base 17: misaligned start → the launcher picks the global-memory kernel
        d = raw if base == 16 else raw[1:]  # same bytes, aligned vs misaligned base
        oo = o + (16 if base == 16 else 15)
        num = torch.empty((n, sp.dn), dtype=torch.float32, device=dev)
        cat = torch.empty((n, sp.dc), dtype=sp.cat_dtype, device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        op = torch.empty(n, dtype=torch.int8, device=dev)
        cnt = torch.zeros(3, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            json_parse(d, oo, n, sp, num, cat, y, op, cnt, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            json_parse(d, oo, n, sp, num, cat, y, op, cnt, s)
        e1.record()
        torch.cuda.synchronize()
        res[name] = (e0.elapsed_time(e1) / 20 * 1e3, num.clone(), cat.clone(), y.clone(), op.clone())
    a, b = res["staged"], res["global"]
    same = all(torch.equal(torch.nan_to_num(x, nan=-7.0), torch.nan_to_num(z, nan=-7.0))
               for x, z in zip(a[1:], b[1:]))
    out[n] = {"staged_us": round(a[0], 1), "global_us": round(b[0], 1), "identical": same,
              "MB": round(len(buf) / 1e6, 1)}
print(json.dumps(out))
