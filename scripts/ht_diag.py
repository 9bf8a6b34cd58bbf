"""HT persistent exact kernel diagnostics: segments, splits and cycles per phase."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models.dense import HT  # noqa: E402
from omldm_amd.ops import dense as D  # noqa: E402

dev = torch.device("cuda")
sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
ring = [synth_batch(sp, 131072, start=k * 131072, seed=25, task=2, n_classes=4).to(dev)
        for k in range(3)]
ht = HT({"nClasses": 4}, sp, dev)
dbg = torch.zeros(8, dtype=torch.int64, device=dev)
out = []
for it in range(8):
    b = ring[it % 3]
    x = b.num.float().contiguous()
    dbg.zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    D.ht_exact(x, b.y, ht.Cn, ht.depth, ht.N, ht.nb, float(ht.grace), ht.delta, ht.tau,
               ht._tree(), ht.cum[1:2], dbg)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    v = dbg.cpu().tolist()
    out.append({"round": it, "ms": round(ms, 3), "nodes": int(ht.nnodes.item()), "chunks": v[0],
                "segments": v[1], "splits": v[2], "cyc_setup": v[3], "cyc_due": v[4],
                "cyc_stat": v[5], "cyc_split": v[6]})
    print(json.dumps(out[-1]), flush=True)
