#!/usr/bin/env python3
"""Host profile of the Hoeffding tree's exact (per-point check) mode: one 131072-row round
at the P = 16 learners-bench geometry, cProfile sorted by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_batch  # noqa: E402
from omldm_amd.models import make_learner  # noqa: E402
from omldm_amd.models.base import RoundContext  # noqa: E402

sp = FeatureSpace(13, 0, 26, 1 << 20)
dev = torch.device("cuda")
ring = [synth_batch(sp, 131072, start=k * 131072, seed=25, task=2, n_classes=4).to(dev)
        for k in range(3)]
ht = make_learner("HT", {"nClasses": 4}, sp, dev)
for k in range(2):
    ht.fit(ring[k], RoundContext(spokes=16))
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
ht.fit(ring[2], RoundContext(spokes=16))
torch.cuda.synchronize()
pr.disable()
print("round ms", (time.perf_counter() - t) * 1e3, "nodes", int(ht.nnodes.item()))
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
