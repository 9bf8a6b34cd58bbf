#!/usr/bin/env python3
"""Times the v3 prep passes (under rocprofv3 --kernel-trace --stats) with parts of the Gram
pass switched off: python scripts/gram_ablate.py ABLATE (bit 0 categorical counts, bit 1
dense MFMA, bit 2 output stores). Headline geometry: 16 spokes × 8192 rows, 2^20 slots."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from omldm_amd.api.batch import FeatureSpace  # noqa: E402
from omldm_amd.io.synthetic import synth_raw  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402
from omldm_amd.ops import native  # noqa: E402

abl = int(sys.argv[1]) if len(sys.argv) > 1 else 0
native.check(native.hip().omldm_scan3_set_gram_ablate(abl), "set_gram_ablate")
space = FeatureSpace(13, 0, 26, 1 << 20)
b = synth_raw(space, 16 * 8192, seed=25).to("cuda")
rule = L.LinearRule()
for k in range(30):
    L.linear_scan3_prepare(b, 8192, 16, space.dim, True, rule, slot=k % 2)
torch.cuda.synchronize()
native.hip().omldm_scan3_set_gram_ablate(0)
print("ok", abl, flush=True)
