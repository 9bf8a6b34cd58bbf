#!/usr/bin/env python3
"""Diagnostics: the bench's engine e2e (JSON then DIB) at a smaller size, with the v3
round counters, the scan error word and the per-stage host ms of each."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from omldm_amd.ops import linear as L  # noqa: E402
from omldm_amd.ops import native  # noqa: E402

order = sys.argv[1:] or ["json", "dib", "dib"]
for fmt in order:
    r0 = L.SCAN3_ROUNDS
    t = time.perf_counter()
    res = bench.engine_e2e_rate(2097152, 524288, fmt=fmt)
    print(fmt, "records/s", res["records_per_s"], "ms/tick", res["ms_per_tick"],
          "v3 rounds", L.SCAN3_ROUNDS - r0, "comb_err", native.hip().omldm_scan3_comb_err(),
          "round ms", res["stage_ms_per_tick"].get("round"), "wall", round(time.perf_counter() - t, 1),
          flush=True)
