#!/usr/bin/env python3
"""Host profile of the engine's tick thread in the end-to-end bench (cProfile around
bench.engine_e2e_rate): which Python calls a tick spends its host time in.
Usage: python scripts/e2e_profile.py [dib|json] [records] > out.txt"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "dib"
records = int(sys.argv[2]) if len(sys.argv) > 2 else 2097152
bench.engine_e2e_rate(1 << 20, fmt=fmt)  # warm (staging slots, kernels)
pr = cProfile.Profile()
pr.enable()
r = bench.engine_e2e_rate(records, fmt=fmt)
pr.disable()
print(r)
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(60)
print(s.getvalue())
