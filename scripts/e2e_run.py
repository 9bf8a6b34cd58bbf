#!/usr/bin/env python3
"""One engine end-to-end run (bench.engine_e2e_rate) for profiling:
python scripts/e2e_run.py [dib|json] [records] [batch]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "dib"
records = int(sys.argv[2]) if len(sys.argv) > 2 else 4194304
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 524288
print(json.dumps(bench.engine_e2e_rate(records, batch, fmt=fmt)), flush=True)
