"""A/B of the file-topic reader on one box: sized first read (default) vs the old fixed
1.5x read of the whole region (hint=0), alternating runs of bench/engine_e2e.py."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
import engine_e2e  # noqa: E402

from omldm_amd.io.transport import FileBroker  # noqa: E402

orig = FileBroker.consume_into


def no_hint(self, topic, partition, offset, max_records, dst, cap, hint=0):
    return orig(self, topic, partition, offset, max_records, dst, cap, hint=0)


res = {"sized": [], "full": []}
for rep in range(3):
    for mode in ("sized", "full"):
        FileBroker.consume_into = orig if mode == "sized" else no_hint
        buf = io.StringIO()
        with redirect_stdout(buf):
            engine_e2e.main(["--records", "4000000", "--batch", sys.argv[1] if len(sys.argv) > 1 else "65536"])
        line = [l for l in buf.getvalue().splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
        res[mode].append(round(d["value"] / 1e6, 1))
        print(mode, res[mode][-1], flush=True)
print(json.dumps({"M_records_per_s": res}))
