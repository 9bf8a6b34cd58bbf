"""Measurement only (not a supported mode): the device-ingest headline with the round's
cross-stream wait on its prep's event dropped (the prep of round k+1 runs beside round k and
ends ~80 µs before it), to price the barrier packet between two rounds. Prints bench.py's
JSON line."""
import sys

sys.path.insert(0, ".")
from omldm_amd.ops import linear as L  # noqa: E402

_prep = L.linear_scan3_prepare


def prep_nowait(*a, **k):
    sp = _prep(*a, **k)
    sp.event = None
    return sp


L.linear_scan3_prepare = prep_nowait
import bench  # noqa: E402

sys.exit(bench.main(sys.argv[1:]))
