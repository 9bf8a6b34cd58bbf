"""Kernel statistics from a rocprofv3 rocpd SQLite database (-o … without a CSV format):
per kernel name — calls, total / mean / min / max µs, share of the summed kernel time.
Usage: python scripts/rocpd_stats.py DB [--grep SUBSTR] [--csv OUT]"""
import argparse
import csv
import sqlite3
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grep", default="")
    ap.add_argument("--csv", default="")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        if a.grep and a.grep not in n:
            continue
        d = (e - s) / 1e3
        v = agg.setdefault(n, [0, 0.0, 1e30, 0.0])
        v[0] += 1
        v[1] += d
        v[2] = min(v[2], d)
        v[3] = max(v[3], d)
    tot = sum(v[1] for v in agg.values()) or 1.0
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    w = csv.writer(open(a.csv, "w") if a.csv else sys.stdout)
    w.writerow(["Name", "Calls", "TotalUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
    for n, (k, t, lo, hi) in out:
        w.writerow([n[:120], k, round(t, 2), round(t / k, 2), round(lo, 2), round(hi, 2),
                    round(100 * t / tot, 2)])


if __name__ == "__main__":
    main()
