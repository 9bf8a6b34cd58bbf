"""Summarise a rocprofv3 CSV kernel (+ memory-copy) trace: per-kernel totals and, for the
steady state, per-step GPU busy time vs wall time (gaps = launch/host overhead)."""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    if "<" in n:
        n = n.split("<")[0]
    return n.replace("void ", "").replace("omldm::", "")[:60]


def main(d: str, marker: str = "linear_round_kernel"):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
          for r in rows]
    try:
        for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "COPY_" + r.get("Direction", r.get("Kind", ""))))
    except FileNotFoundError:
        pass
    ev.sort()
    tot = defaultdict(lambda: [0, 0])
    for a, b, n in ev:
        tot[n][0] += 1
        tot[n][1] += b - a
    print(f"{'kernel/copy':62s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s}")
    for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
        print(f"{n:62s} {c:6d} {t/1e3:10.1f} {t/c/1e3:9.2f}")
    starts = [a for a, b, n in ev if marker in n]
    if len(starts) > 6:
        s0, s1 = starts[-6], starts[-1]
        busy = 0
        cur_end = s0
        for a, b, n in ev:
            if a < s0 or a >= s1 or n.startswith("COPY"):
                continue
            a2 = max(a, cur_end)
            if b > a2:
                busy += b - a2
                cur_end = b
        print(f"\nlast 5 steps: wall {(s1 - s0)/5e3:.1f} us/step, kernel-busy "
              f"{busy/5e3:.1f} us/step")


if __name__ == "__main__":
    main(*sys.argv[1:])
