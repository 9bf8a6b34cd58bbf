"""Timeline of one engine tick from a rocprofv3 --kernel-trace --marker-trace CSV run:
host roctx ranges and GPU kernels between two consecutive ``poll`` ranges, in µs
relative to the tick start. Usage: tick_timeline.py <dir> [tick index]"""
import csv
import glob
import sys


def rows(d, suffix):
    f = glob.glob(f"{d}/**/*{suffix}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main(d, k=10):
    mk = rows(d, "marker_api_trace.csv")
    kt = rows(d, "kernel_trace.csv")
    if not mk:
        print("no marker trace")
        return
    name_key = "Function" if "Function" in mk[0] else [c for c in mk[0] if "Name" in c or "Function" in c][0]
    polls = sorted(int(r["Start_Timestamp"]) for r in mk if r[name_key] == "poll")
    if len(polls) < k + 2:
        k = max(0, len(polls) - 2)
    t0, t1 = polls[k], polls[k + 1]
    ev = []
    for r in mk:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= a < t1:
            ev.append((a, b, "HOST " + r[name_key]))
    for r in kt:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= a < t1 + 2_000_000:
            n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            ev.append((a, b, "GPU  " + n))
    ev.sort()
    print(f"tick {k}: {(t1 - t0) / 1e3:.1f} us")
    for a, b, n in ev:
        if a >= t1:
            break
        print(f"{(a - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
