"""Aggregate a rocprofv3 `--pmc` counter_collection.csv per kernel (sum over dispatches)
and print derived ratios when their inputs are present."""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    if "<" in n:
        n = n.split("<")[0]
    return n.replace("void ", "").replace("omldm::", "")[:48]


def main(path: str):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r.get("Kernel_Name", "?"))
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    names = sorted({c for v in tot.values() for c in v})
    print("kernel".ljust(50), "disp", *[c[:22].rjust(23) for c in names])
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(k.ljust(50), str(len(disp[k])).rjust(4), *[f"{v.get(c, 0):23.4g}" for c in names])
    print()
    for k, v in tot.items():
        out = []
        if v.get("SQ_WAVE_CYCLES"):
            w = v["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in v:
                    out.append(f"{c[3:]}={v[c] / w:.2f}")
        if v.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"LDS_conflict_frac={v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "TCC_HIT_sum" in v and (v["TCC_HIT_sum"] + v.get("TCC_MISS_sum", 0)):
            out.append(f"L2_hit={v['TCC_HIT_sum'] / (v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.2f}")
        if "FETCH_SIZE" in v:
            out.append(f"fetch_MB/disp={2 * v['FETCH_SIZE'] / 1024 / max(1, len(disp[k])):.1f}(x2 rule)")
        if v.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            out.append(f"MFMA_busy_per_GUI={v['SQ_VALU_MFMA_BUSY_CYCLES'] / v['GRBM_GUI_ACTIVE']:.3f}")
        if out:
            print(k.ljust(50), " ".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
