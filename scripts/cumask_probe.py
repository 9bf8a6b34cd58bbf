"""Which XCD / SE / CU a CU-mask bit selects: one single-bit-mask stream per bit, one
workgroup on it reading HW_REG_XCC_ID and HW_REG_HW_ID (csrc/kernels/ingest.hip:
cu_probe_kernel). Prints the bit → XCD map's summary (round-robin c % 8 or blocked
c // 32) and writes the table to gpurun_out/cumask_map.json."""
import json
import os

import torch

from omldm_amd.ops import native
from omldm_amd.ops.ingest import cumask_stream


def main():
    dev = torch.device("cuda:0")
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(2, dtype=torch.int32, device=dev)
    rows = []
    for c in range(total):
        st, raw = cumask_stream({c}, total, dev)
        native.check(native.hip().omldm_cu_probe(out.data_ptr(), raw), "cu_probe")
        st.synchronize()
        xcc, hw = (int(v) for v in out.cpu())
        rows.append({"bit": c, "xcc": xcc & 0xF, "cu": (hw >> 8) & 0xF, "sh": (hw >> 12) & 1,
                     "se": (hw >> 13) & 0x7})
        native.hip().omldm_stream_destroy(raw)
    rr = sum(r["xcc"] == r["bit"] % 8 for r in rows)
    blk = sum(r["xcc"] == r["bit"] // max(1, total // 8) for r in rows)
    print(json.dumps({"cus": total, "round_robin_matches": rr, "blocked_matches": blk,
                      "first": rows[:12]}))
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(rows, open("gpurun_out/cumask_map.json", "w"))


if __name__ == "__main__":
    main()
