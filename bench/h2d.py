"""H2D ingest microbenchmark: SDMA copies (1 or k streams) vs the GPU pull kernel
(csrc/kernels/ingest.hip) reading pinned host memory over PCIe."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omldm_amd.ops import native  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for mb in (4, 21, 64):
        n = mb << 20
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.random_(0, 255)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        t = timeit(lambda: d.copy_(h, non_blocking=True))
        res[f"sdma_1x_{mb}MB_GBs"] = round(n / t / 1e9, 1)
        for k in (2, 4):
            streams = [torch.cuda.Stream(dev) for _ in range(k)]
            cur = torch.cuda.current_stream()

            def multi():
                ch = n // k
                for i, s in enumerate(streams):
                    s.wait_stream(cur)
                    with torch.cuda.stream(s):
                        d[i * ch:(i + 1) * ch].copy_(h[i * ch:(i + 1) * ch], non_blocking=True)
                for s in streams:
                    cur.wait_stream(s)
            t = timeit(multi)
            res[f"sdma_{k}x_{mb}MB_GBs"] = round(n / t / 1e9, 1)
        for blocks in (256, 1024, 4096):
            def pull():
                native.check(native.hip().omldm_pull_copy(h.data_ptr(), d.data_ptr(), n, blocks,
                                                          torch.cuda.current_stream().cuda_stream),
                             "pull")
            t = timeit(pull)
            res[f"pull_{blocks}blk_{mb}MB_GBs"] = round(n / t / 1e9, 1)
        d2 = torch.empty(n, dtype=torch.uint8, device=dev)
        native.check(native.hip().omldm_pull_copy(h.data_ptr(), d2.data_ptr(), n, 1024,
                                                  torch.cuda.current_stream().cuda_stream), "pull")
        torch.cuda.synchronize()
        res[f"pull_correct_{mb}MB"] = bool(torch.equal(d2.cpu(), h))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
