"""Host read-path probe: pread from page-cached files into pageable vs pinned memory,
1 / 8 threads (8 files), the staging pattern of engine.ingest.TickIngest."""
import concurrent.futures as cf
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omldm_amd.ops import native  # noqa: E402

d = tempfile.mkdtemp(prefix="pread_", dir="/tmp")
N, SZ = 8, 64 << 20
paths = []
for i in range(N):
    p = os.path.join(d, f"{i}.bin")
    with open(p, "wb") as f:
        f.write(os.urandom(SZ))
    paths.append(p)
fds = [os.open(p, os.O_RDONLY) for p in paths]
for fd in fds:  # warm the page cache
    os.pread(fd, SZ, 0)
lib = native.host()
res = {}
offs = np.zeros(2, dtype=np.int64)
used = np.zeros(1, dtype=np.int64)


def rd(fd, dst):
    # max_records 0: pure read path (no index work)
    lib.omldm_read_log(fd, 0, dst.ctypes.data, SZ, 0, offs.ctypes.data, used.ctypes.data, 0)


for kind in ("pageable", "pinned"):
    if kind == "pinned":
        bufs = [torch.empty(SZ, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(N)]
    else:
        bufs = [np.ones(SZ, dtype=np.uint8) for _ in range(N)]
    for th in (1, 8):
        ex = cf.ThreadPoolExecutor(th)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            list(ex.map(lambda i: rd(fds[i], bufs[i]), range(N)))
            best = min(best, time.perf_counter() - t)
        ex.shutdown()
        res[f"{kind}_{th}t_GBps"] = round(N * SZ / best / 1e9, 1)
    # plain memcpy bandwidth into the same buffers (8 threads)
    src = [np.ones(SZ, dtype=np.uint8) for _ in range(N)]
    ex = cf.ThreadPoolExecutor(8)
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        list(ex.map(lambda i: ctypes.memmove(bufs[i].ctypes.data, src[i].ctypes.data, SZ), range(N)))
        best = min(best, time.perf_counter() - t)
    ex.shutdown()
    res[f"{kind}_memcpy_8t_GBps"] = round(N * SZ / best / 1e9, 1)
print(json.dumps(res))
for p in paths:
    os.unlink(p)
