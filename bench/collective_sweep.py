#!/usr/bin/env python3
"""Collective sweep for the worker↔hub transport (SURVEY.md §5.8 "bucket sizing", §7.2
``rccl_bucket_sweep``): what one parameter-server round costs over RCCL/xGMI as a
function of message size, hub layout and bucket size.

Three sweeps, all through ``omldm_amd.parallel.comm.Comm`` (the code the protocols use):

* ``op``      — one buffer of each size through every hub layout of the reference's
                HubParallelism: all-reduce (H = G), reduce + broadcast (H = 1),
                per-hub-slice reduce + broadcast (1 < H < G), plus the reduce-scatter /
                all-gather halves. Reports algbw = bytes / time and the ring bus
                bandwidth busbw = algbw · 2(G−1)/G (nccl-tests convention).
* ``bucket``  — M pipeline accumulators of one size synced in one round through
                ``all_reduce_coalesced_`` with ``--bucketBytes`` caps (the Job's
                Synchronous grouping): how the cap trades staging copies for fewer
                collectives.
* ``parts``   — one [dim + 2] round accumulator all-reduced as K key-range slices issued
                back to back (the collective side of Synchronous ``reduceParts``).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collective_sweep.py
    python bench/collective_sweep.py --sizes 65536,4194304       # one rank: timings only
Each measurement prints one JSON line on rank 0 (max over ranks of the mean time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omldm_amd.parallel.comm import init_distributed  # noqa: E402


def _sync(comm, device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    comm.barrier()


def _time(comm, device, fn, iters: int, warmup: int) -> float:
    """Mean seconds per call, max over ranks."""
    for _ in range(warmup):
        fn()
    _sync(comm, device)
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(comm, device)
    el = torch.tensor([(time.perf_counter() - t) / iters], dtype=torch.float64,
                      device=device if comm.backend == "nccl" else "cpu")
    if comm.world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def _emit(comm, rec: dict) -> None:
    if comm.rank == 0:
        print(json.dumps(rec), flush=True)


def sweep_ops(comm, device, sizes, dtype, iters, warmup):
    G = comm.world
    for nbytes in sizes:
        n = max(1, nbytes // torch.tensor([], dtype=dtype).element_size())
        t = torch.ones(n, dtype=dtype, device=device)
        ops = {"all_reduce (H=G)": lambda: comm.hub_reduce_(t, 0, "sweep"),
               "reduce+bcast (H=1)": lambda: comm.hub_reduce_(t, 1, "sweep")}
        if G > 2:
            ops[f"sharded (H={G // 2})"] = lambda: comm.hub_reduce_(t, G // 2, "sweep")
        if G > 1:
            shard = torch.empty(-(-n // G), dtype=dtype, device=device)
            full = torch.empty(shard.numel() * G, dtype=dtype, device=device)
            full[:n].copy_(t)
            ops["reduce_scatter"] = lambda: dist.reduce_scatter_tensor(shard, full,
                                                                       group=comm.group)
            ops["all_gather"] = lambda: dist.all_gather_into_tensor(full, shard,
                                                                    group=comm.group)
        for name, fn in ops.items():
            s = _time(comm, device, fn, iters, warmup)
            algbw = nbytes / s / 1e9
            _emit(comm, {"sweep": "op", "op": name, "bytes": nbytes, "world": G,
                         "us": round(s * 1e6, 2), "algbw_GBps": round(algbw, 2),
                         "busbw_GBps": round(algbw * 2 * (G - 1) / G, 2) if G > 1 else None,
                         "backend": comm.backend})


def sweep_buckets(comm, device, pipelines, dim, caps, dtype, iters, warmup):
    bufs = [torch.ones(dim + 2, dtype=dtype, device=device) for _ in range(pipelines)]
    total = sum(b.numel() * b.element_size() for b in bufs)
    for cap in caps:
        s = _time(comm, device,
                  lambda: comm.all_reduce_coalesced_(bufs, "sweep", 0, bucket_bytes=cap),
                  iters, warmup)
        _emit(comm, {"sweep": "bucket", "pipelines": pipelines, "dim": dim,
                     "bucket_bytes": cap, "total_bytes": total, "world": comm.world,
                     "us": round(s * 1e6, 2), "algbw_GBps": round(total / s / 1e9, 2),
                     "backend": comm.backend})


def sweep_parts(comm, device, dim, parts_list, iters, warmup):
    from omldm_amd.ops.linear import part_bounds

    buf = torch.ones(dim + 2, dtype=torch.float32, device=device)
    for parts in parts_list:
        sl = [part_bounds(dim, k, parts, cuda=device.type == "cuda") for k in range(parts)]

        def run():
            works = [comm.all_reduce_(buf[lo:hi], "sweep", async_op=True)
                     for lo, hi in sl if hi > lo]
            for w in works:
                if w is not None:
                    w.wait()

        s = _time(comm, device, run, iters, warmup)
        _emit(comm, {"sweep": "parts", "dim": dim, "parts": parts, "world": comm.world,
                     "us": round(s * 1e6, 2), "backend": comm.backend})


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,262144,1048576,2097152,4194304,16777216,67108864")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pipelines", type=int, default=16)
    ap.add_argument("--dim-log2", type=int, default=20)
    ap.add_argument("--caps", default="4194304,8388608,16777216,33554432,67108864")
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--sweeps", default="op,bucket,parts")
    a = ap.parse_args(argv)
    comm, device = init_distributed()
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    which = set(a.sweeps.split(","))
    if "op" in which:
        sweep_ops(comm, device, [int(x) for x in a.sizes.split(",")], dtype, a.iters, a.warmup)
    if "bucket" in which:
        sweep_buckets(comm, device, a.pipelines, 1 << a.dim_log2,
                      [int(x) for x in a.caps.split(",")], dtype, a.iters, a.warmup)
    if "parts" in which:
        sweep_parts(comm, device, 1 << a.dim_log2, [int(x) for x in a.parts.split(",")],
                    a.iters, a.warmup)
    if comm.world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
