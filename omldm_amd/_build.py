"""In-tree native build: HIP kernels for gfx950 + host C++ data plane.

Produces (git-ignored, but shipped to the GPU box by gpurun):
  omldm_amd/_native/libomldm_hip.so   every csrc/kernels/*.hip, hipcc --offload-arch=gfx950
  omldm_amd/_native/libomldm_host.so  every csrc/host/*.cpp, g++ (runs on CPU everywhere)

Usage: ``python -m omldm_amd._build [--force] [--jobs N] [--host-only]``.
Objects are cached under build/obj and rebuilt when the source or a header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
NATIVE = os.path.join(ROOT, "omldm_amd", "_native")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("OMLDM_ARCH", "gfx950")

HIP_LIB = os.path.join(NATIVE, "libomldm_hip.so")
HOST_LIB = os.path.join(NATIVE, "libomldm_host.so")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _newest_header(d: str) -> float:
    hs = glob.glob(os.path.join(d, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _stale(out: str, deps: list[float]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(d > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


# per-file extra flags: the k-means chains are issue-bound on one wave, where a packed fp32
# op costs what two plain ones do plus a wait state per dependent step (no SLP packing)
FILE_FLAGS = {"kmeans_seq.hip": ["-fno-slp-vectorize"]}


def hip_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))


def host_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))


def build_hip(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(NATIVE, exist_ok=True)
    hipcc = _hipcc()
    hdr = _newest_header(os.path.join(CSRC, "kernels"))
    objs, todo = [], []
    for src in hip_sources():
        o = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(o)
        if force or _stale(o, [os.path.getmtime(src), hdr]):
            todo.append([hipcc, "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}",
                         "-munsafe-fp-atomics", *FILE_FLAGS.get(os.path.basename(src), []),
                         "-I", os.path.join(CSRC, "kernels"), src, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, todo))
    if force or todo or _stale(HIP_LIB, [os.path.getmtime(o) for o in objs]):
        tmp = HIP_LIB + ".tmp"
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp])
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_host(force: bool = False) -> str:
    os.makedirs(NATIVE, exist_ok=True)
    srcs = host_sources()
    deps = [os.path.getmtime(s) for s in srcs] + [_newest_header(os.path.join(CSRC, "host"))]
    if force or _stale(HOST_LIB, deps):
        cxx = os.environ.get("CXX", "g++")
        tmp = HOST_LIB + ".tmp"
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall",
              "-I", os.path.join(CSRC, "host"), *srcs, "-o", tmp, "-lz", "-ldl"])
        os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build(force: bool = False, jobs: int = 8, host_only: bool = False) -> None:
    build_host(force)
    if not host_only:
        build_hip(force, jobs)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--host-only", action="store_true")
    a = ap.parse_args(argv)
    build(a.force, a.jobs, a.host_only)
    print("built:", HOST_LIB, "" if a.host_only else HIP_LIB)
    return 0


if __name__ == "__main__":
    sys.exit(main())
