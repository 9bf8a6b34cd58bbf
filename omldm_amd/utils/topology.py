"""Host topology: bind each rank to the NUMA node of its GPU.

An MI355X node has two sockets; each GPU sits behind its own PCIe root port on one of
them (measured on the pool: 4 GPUs per socket, ``/sys/class/drm/card*/device/numa_node``).
The training stream crosses PCIe every round (the pull-copy kernel reads pinned host
batches, the persistent predict wave polls a host request line), so the host pages and
the host thread that drives the GPU belong on the GPU's socket — otherwise every PCIe
read also crosses the socket interconnect.

``bind_to_device(device)`` resolves the device's PCI address (torch device properties)
to sysfs, then
* restricts the process' CPU affinity to the node-local CPUs (``local_cpulist``), and
* sets a *preferred* NUMA memory policy for the node (``set_mempolicy(MPOL_PREFERRED)``)
  so that later host allocations (pinned pools, staging rings) are node-local.
It never fails the job: anything missing (no sysfs, CPU build, foreign platform) makes
it a no-op, and ``OMLDM_NUMA_BIND=0`` turns it off.

The reference has no equivalent (Flink schedules subtasks on TaskManager slots without
placement hints — omldm/Job.scala:117).
"""
from __future__ import annotations

import ctypes
import os

_SYS_PCI = "/sys/bus/pci/devices"
_MPOL_PREFERRED = 1
_NR_SET_MEMPOLICY = 238  # x86_64


def parse_cpulist(text: str) -> list[int]:
    """'0-63,128-191' -> [0..63, 128..191]."""
    out: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def pci_address(device) -> str | None:
    import torch

    if not torch.cuda.is_available():
        return None
    idx = device.index if hasattr(device, "index") and device.index is not None else int(device)
    p = torch.cuda.get_device_properties(idx)
    dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if bus is None:
        return None
    return f"{int(dom or 0):04x}:{int(bus):02x}:{int(dev or 0):02x}.0"


def device_locality(addr: str, sys_pci: str = _SYS_PCI) -> tuple[int, list[int]] | None:
    """(numa_node, local cpus) of a PCI function, from sysfs."""
    base = os.path.join(sys_pci, addr)
    try:
        with open(os.path.join(base, "numa_node")) as f:
            node = int(f.read().strip())
        with open(os.path.join(base, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError):
        return None
    return node, cpus


def _set_preferred_node(node: int) -> bool:
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << node)
        rc = libc.syscall(_NR_SET_MEMPOLICY, _MPOL_PREFERRED, ctypes.byref(mask),
                          ctypes.c_ulong(64))
        return rc == 0
    except (OSError, AttributeError):
        return False


def bind_to_device(device, sys_pci: str = _SYS_PCI) -> dict:
    """Bind the calling process (CPU affinity + preferred memory node) to ``device``'s
    NUMA node. Returns what was done (for the job metrics / bench line)."""
    info = {"numa_node": None, "cpus": 0, "mempolicy": False}
    if os.environ.get("OMLDM_NUMA_BIND", "1") == "0":
        return info
    try:
        addr = pci_address(device)
    except Exception:  # noqa: BLE001 - placement is best effort
        addr = None
    loc = device_locality(addr, sys_pci) if addr else None
    if loc is None:
        return info
    node, cpus = loc
    try:
        allowed = os.sched_getaffinity(0)
        local = sorted(set(cpus) & allowed)
        if local:
            os.sched_setaffinity(0, local)
            info["cpus"] = len(local)
    except (OSError, AttributeError):
        pass
    if node >= 0:
        info["numa_node"] = node
        info["mempolicy"] = _set_preferred_node(node)
    return info
