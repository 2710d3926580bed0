"""Per-rank CPU / NUMA affinity: pin a rank's host threads next to its GPU.

Each rank's host side (frame feeder, record unpack, RPC on rank 0, pinned staging
buffers) should run on the CPU socket the GPU hangs off, so its H2D/D2H traffic and
page-locked buffers stay NUMA-local. This must happen BEFORE the process touches the
GPU (pinned allocations are placed by first touch of the allocating thread) and without
initialising HIP (which ``hipDeviceGetPCIBusId`` would do), so the GPU -> PCI -> NUMA
mapping is read from sysfs:

  * KFD topology (``/sys/class/kfd/kfd/topology/nodes/*``): GPU nodes in the order the
    ROCm runtime enumerates them, each with its PCI ``domain`` and ``location_id``
    (bus << 8 | device << 3 | function);
  * ``/sys/bus/pci/devices/<bdf>/numa_node`` and ``/sys/devices/system/node/node<n>/cpulist``.

``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` (numeric lists) remap the local rank.
The reference has one process and one accelerator (/root/reference/sem_seg_server.py:264).
"""
from __future__ import annotations

import glob
import logging
import os
from typing import List, Optional, Set

log = logging.getLogger(__name__)


def parse_cpulist(s: str) -> Set[int]:
    out: Set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def gpu_pci_addresses(sysfs: str = "/sys") -> List[str]:
    """PCI addresses of the GPUs in ROCm enumeration order (KFD topology node order)."""
    out = []
    nodes = sorted(glob.glob(os.path.join(sysfs, "class/kfd/kfd/topology/nodes/*")),
                   key=lambda p: int(os.path.basename(p)))
    for n in nodes:
        props = _read(os.path.join(n, "properties"))
        if not props:
            continue
        kv = {}
        for line in props.splitlines():
            parts = line.split()
            if len(parts) == 2:
                kv[parts[0]] = int(parts[1])
        if kv.get("simd_count", 0) <= 0:  # CPU node
            continue
        loc, dom = kv.get("location_id", 0), kv.get("domain", 0)
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}")
    return out


def gpu_numa_node(local_rank: int, sysfs: str = "/sys") -> Optional[int]:
    addrs = gpu_pci_addresses(sysfs)
    vis = os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
    idx = local_rank
    if vis:
        try:
            ids = [int(v) for v in vis.split(",") if v.strip()]
            idx = ids[local_rank]
        except (ValueError, IndexError):
            return None
    if idx >= len(addrs):
        return None
    v = _read(os.path.join(sysfs, "bus/pci/devices", addrs[idx], "numa_node"))
    if v is None:
        return None
    n = int(v.strip())
    return n if n >= 0 else None


def pin_to_gpu_numa(local_rank: Optional[int] = None, sysfs: str = "/sys") -> Optional[Set[int]]:
    """Restrict this process to the CPUs of its GPU's NUMA node (intersected with the
    current affinity). Returns the CPU set applied, or None when unknown / disabled
    (SSA_NUMA_PIN=0) / already narrower."""
    if os.environ.get("SSA_NUMA_PIN", "1") == "0":
        return None
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    node = gpu_numa_node(local_rank, sysfs)
    if node is None:
        return None
    cl = _read(os.path.join(sysfs, f"devices/system/node/node{node}/cpulist"))
    if not cl:
        return None
    want = parse_cpulist(cl)
    cur = os.sched_getaffinity(0)
    new = want & cur
    if not new or new == cur:
        return None
    os.sched_setaffinity(0, new)
    log.info("local rank %d: GPU on NUMA node %d -> %d CPUs", local_rank, node, len(new))
    return new
