"""Host threads on the GPU's own NUMA node.

The step is dispatch-bound: the command processor fetches every AQL packet
(and the graphs' kernel arguments) from host memory, and the fresh-batch /
sweep legs are host-bound.  On a two-socket host a process left to the
scheduler runs its threads -- and first-touches its pinned buffers and queue
rings -- on either node, and the remote one adds a socket hop to every fetch.
``bind_to_device_numa`` restricts the calling thread (and every thread it
starts afterwards: the loader, the intra-op pool) to the CPUs sysfs lists as
local to the device's PCI function, intersected with the CPUs it is allowed.
"""
from __future__ import annotations

import os
from typing import List, Optional, Set

import torch


def _parse_cpulist(text: str) -> Set[int]:
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def device_local_cpus(device) -> Optional[Set[int]]:
    """CPUs local to ``device``'s PCI function (sysfs local_cpulist), or None."""
    idx = torch.device(device).index
    props = torch.cuda.get_device_properties(0 if idx is None else idx)
    bus = getattr(props, "pci_bus_id", None)
    if bus is None:
        return None
    addr = f"{getattr(props, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(props, 'pci_device_id', 0):02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{addr}/local_cpulist") as f:
            return _parse_cpulist(f.read())
    except (OSError, ValueError):
        return None


def bind_to_device_numa(device) -> Optional[List[int]]:
    """Restrict the calling thread to ``device``'s local CPUs; returns them,
    or None (unknown topology, or none of them allowed: left unchanged)."""
    local = device_local_cpus(device)
    if not local:
        return None
    cpus = local & os.sched_getaffinity(0)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return sorted(cpus)
