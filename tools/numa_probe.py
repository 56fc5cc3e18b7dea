"""Where the GPU sits relative to this process's CPUs: the allowed CPU set,
the GPU's PCI address, NUMA node and local CPU list (sysfs)."""
import json
import os

import torch

props = torch.cuda.get_device_properties(0)
bus = getattr(props, "pci_bus_id", None)
dom = getattr(props, "pci_domain_id", 0)
dev = getattr(props, "pci_device_id", 0)
addr = f"{dom:04x}:{bus:02x}:{dev:02x}.0" if bus is not None else None
out = {"cpu_count": os.cpu_count(), "allowed": len(os.sched_getaffinity(0)), "pci": addr,
       "allowed_list": sorted(os.sched_getaffinity(0))[:8]}
if addr:
    base = f"/sys/bus/pci/devices/{addr}"
    for f in ("numa_node", "local_cpulist"):
        try:
            out[f] = open(f"{base}/{f}").read().strip()
        except OSError as e:
            out[f] = str(e)
try:
    out["nodes"] = {n: open(f"/sys/devices/system/node/{n}/cpulist").read().strip()
                    for n in sorted(os.listdir("/sys/devices/system/node")) if n.startswith("node")}
except OSError as e:
    out["nodes"] = str(e)
print(json.dumps(out))
