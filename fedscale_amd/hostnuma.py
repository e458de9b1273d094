"""Host NUMA placement of the thread that stages uploads for a GPU.

The aggregator's main thread (event_monitor, aggregator.py:965-1007) gathers every upload into pinned host
memory, and the GPU reads it over PCIe: an H2D copy, or the zero-copy round's kernel (fa_reduce_mirror).  Linux
allocates those pinned pages on the NUMA node of the thread that first touches them, so a main thread running
on the socket far from the GPU puts the staging there, and every PCIe read crosses the socket link.  Measured
on an MI355X box whose GPU 0 sits on node 0 (tools/numa_probe.py, profiles/r03_numa_probe.log): config 1's
round takes 0.113 ms with the process on node 0 and 0.120 ms on node 1.

``bind_to_gpu(device)`` restricts the calling thread's CPU affinity to the CPUs of the GPU's NUMA node (within
the CPUs the process may use); threads it starts later inherit it.  It does nothing where the node cannot be
determined (no sysfs entry, no GPU, a single node) or where none of that node's CPUs is allowed.
"""
from __future__ import annotations

import glob
import os
from typing import Optional, Set


def _cpulist(text: str) -> Set[int]:
    out: Set[int] = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_node(device) -> Optional[int]:
    """NUMA node of the GPU's PCI device (sysfs), or None."""
    try:
        import torch

        idx = torch.device(device).index if not isinstance(device, int) else device
        p = torch.cuda.get_device_properties(0 if idx is None else idx)
        path = "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        node = int(open(path).read())
    except Exception:
        return None
    return node if node >= 0 else None


def node_cpus(node: int) -> Set[int]:
    try:
        return _cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read())
    except OSError:
        return set()


def bind_to_gpu(device, match_torch_threads: bool = False, log: bool = False) -> Optional[int]:
    """Bind the calling thread to the CPUs of ``device``'s NUMA node; returns the node, or None if unchanged.
    ``match_torch_threads``: lower torch's intra-op thread count to the node's CPUs (threads started later
    inherit the affinity, so a larger pool would oversubscribe the node); ``log``: report the binding."""
    if len(glob.glob("/sys/devices/system/node/node[0-9]*")) < 2:
        return None
    node = gpu_numa_node(device)
    if node is None:
        return None
    allowed = os.sched_getaffinity(0)
    cpus = node_cpus(node) & allowed
    if not cpus:
        return None
    if cpus != allowed:
        os.sched_setaffinity(0, cpus)
    if match_torch_threads:
        import torch

        if torch.get_num_threads() > len(cpus):
            torch.set_num_threads(len(cpus))
    if log:
        import logging

        logging.getLogger(__name__).info("bound the staging thread to NUMA node %d (%d CPUs) of %s", node,
                                         len(cpus), device)
    return node
