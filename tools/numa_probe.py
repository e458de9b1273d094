"""Host topology of the GPU box: this process's CPU affinity, the NUMA nodes' CPUs, and the NUMA node of GPU 0's PCI
device.  Then config 1's round (bench.c1_host_round) with the process bound to each NUMA node it may run on,
alternated, to see whether the placement of the pinned staging decides the zero-copy round's time.
usage: python tools/numa_probe.py [pairs]"""
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def main():
    import torch

    import bench

    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    aff = os.sched_getaffinity(0)
    nodes = {}
    for n in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        nodes[int(n.rsplit("node", 1)[1])] = cpulist(open(n + "/cpulist").read())
    p = torch.cuda.get_device_properties(0)
    bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    path = "/sys/bus/pci/devices/%s/numa_node" % bdf
    gpu_node = int(open(path).read()) if os.path.exists(path) else None
    info = {"affinity_cpus": len(aff), "nodes": {k: len(v) for k, v in nodes.items()},
            "allowed_per_node": {k: len(v & aff) for k, v in nodes.items()}, "gpu_pci": bdf, "gpu_numa_node": gpu_node}
    print(json.dumps(info), flush=True)
    usable = [k for k, v in nodes.items() if v & aff]
    dev = torch.device("cuda:0")
    res = {k: [] for k in usable}
    for _ in range(pairs):
        for k in usable:
            os.sched_setaffinity(0, nodes[k] & aff)
            res[k].append(bench.c1_host_round(dev, 0, rounds=100)["round_ms_incl_h2d_d2h"])
    os.sched_setaffinity(0, aff)
    print(json.dumps({f"node{k}": {"median_ms": round(float(np.median(v)), 4), "runs": [round(x, 4) for x in v]}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
