"""Config 5's chain cost as bench.py's default line measures it (bench.config_line: the chain form's timed region, then
chain / chain-free rounds alternating over the same resident uploads).
usage: python tools/chain_pair.py [P ...] [budget=F]   (F: HBM fraction for the resident uploads, bench.MEM_FRACTION)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import torch

    from fedscale_amd.state import ShardGroup

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    budget = bench.MEM_FRACTION
    sizes = []
    for a in sys.argv[1:]:
        if a.startswith("budget="):
            budget = float(a.split("=", 1)[1])
        else:
            sizes.append(int(a))
    for P in sizes or [100_000_000, 12_500_000]:
        cfg = dict(bench.CONFIGS["c5"], params=P)
        steps = 2 if P > 50_000_000 else 3
        r = bench.config_line("c5", cfg, dev, 0, 1, ShardGroup(0, 1), 2024, "gloo", steps=steps, warmup=1,
                              budget_fraction=budget)
        print(json.dumps({"params": P, "budget_fraction": budget, "resident_clients": r["resident_clients"],
                          "passes": r["passes"], "round_ms": r["round_ms"], "dominant_kernel_ms": r["dominant_kernel_ms"],
                          "no_chain": r.get("no_chain")}), flush=True)


if __name__ == "__main__":
    main()
