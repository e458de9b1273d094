"""Config 5's chain cost as bench.py's default line measures it (bench.config_line: the chain form's timed region, then
chain / chain-free rounds alternating over the same resident uploads).  usage: python tools/chain_pair.py [P ...]"""
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
    for P in [int(a) for a in sys.argv[1:]] or [100_000_000, 12_500_000]:
        cfg = dict(bench.CONFIGS["c5"], params=P)
        steps = 2 if P > 50_000_000 else 3
        r = bench.config_line("c5", cfg, dev, 0, 1, ShardGroup(0, 1), 2024, "gloo", steps=steps, warmup=1)
        print(json.dumps({"params": P, "round_ms": r["round_ms"], "dominant_kernel_ms": r["dominant_kernel_ms"],
                          "no_chain": r.get("no_chain")}), flush=True)


if __name__ == "__main__":
    main()
