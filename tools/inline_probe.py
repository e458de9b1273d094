"""Why does a config read slower inside the default bench line than in a process of its own?

One process, config 5's shard of 8 (10,000 x 12.5 M q-FedAvg) timed exactly as bench.py's config_line does:
  1. fresh (the first large allocation of the process);
  2. after the other configs' workloads have been allocated, run and freed (headline, c3, c4: the line's order);
  3. the same again after a 20 s pause (the card cools; the memory stays as step 2 left it);
  4. after torch's caching allocator was emptied AND a fresh large allocation pattern (the same as 1).
Steps 1 vs 2 separate "the line's allocation history" from "the card's state"; 2 vs 3 the card's temperature.
Prints one line per step.  python tools/inline_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from fedscale_amd.state import ShardGroup

    dev = torch.device("cuda:0")
    shards = ShardGroup(0, 1)

    def c5s(tag):
        r = bench.config_line("c5s", dict(bench.CONFIGS["c5"], params=100_000_000 // 8), dev, 0, 1, shards, 2024,
                              "gloo", steps=3, warmup=1)
        print(json.dumps({"step": tag, "dominant_kernel_ms": round(r["dominant_kernel_ms"], 3),
                          "hbm_gbps_kernel": round(r["hbm_gbps_kernel"], 1), "resident": r["resident_clients"],
                          "passes": r["passes"]}), flush=True)

    def others():
        for name, cfg in (("headline", bench.CONFIGS["headline"]), ("c3", bench.CONFIGS["c3"]),
                          ("c4", bench.CONFIGS["c4"])):
            r = bench.config_line(name, cfg, dev, 0, 1, shards, 2024, "gloo", steps=5, warmup=2)
            print(json.dumps({"ran": name, "dominant_kernel_ms": round(r["dominant_kernel_ms"], 3)}), flush=True)

    c5s("1 fresh")
    others()
    c5s("2 after the other configs")
    time.sleep(20)
    c5s("3 same, after a 20 s pause")
    others()
    torch.cuda.empty_cache()
    c5s("4 after the other configs again")


if __name__ == "__main__":
    main()
