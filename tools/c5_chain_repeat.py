import json, sys, os
sys.path.insert(0, os.getcwd())
import torch
import bench
from fedscale_amd.state import ShardGroup
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
sh = ShardGroup(0, 1)
for i in range(3):
    r = bench.config_line("c5", bench.CONFIGS["c5"], dev, 0, 1, sh, 0, "nccl", steps=2, warmup=1)
    print(json.dumps({"kern_ms": round(r["dominant_kernel_ms"], 1), "gbps": round(r["hbm_gbps_kernel"]),
                      "no_chain_ms": round(r["no_chain"]["dominant_kernel_ms"], 1),
                      "chain_cost_pct": round(r["no_chain"]["chain_cost_pct"], 2)}), flush=True)
