"""Is config 5's one-GPU chain cost a power-cap effect?  The chain form and the chain-free kernel over the same
resident uploads (bench.Workload, share_inputs), each run back to back for its own region, alternating, with the
card's power and shader clock sampled per region.  If the chain rounds draw more power at the 1400 W cap, their
shader clock sits lower than the chain-free rounds'.  usage: python tools/chain_power_probe.py [P] [seconds] [HBM budget fraction for the resident uploads]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd.cardstate import CardSampler  # noqa: E402
from fedscale_amd.state import ShardGroup  # noqa: E402


def region(w, dev, seconds, tag):
    s = CardSampler(dev, period_s=0.02)
    ms = []
    torch.cuda.synchronize(dev)
    s.start()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        w.step(e)
        torch.cuda.synchronize(dev)
        ms.append(e[0].elapsed_time(e[1]))
    card = s.stop().summary()
    rec = {"region": tag, "rounds": len(ms), "round_ms": [round(m, 3) for m in ms],
           "mean_ms": sum(ms) / len(ms), "tb_s": w.alg_bytes / (sum(ms) / len(ms) * 1e-3) / 1e12,
           "card": {k: round(v["mean"], 2) for k, v in card.items() if isinstance(v, dict)}}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    budget = float(sys.argv[3]) if len(sys.argv) > 3 else bench.MEM_FRACTION
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = dict(bench.CONFIGS["c5"], params=P)
    sh = ShardGroup(0, 1)
    wc = bench.Workload(cfg["policy"], cfg["clients"], cfg["params"], 0, 1, dev, 2024, sh,
                        budget_fraction=budget, mean_chain=True)
    wf = bench.Workload(cfg["policy"], cfg["clients"], cfg["params"], 0, 1, dev, 2024, sh,
                        budget_fraction=budget, mean_chain=False, share_inputs=wc)
    print(json.dumps({"params": P, "budget_fraction": budget, "resident_clients": wc.C, "passes": len(wc.passes)}),
          flush=True)
    wc.step()
    wf.step()
    out = {"chain": [], "free": []}
    for rep in range(3):
        out["chain"].append(region(wc, dev, seconds, f"chain_r{rep}"))
        out["free"].append(region(wf, dev, seconds, f"free_r{rep}"))
    mc = sum(r["mean_ms"] for r in out["chain"]) / 3
    mf = sum(r["mean_ms"] for r in out["free"]) / 3
    pc = sum(r["card"].get("power_w", 0) for r in out["chain"]) / 3
    pf = sum(r["card"].get("power_w", 0) for r in out["free"]) / 3
    sc = sum(r["card"].get("sclk_mhz", 0) for r in out["chain"]) / 3
    sf = sum(r["card"].get("sclk_mhz", 0) for r in out["free"]) / 3
    print(json.dumps({"chain_cost_pct": 100 * (mc / mf - 1), "power_w": [pc, pf], "sclk_mhz": [sc, sf]}), flush=True)
    wf.xs = []
    wf.free()
    wc.free()


if __name__ == "__main__":
    main()
