"""q-FedAvg phase 1 (fa_qfed_accumulate) against the FedAvg reduce (fa_reduce, FA_FINALIZE) on the SAME resident
1000 x 25M updates, interleaved in one process: the two kernels' rates on one box, so box-to-box HBM spread
cancels out of their ratio.  usage: python tools/qfed_vs_reduce.py [K] [P] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=3)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=4, scale_noise=0.0)
    last = last[0]
    alpha = torch.rand(K, device="cuda") + 0.5
    delta = torch.empty(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = kx.qfed_workspace(K, "cuda")
    out = torch.empty(ld, device="cuda")
    denom = float(np.float32(K))

    def qfed():
        kx.qfed_accumulate(x, K, P, last=last, alpha=alpha, lr=0.05, delta=delta, sqnorm=sq, workspace=ws,
                           accumulate=False)

    def fedavg():
        kx.reduce(x, K, P, out, denom=denom, finalize=True)

    runs = {"qfedavg": (qfed, 4 * K * P + 8 * P + 8 * K), "fedavg": (fedavg, 4 * K * P + 4 * P)}
    times = {n: [] for n in runs}
    for _ in range(rounds):
        for n, (f, _) in runs.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
    res = {"K": K, "P": P, "rounds": rounds}
    for n, (_, b) in runs.items():
        ms = float(np.median(times[n]))
        res[n] = {"ms": round(ms, 3), "GBps": round(b / (ms * 1e-3) / 1e9, 1)}
    res["qfedavg_over_fedavg_rate"] = round(res["qfedavg"]["GBps"] / res["fedavg"]["GBps"], 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
