"""Row-stride (ld) sensitivity of one fa_reduce window: 1000 clients x 6.25M columns (one round of 32-wide tiles,
the shape of every headline window) with rows ld floats apart, interleaved in one process.
usage: python tools/ld_probe.py [rounds]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedscale_amd import kernels as kx

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    K, P = 1000, 6_250_048
    lds = [6_250_048, 6_250_048 + 1024, 12_500_032, 12_500_032 + 1024, 25_000_000, 25_000_000 + 1024]
    x = torch.empty(K * max(lds), device="cuda")
    x.uniform_()
    out = torch.empty(P, device="cuda")
    times = {ld: [] for ld in lds}
    for _ in range(rounds):
        for ld in lds:
            v = x[:K * ld].view(K, ld)
            kx.reduce(v, K, P, out, denom=float(K), finalize=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                kx.reduce(v, K, P, out, denom=float(K), finalize=True)
            e1.record()
            torch.cuda.synchronize()
            times[ld].append(e0.elapsed_time(e1) / 3)
    b = 4 * K * P + 4 * P
    print(json.dumps({"K": K, "P": P, **{f"ld{ld}": {"ms": round(float(np.median(t)), 3),
                                                     "GBps": round(b / (np.median(t) * 1e-3) / 1e9, 1)}
                                         for ld, t in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
