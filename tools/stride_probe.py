"""Is the large-P slowdown the row STRIDE? fa_reduce over the same K x 25M columns with rows 25M, 50M or 100M
floats apart (ld), interleaved in one process.  usage: python tools/stride_probe.py [K] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedscale_amd import kernels as kx

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 231
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    P = 25_000_000
    x = torch.empty(K * 100_000_000, device="cuda")
    x.uniform_()
    out = torch.empty(P, device="cuda")
    times = {}
    for _ in range(rounds):
        for ld in (25_000_000, 50_000_000, 100_000_000):
            v = x[:K * ld].view(K, ld)
            kx.reduce(v, K, P, out, denom=float(K), finalize=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                kx.reduce(v, K, P, out, denom=float(K), finalize=True)
            e1.record()
            torch.cuda.synchronize()
            times.setdefault(ld, []).append(e0.elapsed_time(e1) / 3)
    b = 4 * K * P + 4 * P
    res = {"K": K, "P": P, **{f"ld{ld}": {"ms": round(float(np.median(t)), 3),
                                          "GBps": round(b / (np.median(t) * 1e-3) / 1e9, 1)}
                              for ld, t in times.items()}}
    # the whole 100M-column rows in ONE launch against four launches over 25M-column windows of them
    v = x[:K * 100_000_000].view(K, 100_000_000)
    big = torch.empty(100_000_000, device="cuda")
    big2 = torch.empty(100_000_000, device="cuda")

    def one():
        kx.reduce(v, K, 100_000_000, big, denom=float(K), finalize=True)

    from fedscale_amd._native import call

    st = torch.cuda.current_stream().cuda_stream

    def windows(n=4):  # the C ABI directly: a column window is x + i*w with the same ld
        w = 100_000_000 // n
        for i in range(n):
            call("fa_reduce", v.data_ptr() + 4 * i * w, 100_000_000, K, w, None, None, big2.data_ptr() + 4 * i * w,
                 float(K), kx.FA_FINALIZE, st)

    tw = {"one_launch": [], "four_windows": []}
    for _ in range(rounds):
        for name, f in (("one_launch", one), ("four_windows", windows)):
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            torch.cuda.synchronize()
            tw[name].append(e0.elapsed_time(e1) / 3)
    assert torch.equal(big, big2), "windowed result differs"
    b = 4 * K * 100_000_000 + 4 * 100_000_000
    for name, t in tw.items():
        res[f"p100M_{name}"] = {"ms": round(float(np.median(t)), 3), "GBps": round(b / (np.median(t) * 1e-3) / 1e9, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
