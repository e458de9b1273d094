"""FedYoGi at 1000 x 25 M on one box, interleaved in one process: the fused epilogue (fa_reduce_yogi, what the
drop-in runs), the same step unfused (fa_reduce FA_FINALIZE into the mean, then fa_yogi_step), and plain FedAvg
(fa_reduce FA_FINALIZE) for reference.  The fused and unfused outputs must be the same bits.
usage: python tools/yogi_ab.py [K] [P] [rounds]"""
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
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=5)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=6, scale_noise=0.0)
    last = last[0]
    hp = dict(eta=float(np.float32(3e-3)), tau=float(np.float32(1e-8)), beta=float(np.float32(0.9)),
              omb=float(np.float32(0.1)), omb2=float(np.float32(0.01)))
    m0, v0 = torch.zeros(ld, device="cuda"), torch.full((ld,), 1e-8, device="cuda")
    bufs = {n: (m0.clone(), v0.clone(), torch.empty(ld, device="cuda"), torch.empty(ld, device="cuda"))
            for n in ("fused", "unfused")}
    out_avg = torch.empty(ld, device="cuda")
    den = float(np.float32(K))

    def fused():
        m, v, out, mean = bufs["fused"]
        kx.reduce_yogi(x, K, P, last=last, m=m, v=v, out=out, denom=den, init=False, mean_out=mean, **hp)

    def unfused():
        m, v, out, mean = bufs["unfused"]
        kx.reduce(x, K, P, mean, denom=den, finalize=True)
        kx.yogi_step(mean, last, m, v, out, P, init=False, **hp)

    def fedavg():
        kx.reduce(x, K, P, out_avg, denom=den, finalize=True)

    fns = {"fused": fused, "unfused": unfused, "fedavg": fedavg}
    for f in fns.values():  # one identical step each: fused and unfused must agree bit for bit
        f()
    torch.cuda.synchronize()
    for i in range(4):
        assert torch.equal(bufs["fused"][i], bufs["unfused"][i]), f"fused and unfused differ in buffer {i}"
    times = {n: [] for n in fns}
    for _ in range(rounds):
        for n, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
    print(f"--- K={K} P={P}: GB/s over 4KP + 24P (FedYoGi) / 4KP + 4P (FedAvg)")
    for n in sorted(times, key=lambda n: np.median(times[n])):
        ms = float(np.median(times[n]))
        alg = 4 * K * P + (4 * P if n == "fedavg" else 24 * P)
        print(f"{n:10s} {ms:8.3f} ms {alg / (ms * 1e-3) / 1e9:9.1f} GB/s  (min {min(times[n]):.3f})", flush=True)


if __name__ == "__main__":
    main()
