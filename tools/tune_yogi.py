"""Interleaved A/B timing of fa_reduce_yogi (fused FedAvg + FedYoGi) variants in ONE process
(fedscale_amd/variants/*.so + libfedagg.so).  usage: python tools/tune_yogi.py [K] [P] [rounds]"""
import ctypes
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    V, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "*.so"))) + [
            os.path.join(ROOT, "fedscale_amd", "libfedagg.so")]:
        f = ctypes.CDLL(path).fa_reduce_yogi
        f.restype = I32
        f.argtypes = [V, I64, I32, I64, V, V, F, V, V, V, V, V, F, F, F, F, F, I32, V]
        libs[os.path.basename(path)] = f
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=5)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=6, scale_noise=0.0)
    m = torch.zeros(ld, device="cuda")
    v = torch.full((ld,), 1e-8, device="cuda")
    out = torch.empty(ld, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    hp = (float(np.float32(3e-3)), float(np.float32(1e-8)), float(np.float32(0.9)), float(np.float32(0.1)),
          float(np.float32(0.01)))
    times = {n: [] for n in libs}
    for _ in range(rounds):
        for n, f in libs.items():
            def call():
                assert f(x.data_ptr(), ld, K, P, None, None, float(K), last.data_ptr(), m.data_ptr(), v.data_ptr(),
                         out.data_ptr(), None, *hp, 2, st) == 0
            call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                call()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
    alg = 4 * K * P + 24 * P
    print(f"--- fa_reduce_yogi K={K} P={P}")
    for n in sorted(times, key=lambda n: np.median(times[n])):
        ms = float(np.median(times[n]))
        print(f"{n:40s} {ms:8.3f} ms {alg / (ms * 1e-3) / 1e9:9.1f} GB/s")


if __name__ == "__main__":
    main()
