"""Interleaved timing of fa_qfed_accumulate variants (fedscale_amd/variants/libfedagg_qf_*.so) in one process.
usage: python tools/tune_qfed.py [K] [P] [rounds]"""
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
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    V, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "libfedagg_qf_*.so"))) + [
            os.path.join(ROOT, "fedscale_amd", "libfedagg.so")]:
        lib = ctypes.CDLL(path)
        f = lib.fa_qfed_accumulate
        f.restype = I32
        f.argtypes = [V, I64, I32, I64, V, V, F, V, V, V, I32, V]
        libs[os.path.basename(path)] = f
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=3)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=3 + 90000, scale_noise=0.0)
    alpha = torch.rand(K, device="cuda") + 0.5
    delta = torch.empty(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = torch.empty(4096 * K, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    times = {n: [] for n in libs}
    ref = None
    for r in range(rounds):
        for n, f in libs.items():
            args = (x.data_ptr(), ld, K, P, last.data_ptr(), alpha.data_ptr(), 0.05, delta.data_ptr(), sq.data_ptr(),
                    ws.data_ptr(), 0, st)
            assert f(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f(*args)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
            if ref is None:
                ref = delta.clone()
            else:
                assert torch.equal(delta, ref), f"{n}: delta differs"
    b = 4 * K * P + 8 * P
    print(f"--- K={K} P={P}")
    for n, t in sorted(times.items(), key=lambda kv: np.median(kv[1])):
        print(f"{n:44s} {np.median(t):8.3f} ms {b / (np.median(t) * 1e-3) / 1e9:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
