"""Interleaved A/B timing of fa_reduce variants in ONE process (cdna guide §5.4 rule 24).

usage: python tools/tune_reduce.py [K] [P] [rounds]   (variants: fedscale_amd/variants/*.so)
       python tools/tune_reduce.py sweep K1:P1,K2:P2,... [rounds]
"""
import ctypes
import glob
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
YOGI = os.environ.get("TUNE_YOGI") == "1"  # time fa_reduce_yogi (FedYoGi fused) instead of fa_reduce


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
        allres = {}
        for spec in sys.argv[2].split(","):
            K, P = (int(v) for v in spec.split(":"))
            allres[spec] = run(K, P, rounds)
            torch.cuda.empty_cache()
        json.dump(allres, open(os.path.join(ROOT, "gpurun_out", "tune_sweep.json"), "w"), indent=1)
        return
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    run(K, P, rounds)


def run(K, P, rounds):
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "*.so"))) + [
            os.path.join(ROOT, "fedscale_amd", "libfedagg.so")]:
        lib = ctypes.CDLL(path)
        if YOGI:
            f = lib.fa_reduce_yogi
            vp, fl = ctypes.c_void_p, ctypes.c_float
            f.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, vp, vp, fl, vp, vp, vp, vp, vp,
                          fl, fl, fl, fl, fl, ctypes.c_int32, vp]
        else:
            f = lib.fa_reduce
            f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p]
        f.restype = ctypes.c_int32
        libs[os.path.basename(path)] = f
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=5)
    out = torch.empty(ld, device="cuda")
    ref = None
    st = torch.cuda.current_stream().cuda_stream
    if YOGI:  # fused FedYoGi epilogue (fa_reduce_yogi), m/v re-initialised by every call (FA_YOGI_INIT)
        last, m, v = (torch.zeros(ld, device="cuda") for _ in range(3))
        plain = {n: f for n, f in libs.items()}
        for n, f0 in plain.items():
            libs[n] = (lambda f0: lambda xp, ld_, K_, P_, a, acc, outp, den, fl, s_: f0(
                xp, ld_, K_, P_, None, None, den, last.data_ptr(), m.data_ptr(), v.data_ptr(), outp, None,
                3e-3, 1e-8, 0.9, 0.1, 0.01, fl | 4, s_))(f0)
    times = {n: [] for n in libs}
    for r in range(rounds):
        for n, f in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            f(x.data_ptr(), ld, K, P, None, None, out.data_ptr(), float(K), 2, st)  # warm
            e0.record()
            for _ in range(3):
                rc = f(x.data_ptr(), ld, K, P, None, None, out.data_ptr(), float(K), 2, st)
                assert rc == 0
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), f"{n} result differs"
    bytes_ = 4 * K * P + (24 * P if YOGI else 4 * P)
    res = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "GBps": bytes_ / (np.median(t) * 1e-3) / 1e9} for n, t in times.items()}
    print(f"--- K={K} P={P}", flush=True)
    for n, v in sorted(res.items(), key=lambda kv: kv[1]["median_ms"]):
        print(f"{n:40s} {v['median_ms']:8.3f} ms  {v['GBps']:8.1f} GB/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"K": K, "P": P, "results": res}, open(os.path.join(ROOT, "gpurun_out", f"tune_k{K}_p{P}.json"), "w"),
              indent=1)
    del x
    return res


if __name__ == "__main__":
    main()
