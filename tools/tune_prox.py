"""Kernel-level timing of fa_prox_update variants (fedscale_amd/variants/libfedagg_mt_*.so, built with
tools/build_mt_variants.sh) against libfedagg.so on the ResNet-18 layout (62 tensors, 11.18 M fp32): HIP events
around 20 back-to-back launches, interleaved, medians.  Every variant's result must equal the default's.
usage: python tools/tune_prox.py [rounds]"""
import ctypes
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedscale_amd import synth

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    names, shapes, dtypes = synth.resnet18_layout()
    # the model's parameters (what FedProx walks, optimizers.py:6-10): no BatchNorm running statistics
    shapes = [s for n, s, d in zip(names, shapes, dtypes) if d == torch.float32 and "running" not in n]
    g = torch.Generator(device="cuda").manual_seed(0)
    params = [torch.randn(s, device="cuda", generator=g) for s in shapes]
    glob_ = [torch.randn(s, device="cuda", generator=g) for s in shapes]
    T = len(params)
    pp = np.asarray([p.data_ptr() for p in params], dtype=np.uint64)
    gp = np.asarray([t.data_ptr() for t in glob_], dtype=np.uint64)
    nn = np.asarray([p.numel() for p in params], dtype=np.int64)
    n_total = int(nn.sum())
    libs = {}
    for path in [os.path.join(ROOT, "fedscale_amd", "libfedagg.so")] + sorted(
            glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "libfedagg_mt_*.so"))):
        f = ctypes.CDLL(path).fa_prox_update
        f.restype = ctypes.c_int32
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_float,
                      ctypes.c_void_p]
        libs[os.path.basename(path)[:-3]] = f
    st = torch.cuda.current_stream().cuda_stream
    start = [p.clone() for p in params]
    ref = None
    times = {n: [] for n in libs}
    for r in range(rounds):
        for n, f in libs.items():
            for p, s in zip(params, start):
                p.copy_(s)
            assert f(pp.ctypes.data, gp.ctypes.data, nn.ctypes.data, T, 0.01, st) == 0
            torch.cuda.synchronize()
            got = torch.cat([p.reshape(-1) for p in params])
            if ref is None:
                ref = got.clone()
            assert torch.equal(got, ref), f"{n}: result differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f(pp.ctypes.data, gp.ctypes.data, nn.ctypes.data, T, 0.0, st)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 20)
    b = 12 * n_total
    print(f"--- fa_prox_update, ResNet-18 layout: {T} tensors, {n_total} fp32, 12P = {b / 1e6:.1f} MB per launch")
    for n in sorted(times, key=lambda k: np.median(times[k])):
        ms = float(np.median(times[n]))
        print(f"{n:36s} {ms * 1e3:8.2f} us {b / (ms * 1e-3) / 1e9:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
