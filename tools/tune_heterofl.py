"""Interleaved A/B timing of fa_prefix_box_combine variants (fedscale_amd/variants/*.so + libfedagg.so) in ONE
process on the heterofl_bench workload (ResNet-18 layout, K clients at rates 1 / 0.5), FLAT plan.
usage: python tools/tune_heterofl.py [K] [rounds]"""
import ctypes
import glob
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.heterofl import PrefixBoxPlan

    names, shapes, dtypes = synth.resnet18_layout()
    gshapes = [s for s, d in zip(shapes, dtypes) if d == torch.float32]
    rates = [1.0 if m % 5 else 0.5 for m in range(K)]

    def box(s, r, first):
        if len(s) >= 2:
            o = s[0] if s[0] == 10 else math.ceil(r * s[0])
            i = s[1] if first else math.ceil(r * s[1])
            return (o, i) + tuple(s[2:])
        return (s[0],) if s[0] == 10 else (math.ceil(r * s[0]),)

    from fedscale_amd.cloud.aggregation import heterofl

    lshapes = [[box(s, r, k == 0) for k, s in enumerate(gshapes)] for r in rates]
    plans = {}
    default_elems = heterofl.FLAT_ELEMS

    def plan_for(name):  # variants built with -DHB_FLAT_J=J (file name "_j<J>_") need J*1024-element chunks
        j = int(name.split("_j")[1].split("_")[0]) if "_j" in name else default_elems // 1024
        if j not in plans:
            heterofl.FLAT_ELEMS = j * 1024
            plans[j] = PrefixBoxPlan(gshapes, lshapes, "cuda:0")
            heterofl.FLAT_ELEMS = default_elems
        return plans[j]

    plan = plan_for("default")
    xs = torch.empty(1, plan.upload_elems, device="cuda:0")
    synth.fill(xs, 1, plan.upload_elems, seed=9)
    xs = xs[0]
    glob_ = torch.empty(1, plan.P + 64, device="cuda:0")
    synth.fill(glob_, 1, plan.P, seed=10)
    glob_ = glob_[0]
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "*.so"))) + [
            os.path.join(ROOT, "fedscale_amd", "libfedagg.so")]:
        f = ctypes.CDLL(path).fa_prefix_box_combine
        f.restype = ctypes.c_int32
        V = ctypes.c_void_p
        f.argtypes = [V, V, ctypes.c_int32, V, ctypes.c_int32, V, V, ctypes.c_int32, V, V]
        libs[os.path.basename(path)] = f
    st = torch.cuda.current_stream().cuda_stream

    def args_for(n):
        p = plan_for(n)
        return (xs.data_ptr(), p.d_desc.data_ptr(), p.K, p.d_tens.data_ptr(), p.T, p.d_ct.data_ptr(),
                p.d_cf.data_ptr(), p.nchunks, glob_.data_ptr(), st)

    times = {n: [] for n in libs}
    for _ in range(rounds):
        for n, f in libs.items():
            args = args_for(n)
            assert f(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f(*args)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 10)
    alg = 4 * plan.upload_data_elems + 8 * plan.P
    print(f"--- HeteroFL K={K} ResNet-18, {plan.nchunks} chunks")
    for n in sorted(times, key=lambda n: np.median(times[n])):
        ms = float(np.median(times[n]))
        print(f"{n:40s} {ms:8.4f} ms {alg / (ms * 1e-3) / 1e9:9.1f} GB/s")


if __name__ == "__main__":
    main()
