"""Config 2 (100 clients x 1M fp32, 400 MB per round) probe: fa_reduce variants against a bare stream read of
the same bytes, every launch on a different one of NSETS rotating input sets (1.6 GB: the 256 MiB Infinity
Cache cannot serve a repeat), interleaved in one process.

usage: python tools/c2_probe.py [K] [P] [reps]
Each library in fedscale_amd/variants/*.so plus the production libfedagg.so; per variant:
  event_us   median of per-launch HIP-event times (what bench.py's config lines report)
  chain_us   mean per launch of 20 back-to-back launches between one event pair (launch gaps included)
and for tools/libhbm_ceiling.so (the read-only float4 nt kernel) the same per grid size.
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
NSETS = 4


def main():
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    ld = round_up(P, 64)
    xs = []
    for i in range(NSETS):
        x = torch.empty(K, ld, device="cuda")
        synth.fill(x, K, P, seed=11 + i)
        xs.append(x)
    out = torch.empty(ld, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    fns = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "libfedagg_v*.so"))) + [
            os.path.join(ROOT, "fedscale_amd", "libfedagg.so")]:
        lib = ctypes.CDLL(path)
        f = lib.fa_reduce
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p]
        f.restype = ctypes.c_int32
        fns[os.path.basename(path)] = (lambda f: lambda x: f(x.data_ptr(), ld, K, P, None, None, out.data_ptr(),
                                                             float(K), 2, st))(f)
    rd = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_ceiling.so")).hbm_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    sink = torch.empty(8192 * 256, device="cuda")
    n_read = K * ld  # the same bytes as one round (rows are contiguous)
    for grid in (256, 512, 1024, 2048):
        fns[f"bare_read_grid{grid}"] = (lambda g: lambda x: rd(x.data_ptr(), n_read, sink.data_ptr(), g, 8, st))(grid)

    ref = {}
    res = {n: {"event_us": [], "chain_us": []} for n in fns}
    it = 0
    for r in range(reps):
        for n, f in fns.items():
            for _ in range(2):  # warm
                f(xs[it % NSETS]); it += 1
            evs = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f(xs[it % NSETS]); it += 1
                e1.record()
                evs.append((e0, e1))
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record()
            for _ in range(20):
                f(xs[it % NSETS]); it += 1
            c1.record()
            torch.cuda.synchronize()
            res[n]["event_us"] += [a.elapsed_time(b) * 1e3 for a, b in evs]
            res[n]["chain_us"].append(c0.elapsed_time(c1) * 1e3 / 20)
            if not n.startswith("bare"):
                f(xs[0])
                torch.cuda.synchronize()
                if "out" not in ref:
                    ref["out"] = out.clone()
                else:
                    assert torch.equal(out, ref["out"]), f"{n}: result differs"
    nbytes = 4 * K * P + 4 * P
    summary = {}
    for n, v in res.items():
        ev, ch = float(np.median(v["event_us"])), float(np.median(v["chain_us"]))
        b = nbytes if not n.startswith("bare") else 4 * n_read
        summary[n] = {"event_us": ev, "chain_us": ch, "event_GBps": b / ev / 1e3, "chain_GBps": b / ch / 1e3}
    print(f"--- K={K} P={P} ({NSETS} rotating sets, reps={reps})")
    for n, v in sorted(summary.items(), key=lambda kv: kv[1]["event_us"]):
        print(f"{n:44s} event {v['event_us']:7.1f} us {v['event_GBps']:7.0f} GB/s | chained {v['chain_us']:7.1f} us "
              f"{v['chain_GBps']:7.0f} GB/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"K": K, "P": P, "summary": summary}, open(os.path.join(ROOT, "gpurun_out", f"c2_probe_k{K}_p{P}.json"),
                                                         "w"), indent=1)


if __name__ == "__main__":
    main()
