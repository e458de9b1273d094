"""Measure the HBM stream-read ceiling (GB/s) of this MI355X with tools/hbm_ceiling.hip.
usage: python tools/hbm_ceiling.py [GiB]   -> prints JSON, writes gpurun_out/hbm_ceiling.json"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 64
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_ceiling.so"))
    f = lib.hbm_read
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n = int(gib * (1 << 30) / 4) // 1024 * 1024
    x = torch.ones(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for grid in (192, 256, 384, 512, 768, 1024, 2048, 4096, 8192):
        out = torch.empty(grid * 256, device="cuda")
        for unroll in (8, 16):
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f(x.data_ptr(), n, out.data_ptr(), grid, unroll, st)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[f"grid{grid}_u{unroll}"] = n * 4 / (np.median(ts[1:]) * 1e-3) / 1e9
    best = max(res.values())
    out = {"bytes": n * 4, "GBps": res, "ceiling_GBps": best}
    print(json.dumps(out))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "hbm_ceiling.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
