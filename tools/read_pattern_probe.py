"""Round 6: sweep read shapes against the round-1 stream-read ceiling (tools/read_pattern_probe.hip).
usage: python tools/read_pattern_probe.py [GiB]   -> one JSON line per (variant, grid), then the best of each variant"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {0: "stride_nt_u8", 1: "stride_default_u8", 2: "contiguous_nt_u8", 3: "stride_nt_u8_512t", 4: "stride_nt_u4",
            5: "stride_nt_u12", 10: "buf_aux0", 11: "buf_sc0", 12: "buf_nt", 13: "buf_sc0_nt", 14: "buf_sc1",
            15: "buf_sc1_nt"}
GRIDS = (128, 160, 176, 192, 208, 224, 240, 256, 320, 384, 512)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 32
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libread_pattern_probe.so"))
    f = lib.probe_read
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n = int(gib * (1 << 30) / 4) // 4096 * 4096
    x = torch.ones(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    out = torch.empty(max(GRIDS) * 512, device="cuda")
    best = {}
    for v, name in VARIANTS.items():
        for grid in GRIDS:
            ts = []
            for _ in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if f(x.data_ptr(), n, out.data_ptr(), grid, v, st) != 0:
                    raise RuntimeError(f"launch failed: {name} grid {grid}")
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            gbps = n * 4 / (float(np.median(ts[1:])) * 1e-3) / 1e9
            print(json.dumps({"variant": name, "grid": grid, "GBps": round(gbps, 1)}), flush=True)
            if gbps > best.get(name, (0, 0))[0]:
                best[name] = (round(gbps, 1), grid)
    print(json.dumps({"bytes": n * 4, "best": best}), flush=True)


if __name__ == "__main__":
    main()
