"""Measure D2H options for egress: torch copy_ into pinned memory (copy engine) vs a kernel pushing into pinned
host memory, for the ResNet-18 (45 MB) and 25 M (100 MB) models.  usage: python tools/d2h_probe.py"""
import ctypes
import json
import os
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bw(nbytes, fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
        torch.cuda.synchronize()  # egress waits for each copy
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libd2h_probe.so"))
    lib.d2h_push.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    res = {}
    st = torch.cuda.current_stream().cuda_stream
    for mb in (45, 100):
        n = mb * (1 << 20) // 4
        d = torch.randn(n, device="cuda")
        h = torch.empty(n).pin_memory()
        res[f"copy_engine_{mb}MB"] = bw(n * 4, lambda: h.copy_(d, non_blocking=True))
        res[f"copy_engine_blocking_{mb}MB"] = bw(n * 4, lambda: h.copy_(d))
        for grid in (256, 1024, 4096):
            h.zero_()
            res[f"kernel_push_{mb}MB_grid{grid}"] = bw(n * 4, lambda: lib.d2h_push(d.data_ptr(), h.data_ptr(), n, grid, st))
            assert torch.equal(h, d.cpu()), "push kernel result differs"
    print(json.dumps(res, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "d2h_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
