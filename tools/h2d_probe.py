"""Measure H2D options: torch copy_ from pinned (copy engine) vs a kernel pulling pinned host memory."""
import ctypes
import json
import os
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bw(nbytes, fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libh2d_probe.so"))
    lib.h2d_pull.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    res = {}
    st = torch.cuda.current_stream().cuda_stream
    for mb in (45, 400):
        n = mb * (1 << 20) // 4
        h = torch.ones(n).pin_memory()
        d = torch.empty(n, device="cuda")
        res[f"copy_engine_{mb}MB"] = bw(n * 4, lambda: d.copy_(h, non_blocking=True))
        for grid in (256, 1024, 4096):
            res[f"kernel_pull_{mb}MB_grid{grid}"] = bw(n * 4, lambda: lib.h2d_pull(h.data_ptr(), d.data_ptr(), n, grid, st))
        assert torch.equal(d.cpu(), h)
        pageable = torch.ones(n)
        res[f"copy_pageable_{mb}MB"] = bw(n * 4, lambda: d.copy_(pageable), reps=3)
    print(json.dumps(res, indent=1))
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "h2d_probe.json"), "w"), indent=1)


if __name__ == "__main__" and not os.environ.get("PACK_PROBE"):
    main()


def pack_probe():
    """Host pack of one ResNet-18 client update into pinned memory, by worker count (no GPU work)."""
    import sys
    sys.path.insert(0, ROOT)
    from fedscale_amd import synth
    from fedscale_amd.bucket import BucketLayout

    names, shapes, dtypes = synth.resnet18_layout()
    lay = BucketLayout(names, shapes, dtypes)
    rng = np.random.default_rng(0)
    pool = []
    for i in range(8):
        pool.append({n: (rng.standard_normal(s, dtype=np.float32) if t == torch.float32 else
                         np.array(3, dtype=np.int64).reshape(s)) for n, s, t in zip(names, shapes, dtypes)})
    hf = torch.zeros(lay.ld).pin_memory()
    hi = np.zeros(lay.ldq, np.int64)
    out = {}
    for w in (1, 2, 4, 8, 16):
        for rep in range(2):
            t0 = time.perf_counter()
            for r in range(24):
                lay.pack_host(pool[r % 8], hf.numpy(), hi, workers=w)
            dt = (time.perf_counter() - t0) / 24
        out[f"pack_workers{w}_GBps"] = lay.P * 4 / dt / 1e9
    big = [np.random.rand(lay.P).astype(np.float32) for _ in range(8)]
    t0 = time.perf_counter()
    for r in range(24):
        np.copyto(hf.numpy()[:lay.P], big[r % 8])
    out["single_memcpy_GBps"] = lay.P * 4 / ((time.perf_counter() - t0) / 24) / 1e9
    hft = hf[:lay.P]
    bigt = [torch.from_numpy(b) for b in big]
    for nt in (1, 4, 8, 16):
        torch.set_num_threads(nt)
        t0 = time.perf_counter()
        for r in range(24):
            hft.copy_(bigt[r % 8])
        out[f"torch_copy_threads{nt}_GBps"] = lay.P * 4 / ((time.perf_counter() - t0) / 24) / 1e9
    from concurrent.futures import ThreadPoolExecutor
    for nt in (4, 8):
        ex = ThreadPoolExecutor(nt)
        step = lay.P // nt
        def part(i, r):
            np.copyto(hf.numpy()[i * step:(i + 1) * step], big[r % 8][i * step:(i + 1) * step])
        t0 = time.perf_counter()
        for r in range(24):
            list(ex.map(lambda i: part(i, r), range(nt)))
        out[f"np_threads{nt}_GBps"] = step * nt * 4 / ((time.perf_counter() - t0) / 24) / 1e9
    print(json.dumps(out, indent=1))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "pack_probe.json"), "w"), indent=1)


if __name__ == "__main__" and os.environ.get("PACK_PROBE"):
    pack_probe()
