"""Host gather rate (fa_host_gather: pageable numpy pieces -> one pinned row) against its worker count: the
host-memory side of multi-GPU ingress, where one gather feeds the N GPUs' slices.  A pool of 8
distinct 100 MB updates (10 pieces of 10 MB each) rotates so the host caches cannot serve repeats.
usage: python tools/gather_probe.py [workers,...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from fedscale_amd import _native

    workers = [int(w) for w in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 4, 8, 12, 16, 24, 32]
    piece, pieces, pool_n = 2_500_000, 10, 8
    rng = np.random.default_rng(0)
    pool = [[rng.standard_normal(piece, dtype=np.float32) for _ in range(pieces)] for _ in range(pool_n)]
    dst = torch.empty(piece * pieces, dtype=torch.float32)
    if torch.cuda.is_available():
        dst = dst.pin_memory()  # else (a host without a GPU) a pageable row
    dptr = dst.data_ptr()
    offs = np.arange(pieces, dtype=np.int64) * piece * 4
    sizes = np.full(pieces, piece * 4, dtype=np.int64)
    plans = [np.asarray([a.ctypes.data for a in upd], dtype=np.uint64) for upd in pool]
    nbytes = piece * pieces * 4
    out = {"streaming_stores": os.environ.get("FEDAGG_GATHER_NT", "1") != "0", "bytes_per_update": nbytes, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    for w in workers:
        for p in plans[:2]:  # warm the pool of this size
            _native.call("fa_host_gather", dptr, p.ctypes.data, offs.ctypes.data, sizes.ctypes.data, pieces, w)
        ts = []
        for r in range(24):
            p = plans[r % pool_n]
            t0 = time.perf_counter()
            _native.call("fa_host_gather", dptr, p.ctypes.data, offs.ctypes.data, sizes.ctypes.data, pieces, w)
            ts.append(time.perf_counter() - t0)
        out[f"workers{w}_GBps"] = round(nbytes / float(np.median(ts)) / 1e9, 2)
    ref = np.concatenate(pool[23 % pool_n])
    out["last_gather_exact"] = bool(np.array_equal(dst.numpy(), ref))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
