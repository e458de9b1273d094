"""N-GPU ingress: host-DRAM passes per upload.  Two ways to get one upload's parameter slices
onto N parts (ShardedModelAdapter), per upload, from the executor's pickled payload decoded zero-copy
(fedscale_amd/ingress.py: the arrays are views of the payload bytes, aggregator.py:704):

  gather   (round-3 path) fa_host_gather of every array into a pinned full-model row (payload read + pinned
           write, streaming stores), then one H2D per part out of the row (DMA read): 3 host-DRAM passes;
  register hipHostRegister of the payload's pages in place, one H2D per (part, tensor piece) straight out of the
           payload (DMA read only: 1 pass), then hipHostUnregister — the registration's page pinning and IOMMU
           mapping are paid per upload, since every upload is a fresh bytes object;
  reuse    the same copies out of an already registered payload (registration amortised: an upper bound, as if
           the gRPC layer received into a registered buffer pool).

All parts live on cuda:0 here (one-GPU box), each with its own stream and destination row; on a node each part's
copy has its own PCIe link, so the host side (what this measures beside the link) is the question.
usage: python tools/register_probe.py [layout=p25m|resnet18] [parts=1,2,4] [uploads=16]
Prints one JSON line per (layout, parts, path).
"""
import ctypes
import json
import os
import pickle
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
H2D = 1
PAGE = 4096


def _layout(which):
    from fedscale_amd import synth

    if which == "resnet18":
        names, shapes, dtypes = synth.resnet18_layout()
        keep = [(n, s) for n, s, d in zip(names, shapes, dtypes) if d == torch.float32]
        return [k[0] for k in keep], [k[1] for k in keep]
    return [f"l{i}.weight" for i in range(10)], [(2500, 1000)] * 10


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "p25m"
    parts_list = [int(p) for p in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4").split(",")]
    n_up = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    from fedscale_amd import ingress
    from fedscale_amd.bucket import BucketLayout, HostRow, round_up
    from fedscale_amd.synth import LayoutModule

    names, shapes = _layout(which)
    model = LayoutModule(names, shapes, [torch.float32] * len(names))
    L = BucketLayout.from_state_dict(model.state_dict())
    rng = np.random.default_rng(0)
    payloads = []
    for i in range(4):
        up = {n: rng.standard_normal(s, dtype=np.float32) for n, s in zip(names, shapes)}
        payloads.append(pickle.dumps({"client_id": i, "moving_loss": 1.0, "update_weight": up}))
        del up
    P = L.P_full
    nbytes = 4 * P
    for N in parts_list:
        S = round_up(-(-P // N), 64)
        dst = [torch.empty(S, device="cuda") for _ in range(N)]
        streams = [torch.cuda.Stream() for _ in range(N)]
        bounds = [(min(P, r * S), min(P, (r + 1) * S)) for r in range(N)]

        def pieces(arrays):
            """(part, dst byte offset, src address, bytes) of every tensor piece of every part's slice."""
            out, p0 = [], 0
            for a in arrays:
                n = a.size
                for r, (b0, b1) in enumerate(bounds):
                    lo, hi = max(p0, b0), min(p0 + n, b1)
                    if lo < hi:
                        out.append((r, (lo - b0) * 4, a.ctypes.data + (lo - p0) * 4, (hi - lo) * 4))
                p0 += n
            return out

        rows = [HostRow(L.ld, L.ldq) for _ in range(2)]
        res = {}
        for path in ("gather", "register", "reuse", "gather"):
            torch.cuda.synchronize()
            regs = []
            if path == "reuse":  # register every payload once, outside the timing
                for pb in payloads:
                    base = np.frombuffer(pb, np.uint8).ctypes.data
                    a0, a1 = base // PAGE * PAGE, -(-(base + len(pb)) // PAGE) * PAGE
                    assert hip.hipHostRegister(a0, a1 - a0, 0) == 0
                    regs.append(a0)
            reg_ms = []
            t0 = time.perf_counter()
            for k in range(n_up):
                pb = payloads[k % 4]
                res_k = ingress.loads(pb)
                arrays = [res_k["update_weight"][n] for n in names]
                if path == "gather":
                    row = rows[k % 2]
                    row.wait()
                    L.run_host_gather(L.host_gather_plan(arrays), row.f_np, row.i_np, workers=8)
                    for r, (b0, b1) in enumerate(bounds):
                        with torch.cuda.stream(streams[r]):
                            dst[r][:b1 - b0].copy_(row.f[b0:b1], non_blocking=True)
                            ev = torch.cuda.Event()
                            ev.record(streams[r])
                            row.pending.append(ev)
                else:
                    if path == "register":
                        base = np.frombuffer(pb, np.uint8).ctypes.data
                        a0, a1 = base // PAGE * PAGE, -(-(base + len(pb)) // PAGE) * PAGE
                        tr = time.perf_counter()
                        assert hip.hipHostRegister(a0, a1 - a0, 0) == 0
                        reg_ms.append((time.perf_counter() - tr) * 1e3)
                    for r, off, src, nb in pieces(arrays):
                        assert hip.hipMemcpyAsync(dst[r].data_ptr() + off, src, nb, H2D,
                                                  streams[r].cuda_stream) == 0
                    if path == "register":  # the pages stay pinned until every copy out of them is done
                        for s in streams:
                            s.synchronize()
                        tu = time.perf_counter()
                        assert hip.hipHostUnregister(a0) == 0
                        reg_ms[-1] += (time.perf_counter() - tu) * 1e3
                    else:
                        for s in streams:  # the next upload may reuse this payload's buffer
                            s.synchronize()
            for s in streams:
                s.synchronize()
            dt = (time.perf_counter() - t0) / n_up
            for a0 in regs:
                hip.hipHostUnregister(a0)
            key = path if path not in res else path + "_again"
            res[key] = {"ms_per_upload": dt * 1e3, "GBps": nbytes / dt / 1e9,
                        "host_dram_passes": {"gather": 3, "register": 1, "reuse": 1}[path]}
            if reg_ms:
                res[key]["register_unregister_ms"] = float(np.median(reg_ms))
        print(json.dumps({"layout": which, "params": P, "MB_per_upload": nbytes / 1e6, "parts": N,
                          "pieces_per_upload": len(pieces([np.empty(int(np.prod(s)), np.float32) for s in shapes])),
                          "paths": res}), flush=True)


if __name__ == "__main__":
    main()
