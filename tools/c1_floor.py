"""The device floor under BASELINE config 1's round (10 x 24,492 fp32): what one H2D of the ten
staged rows, the reduce and the D2H of the model cost with no Python in between, eager and replayed from a
HIP graph, beside the drop-in's whole round.  Median over rounds, milliseconds.
usage: python tools/c1_floor.py [rounds]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(ts):
    return round(float(np.median(ts)) * 1e3, 4)


def main():
    import torch

    from fedscale_amd import kernels as kx
    from fedscale_amd.bucket import round_up

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    K, P = 10, 24492
    ld = round_up(P, 64)
    hx = torch.randn(K, ld).pin_memory()
    x = torch.empty(K, ld, device=dev)
    out = torch.empty(ld, device=dev)
    hout = torch.empty(ld).pin_memory()
    denom = float(np.float32(K))
    st = torch.cuda.current_stream(dev)

    def seq(h2d=True, red=True, d2h=True):
        if h2d:
            x.copy_(hx, non_blocking=True)
        if red:
            kx.reduce(x, K, P, out, denom=denom, finalize=True)
        if d2h:
            hout.copy_(out, non_blocking=True)

    res = {}
    for name, kw in (("sync_only", dict(h2d=False, red=False, d2h=False)),
                     ("h2d_1MB", dict(red=False, d2h=False)),
                     ("reduce", dict(h2d=False, d2h=False)),
                     ("d2h_98KB", dict(h2d=False, red=False)),
                     ("h2d_reduce_d2h_eager", {})):
        ts = []
        for r in range(rounds + 20):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            seq(**kw)
            st.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = med(ts[20:])
    # the same three steps captured once and replayed (one graph launch + one sync per round)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    side.wait_stream(st)
    with torch.cuda.stream(side):
        seq()  # warm the kernel and the copy paths off the capture
        side.synchronize()
        with torch.cuda.graph(g, stream=side):
            seq()
    ts = []
    for r in range(rounds + 20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.current_stream(dev).synchronize()
        ts.append(time.perf_counter() - t0)
    res["h2d_reduce_d2h_graph"] = med(ts[20:])
    expect = (hx[:, :P].sum(0, dtype=torch.float32) / 1).numpy()  # not bit-exact order: a sanity check only
    g.replay()
    torch.cuda.synchronize(dev)
    res["graph_output_matches_eager_reduce"] = bool(np.allclose(hout[:P].numpy() * K, expect, rtol=1e-4, atol=1e-4))
    print(json.dumps(res | {"unit": "ms", "rounds": rounds}))


if __name__ == "__main__":
    main()
