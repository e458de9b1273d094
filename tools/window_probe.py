"""fa_reduce (FedAvg mean) over K x P in ONE launch against n launches over equal column windows of the same
rows (same ld, same bits), interleaved in one process.  usage: python tools/window_probe.py [K] [P] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedscale_amd import synth
    from fedscale_amd._native import FA_FINALIZE, call
    from fedscale_amd.bucket import round_up

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=5)
    outs = {}
    st = torch.cuda.current_stream().cuda_stream
    denom = float(np.float32(K))

    def launcher(n):
        w = round_up(-(-P // n), 64)
        out = outs.setdefault(n, torch.empty(ld, device="cuda"))

        def f():
            for c0 in range(0, P, w):
                pw = min(w, P - c0)
                call("fa_reduce", x.data_ptr() + 4 * c0, ld, K, pw, None, None, out.data_ptr() + 4 * c0, denom,
                     FA_FINALIZE, st)
        return f

    ns = (1, 2, 3, 4)
    fs = {n: launcher(n) for n in ns}
    times = {n: [] for n in ns}
    for _ in range(rounds):
        for n in ns:
            fs[n]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fs[n]()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
    for n in ns[1:]:
        assert torch.equal(outs[n][:P], outs[1][:P]), f"{n} windows: result differs"
    b = 4 * K * P + 4 * P
    print(json.dumps({"K": K, "P": P, **{f"windows{n}": {"ms": round(float(np.median(t)), 3),
                                                         "GBps": round(b / (np.median(t) * 1e-3) / 1e9, 1)}
                                         for n, t in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
