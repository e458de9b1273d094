"""k_yogi_step alone (fa_yogi_step, 28 P bytes: cur, last, m, v read; m, v, new written) at config 4's sizes, back to
back on rotating buffer sets (> the 256 MiB Infinity Cache), HIP events on the launch stream.  Loads the library of
FEDAGG_LIB (tools/build_ab.sh variants).  usage: python tools/yogi_step_probe.py [P ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedscale_amd import _native, kernels as kx  # noqa: E402


def main():
    Ps = [int(a) for a in sys.argv[1:]] or [25_000_000, 6_250_048, 3_125_056]
    hp = dict(eta=float(np.float32(3e-3)), tau=float(np.float32(1e-8)), beta=float(np.float32(0.9)),
              omb=float(np.float32(0.1)), omb2=float(np.float32(0.01)))
    out = {"lib": os.path.basename(_native.build_info()["path"]), "defs": _native.build_info()["defs"]}
    for P in Ps:
        sets = [[torch.rand(P, device="cuda") for _ in range(5)] for _ in range(3)]
        for s in sets:
            kx.yogi_step(s[0], s[1], s[2], s[3], s[4], P, init=True, **hp)
        torch.cuda.synchronize()
        n = 60
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            s = sets[i % 3]
            kx.yogi_step(s[0], s[1], s[2], s[3], s[4], P, init=False, **hp)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        out[str(P)] = {"ms": ms, "GBps": 28 * P / (ms * 1e-3) / 1e9}
        del sets
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
