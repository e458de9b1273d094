"""Device-resident HeteroFL combination rate (examples/heterofl/customized_aggregator.py:78-119) on a
ResNet-18 layout: K clients at model rates drawn like the example's config (80 % rate 1, 20 % rate 0.5).
usage: python tools/heterofl_bench.py [K] [reps]"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.heterofl import PrefixBoxPlan

    names, shapes, dtypes = synth.resnet18_layout()
    gshapes = [s for s, d in zip(shapes, dtypes) if d == torch.float32]
    rates = [1.0 if m % 5 else 0.5 for m in range(K)]

    def box(s, r, first):
        if len(s) >= 2:  # conv / linear weight: output and input prefixes (first conv keeps its 3 inputs)
            o = s[0] if s[0] == 10 else math.ceil(r * s[0])
            i = s[1] if first else math.ceil(r * s[1])
            return (o, i) + tuple(s[2:])
        if len(s) == 1:
            return (s[0],) if s[0] == 10 else (math.ceil(r * s[0]),)
        return s

    from fedscale_amd.cloud.aggregation import heterofl

    if os.environ.get("HB_FLAT_ELEMS"):  # tuning builds with -DHB_FLAT_J=J need J*1024 here
        heterofl.FLAT_ELEMS = int(os.environ["HB_FLAT_ELEMS"])
    lshapes = [[box(s, r, k == 0) for k, s in enumerate(gshapes)] for r in rates]
    plans = {}
    for flat in (False, True):  # A/B in one process: the ROW/ELEMENT plan, then FLAT (production)
        heterofl.USE_FLAT = flat
        plans[flat] = PrefixBoxPlan(gshapes, lshapes, "cuda:0")
    plan = plans[True]
    xs = torch.empty(1, plan.upload_elems, device="cuda:0")
    synth.fill(xs, 1, plan.upload_elems, seed=9)
    xs = xs[0]
    glob = torch.empty(1, plan.P + 64, device="cuda:0")
    synth.fill(glob, 1, plan.P, seed=10)
    glob = glob[0]
    ms = {False: [], True: []}
    for rnd in range(3):
        for flat, pl in plans.items():
            pl.run(xs, glob)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                pl.run(xs, glob)
            e1.record()
            torch.cuda.synchronize()
            ms[flat].append(e0.elapsed_time(e1) / reps)
    alg = 4 * plan.upload_data_elems + 8 * plan.P  # every uploaded parameter read once; global read + written
    m = float(np.median(ms[True]))
    m_row = float(np.median(ms[False]))
    out = {"K": K, "P": plan.P, "upload_elems": plan.upload_data_elems, "padded_elems": plan.upload_elems,
           "kernel_ms": m, "GBps": alg / (m * 1e-3) / 1e9, "client_updates_per_s": K / (m * 1e-3),
           "chunks": plan.nchunks, "row_plan_kernel_ms": m_row, "row_plan_GBps": alg / (m_row * 1e-3) / 1e9,
           "row_plan_chunks": plans[False].nchunks}
    print(json.dumps(out))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "heterofl_bench.json"), "w"), indent=1)


if __name__ == "__main__" and not (len(sys.argv) > 3 and sys.argv[3] == "ingress"):
    main()


def ingress(K=100):
    """PCIe-inclusive HeteroFL round: K uploads (dicts of numpy prefix boxes in host memory) staged on
    arrival (PrefixBoxStaging: pinned pack + async H2D per client), then the combination; against the
    pack-everything-at-combine path (combine_prefix_boxes)."""
    import time
    from collections import OrderedDict

    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.heterofl import PrefixBoxStaging, combine_prefix_boxes

    names, shapes, dtypes = synth.resnet18_layout()
    gnames = [n for n, d in zip(names, dtypes) if d == torch.float32]
    gshapes = [s for s, d in zip(shapes, dtypes) if d == torch.float32]
    rng = np.random.default_rng(0)

    def box(s, r, first):
        if len(s) >= 2:
            o = s[0] if s[0] == 10 else math.ceil(r * s[0])
            i = s[1] if first else math.ceil(r * s[1])
            return (o, i) + tuple(s[2:])
        return (s[0],) if s[0] == 10 else (math.ceil(r * s[0]),)

    pool = []
    for r in (1.0, 1.0, 1.0, 1.0, 0.5):
        pool.append({n: rng.standard_normal(box(s, r, k == 0), dtype=np.float32)
                     for k, (n, s) in enumerate(zip(gnames, gshapes))})
    glob = OrderedDict((n, torch.zeros(s)) for n, s in zip(gnames, gshapes))
    out = {}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = PrefixBoxStaging(gshapes, K, "cuda:0")
        for m in range(K):
            st.add(gnames, pool[m % 5])
        st.combine(glob)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        combine_prefix_boxes(glob, [pool[m % 5] for m in range(K)], device="cuda:0")
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        nbytes = 4 * sum(sum(a.size for a in pool[m % 5].values()) for m in range(K))
        out = {"K": K, "upload_bytes": nbytes, "staged_on_arrival_s": t1 - t0,
               "staged_GBps": nbytes / (t1 - t0) / 1e9, "pack_at_combine_s": t2 - t1,
               "pack_at_combine_GBps": nbytes / (t2 - t1) / 1e9}
    print(json.dumps(out))
    return out


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "ingress":
    ingress(int(sys.argv[1]))
