"""Config 1's host round (FEMNIST CNN, K = 10, the drop-in from host dicts to get_weights) broken down call by call,
plus the floors of its parts measured in isolation (round 6, VERDICT r5 #4: get the device round below the CPU loop).

Prints JSON lines: ``breakdown`` (median µs per round of each wrapped call, nested timers include their children) and
``floors`` (the same work without the drop-in's Python: the bare ctypes launch + event wait, the staging copies, the
clones), and ``round`` (the unwrapped round, median of 300)."""
import argparse
import collections
import ctypes
import functools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import _native  # noqa: E402
from fedscale_amd import kernels as kx  # noqa: E402
from fedscale_amd import round as rd  # noqa: E402
from fedscale_amd import bucket, state, synth  # noqa: E402
from fedscale_amd.cloud.aggregation import aggregator as agm  # noqa: E402
from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer  # noqa: E402
from fedscale_amd.cloud.internal import torch_model_adapter as tma  # noqa: E402

ACC = collections.defaultdict(float)


def timed(owner, name):
    fn = getattr(owner, name)
    label = f"{getattr(owner, '__name__', owner)}.{name}"

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t0

    setattr(owner, name, w)
    return fn


def make(dev):
    job = bench.c1_job_conf()
    args = argparse.Namespace(**job["args"])
    K = args.num_participants
    names, shapes, base, ups = bench._c1_updates(1, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    ad = tma.TorchModelAdapter(model, optimizer=TorchServerOptimizer(args.gradient_policy, args, dev), device=dev)
    return agm.DeviceAggregator(ad, args), K, ups


def run_rounds(agg, K, ups, n=300, warm=20):
    out = []
    for r in range(n + warm):
        ACC.clear()
        t0 = time.perf_counter()
        agg.start_round(K)
        for k in range(K):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        agg.model_wrapper.get_weights()
        ACC["round"] = time.perf_counter() - t0
        if r >= warm:
            out.append(dict(ACC))
    return out


def med(rows, key):
    return round(float(np.median([r.get(key, 0.0) for r in rows])) * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    agg, K, ups = make(dev)
    rows = run_rounds(agg, K, ups)
    print(json.dumps({"round_unwrapped_us": med(rows, "round")}), flush=True)
    # the drop-in's round with each knob off in turn (A/B of this round's changes), interleaved
    knobs = {"all_on": {}, "head_launch_off": {"SPLIT": False}, "split_0.7": {"FRAC": 0.7}, "split_0.8": {"FRAC": 0.8},
             "split_0.9": {"FRAC": 0.9}}
    res = {k: [] for k in knobs}
    frac0 = rd.DeviceRound.SPLIT_FRACTION  # "all_on": the product default
    aggs = {k: make(dev) for k in knobs}
    for rep in range(6):
        for k, kv in knobs.items():
            a, KK, u = aggs[k]
            for attr, v in kv.items():
                if attr not in ("SPLIT", "FRAC"):
                    setattr(a.model_wrapper, attr, v)
            rd.DeviceRound.SPLIT_SMALL_ROUNDS = kv.get("SPLIT", True)
            rd.DeviceRound.SPLIT_FRACTION = kv.get("FRAC", frac0)
            rows = run_rounds(a, KK, u, n=100, warm=10)
            rd.DeviceRound.SPLIT_SMALL_ROUNDS = True
            rd.DeviceRound.SPLIT_FRACTION = frac0
            res[k].append(med(rows, "round"))
    print(json.dumps({"ab_round_us": {k: sorted(v) for k, v in res.items()}}), flush=True)
    # as bench.py runs it: the main thread bound to the GPU's NUMA node (hostnuma.bind_to_gpu), and bench's own round
    from fedscale_amd.hostnuma import bind_to_gpu

    node = bind_to_gpu(dev)
    a, KK, u = make(dev)
    rows = run_rounds(a, KK, u)
    c1 = bench.c1_host_round(dev, 1)
    print(json.dumps({"numa_bound": {"node": node, "round_us": med(rows, "round"),
                                     "bench_c1_host_round_us": c1["round_ms_incl_h2d_d2h"] * 1e3}}), flush=True)
    wraps = [(bucket.ClientStaging, "put"), (bucket.ClientStaging, "_put_bulk_views"),
             (bucket.ClientStaging, "_claim_bulk"), (bucket.ClientStaging, "host_rows"),
             (bucket.ClientStaging, "release_host_rows"), (rd.DeviceRound, "add"), (rd.DeviceRound, "finalize_mean"),
             (tma.TorchModelAdapter, "begin_round"), (tma.TorchModelAdapter, "apply_round"),
             (tma.TorchModelAdapter, "_apply_round"), (tma.TorchModelAdapter, "_mirror_target"),
             (tma.TorchModelAdapter, "_commit_scratch"), (tma.TorchModelAdapter, "_acquire_host"),
             (tma.TorchModelAdapter, "_release_host"), (tma.TorchModelAdapter, "_clone_weights"),
             (tma.TorchModelAdapter, "round_mean_weights"), (tma.TorchModelAdapter, "get_weights"),
             (kx, "reduce_mirror"), (kx, "side_accumulate"), (kx, "side_close"), (_native, "call"),
             (agm.DeviceAggregator, "on_result"), (agm.DeviceAggregatorMixin, "update_weight_aggregation"),
             (state.DeviceStream, "__enter__"), (state.DeviceStream, "__exit__"), (state.DeviceStream, "joined"),
             (torch.cuda.Event, "synchronize"), (torch.cuda.Event, "record")]
    for owner, name in wraps:
        if hasattr(owner, name):
            timed(owner, name)
    agg2, K, ups = make(dev)
    rows = run_rounds(agg2, K, ups)
    keys = sorted({k for r in rows for k in r})
    print(json.dumps({"breakdown_us": dict(sorted(((k, med(rows, k)) for k in keys), key=lambda kv: -kv[1]))}),
          flush=True)
    # floors: the same work with no drop-in Python around it
    lib = _native.load()
    L = agg2.model_wrapper.layout
    hx = torch.zeros(K, L.ld, dtype=torch.float32).pin_memory()
    hxn = hx.numpy()
    outd = torch.zeros(L.ld, dtype=torch.float32, device=dev)
    mir = torch.zeros((L.P_full + 3) // 4 * 4, dtype=torch.float32).pin_memory()
    st = torch.cuda.current_stream(dev).cuda_stream
    ev = torch.cuda.Event()
    views = [[hxn[k, e.offset:e.offset + e.numel].reshape(e.shape) for e in L.entries] for k in range(K)]
    fl = {"launch_and_wait": [], "launch_call": [], "stage_copies": [], "clones": [], "event_record": []}
    mviews = [mir.numpy()[e.offset:e.offset + e.numel].reshape(e.shape) for e in L.entries]
    denom = float(np.float32(K))
    for r in range(320):
        t0 = time.perf_counter()
        for k in range(K):
            for dst, a in zip(views[k], ups[k].values()):
                dst[...] = a
        t1 = time.perf_counter()
        lib.fa_reduce_mirror(hx.data_ptr(), L.ld, K, L.P, None, None, outd.data_ptr(), mir.data_ptr(), ctypes.c_float(denom),
                             _native.FA_FINALIZE, st)
        t2 = time.perf_counter()
        ev.record()
        t3 = time.perf_counter()
        ev.synchronize()
        t4 = time.perf_counter()
        cl = [torch.from_numpy(a.copy()) for a in mviews]
        t5 = time.perf_counter()
        if r >= 20:
            fl["stage_copies"].append(t1 - t0)
            fl["launch_call"].append(t2 - t1)
            fl["event_record"].append(t3 - t2)
            fl["launch_and_wait"].append(t4 - t1)
            fl["clones"].append(t5 - t4)
        del cl
    print(json.dumps({"floors_us": {k: round(float(np.median(v)) * 1e6, 2) for k, v in fl.items()}}), flush=True)
    # how the host waits: event synchronize against spinning on event.query(), and the kernel's own time by events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w = {"record_sync": [], "record_spin_query": [], "stream_sync": [], "kernel_by_events_us": []}
    for r in range(320):
        for mode in ("record_sync", "record_spin_query", "stream_sync"):
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            if mode == "record_sync":
                e0.record()
            lib.fa_reduce_mirror(hx.data_ptr(), L.ld, K, L.P, None, None, outd.data_ptr(), mir.data_ptr(), denom,
                                 _native.FA_FINALIZE, st)
            if mode == "stream_sync":
                torch.cuda.current_stream(dev).synchronize()
            else:
                (e1 if mode == "record_sync" else ev).record()
                if mode == "record_sync":
                    e1.synchronize()
                else:
                    while not ev.query():
                        pass
            t2 = time.perf_counter()
            if r >= 20:
                w[mode].append(t2 - t1)
                if mode == "record_sync":
                    w["kernel_by_events_us"].append(e0.elapsed_time(e1) * 1e-3)
    print(json.dumps({"wait_us": {k: round(float(np.median(v)) * 1e6, 2) for k, v in w.items()}}), flush=True)


if __name__ == "__main__":
    main()
