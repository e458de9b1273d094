"""Host cost of the one-process multi-GPU adapter (ShardedModelAdapter) per upload, against the number of
parts.  On the one-GPU box every part lives on cuda:0 (copy transport), so the device work is that of one
GPU whatever N is; what grows with N is the host side: one gather into the pinned full-model row per
upload, then one slice copy + staging bookkeeping per part.

usage: python tools/sharded_ingress_bench.py [K] [rounds] [layout=femnist|resnet18|p25m] [parts=1,2,4,8] [payload]
Prints one JSON line per (layout, parts): ms per upload through update_weight_aggregation (host dicts in)
and ms per round for the finish + get_weights().  ``payload``: the uploads arrive as the executor's pickled
payloads, decoded zero-copy as the mixin's deserialize_response does (aggregator.py:704), and each line is run
twice — registered in place (round 4, RegisteredUpload) and through the pinned-row gather (REGISTER_MIN_ENTRY_BYTES
= -1) — interleaved in one process.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _layout(which):
    from fedscale_amd import synth

    if which == "resnet18":
        return synth.resnet18_layout()
    if which == "p25m":
        return [f"l{i}.weight" for i in range(10)], [(2500, 1000)] * 10, [torch.float32] * 10
    return synth.femnist_cnn_layout()


def run(K, rounds, which, n_parts, payload=False, register=True):
    import pickle

    from fedscale_amd import ingress, synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    names, shapes, dtypes = _layout(which)
    model = synth.LayoutModule(names, shapes, dtypes)
    if n_parts == 0:
        adapter = TorchModelAdapter(model, device="cuda:0")
    else:
        adapter = ShardedModelAdapter(model, devices=[0] * n_parts, transport="copy")
        if not register:
            adapter.REGISTER_MIN_ENTRY_BYTES = -1
    agg = DeviceAggregator(adapter)
    rng = np.random.default_rng(0)
    pool = []
    for _ in range(4):
        up = {}
        for n, s, d in zip(names, shapes, dtypes):
            if d == torch.float32:
                up[n] = rng.standard_normal(s, dtype=np.float32) * np.float32(0.05)
            else:
                up[n] = np.array(rng.integers(0, 100), dtype=np.int64).reshape(s)
        pool.append(pickle.dumps({"update_weight": up}) if payload else up)
    t_add, t_fin = [], []
    for r in range(rounds + 2):
        torch.cuda.synchronize()
        agg.start_round(K)
        t0 = time.perf_counter()
        def upd(k):
            return ingress.loads(pool[k % 4])["update_weight"] if payload else pool[k % 4]

        for k in range(K - 1):
            agg.on_result({"client_id": k, "update_weight": upd(k), "moving_loss": 1.0})
        t1 = time.perf_counter()
        agg.on_result({"client_id": K - 1, "update_weight": upd(K - 1), "moving_loss": 1.0})
        adapter.get_weights()
        t2 = time.perf_counter()
        if r > 1:  # two warm-up rounds: staging, pinned rows and both egress snapshots allocated
            t_add.append((t1 - t0) / (K - 1))
            t_fin.append(t2 - t1)
    P = sum(int(np.prod(s)) for s, d in zip(shapes, dtypes) if d == torch.float32)
    out_extra = {}
    if n_parts:
        out_extra = {"registered_uploads": adapter.registered_uploads, "ingress": "payload" if payload else "dicts"}
        adapter.close()
    return {**out_extra, "layout": which, "parts": n_parts or "single adapter", "clients": K, "params": P,
            "ms_per_upload": float(np.median(t_add)) * 1e3, "finish_and_get_weights_ms": float(np.median(t_fin)) * 1e3,
            "upload_gbps": 4 * P / float(np.median(t_add)) / 1e9}


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    which = sys.argv[3] if len(sys.argv) > 3 else "femnist"
    parts = [int(p) for p in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1, 2, 4, 8]
    payload = len(sys.argv) > 5 and sys.argv[5] == "payload"
    import gc

    for n in parts:
        for reg in ((True, False, True) if payload and n else (True,)):
            print(json.dumps(dict(run(K, rounds, which, n, payload, reg), register=reg)), flush=True)
            gc.collect()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
