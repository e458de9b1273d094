"""Host cost of the one-process multi-GPU adapter (ShardedModelAdapter) per upload, against the number of
parts.  On the one-GPU box every part lives on cuda:0 (copy transport), so the device work is that of one
GPU whatever N is; what grows with N is the host side: one gather into the pinned full-model row per
upload, then one slice copy + staging bookkeeping per part.

usage: python tools/sharded_ingress_bench.py [K] [rounds] [layout=femnist|resnet18] [parts=1,2,4,8]
Prints one JSON line per (layout, parts): ms per upload through update_weight_aggregation (host dicts in)
and ms per round for the finish + get_weights().
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(K, rounds, which, n_parts):
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    names, shapes, dtypes = synth.resnet18_layout() if which == "resnet18" else synth.femnist_cnn_layout()
    model = synth.LayoutModule(names, shapes, dtypes)
    if n_parts == 0:
        adapter = TorchModelAdapter(model, device="cuda:0")
    else:
        adapter = ShardedModelAdapter(model, devices=[0] * n_parts, transport="copy")
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
        pool.append(up)
    t_add, t_fin = [], []
    for r in range(rounds + 2):
        torch.cuda.synchronize()
        agg.start_round(K)
        t0 = time.perf_counter()
        for k in range(K - 1):
            agg.on_result({"client_id": k, "update_weight": pool[k % 4], "moving_loss": 1.0})
        t1 = time.perf_counter()
        agg.on_result({"client_id": K - 1, "update_weight": pool[(K - 1) % 4], "moving_loss": 1.0})
        adapter.get_weights()
        t2 = time.perf_counter()
        if r > 1:  # two warm-up rounds: staging, pinned rows and both egress snapshots allocated
            t_add.append((t1 - t0) / (K - 1))
            t_fin.append(t2 - t1)
    P = sum(int(np.prod(s)) for s, d in zip(shapes, dtypes) if d == torch.float32)
    return {"layout": which, "parts": n_parts or "single adapter", "clients": K, "params": P,
            "ms_per_upload": float(np.median(t_add)) * 1e3, "finish_and_get_weights_ms": float(np.median(t_fin)) * 1e3,
            "upload_gbps": 4 * P / float(np.median(t_add)) / 1e9}


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    which = sys.argv[3] if len(sys.argv) > 3 else "femnist"
    parts = [int(p) for p in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1, 2, 4, 8]
    import gc

    for n in parts:
        print(json.dumps(run(K, rounds, which, n)), flush=True)
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
