"""Host-ingress-inclusive aggregation rate: client updates arrive as dicts of numpy
arrays in pageable host memory (what pickle.loads of the gRPC payload yields, aggregator.py:704 /
torch_client.py:76-78), pass through DeviceAggregator.update_weight_aggregation (pack into pinned host
memory -> async H2D -> chunked in-order reduction), and the round ends with get_weights() (D2H egress,
torch_model_adapter.py:41-47).

usage: python tools/ingress_bench.py [K] [rounds] [layout=resnet18|femnist|p25m] [pack_workers,...]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    which = sys.argv[3] if len(sys.argv) > 3 else "resnet18"
    worker_list = [int(w) for w in sys.argv[4].split(",")] if len(sys.argv) > 4 else [None]
    allout = [run(K, rounds, which, w) for w in worker_list]
    # full ingress from the executor's pickled payload (aggregator.py:704 deserialize_response)
    allout.append(run(K, rounds, which, None, loader="pickle"))
    # the mixin's deserialize_response: the same payload without copying its arrays (fedscale_amd/ingress.py)
    allout.append(run(K, rounds, which, None, loader="zerocopy"))
    # ... with the gather + H2D of each update on a background thread (ClientStaging(async_ingress=True)):
    # with no big copy left in deserialize_response, the main thread's next unpickle overlaps the gather
    allout.append(run(K, rounds, which, None, loader="zerocopy", async_ingress=True))
    # the mixin's add_event_handler: a servicer thread decodes each upload on arrival and queues it, the
    # main loop pops the queue (aggregator.py:958-959, 830-840, 984-994)
    allout.append(run(K, rounds, which, None, loader="arrival"))
    allout.append(run(K, rounds, which, None, loader="arrival", async_ingress=True))
    allout.append(egress(which))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(allout, open(os.path.join(ROOT, "gpurun_out", f"ingress_{which}_k{K}.json"), "w"), indent=1)


def _layout(which):
    """resnet18 (config 3), femnist (config 1) or p25m: the headline's 25 M fp32 parameters as 10 tensors
    of 2.5 M (a 100 MB update)."""
    import torch

    from fedscale_amd import synth

    if which == "resnet18":
        return synth.resnet18_layout()
    if which == "p25m":
        return [f"l{i}.weight" for i in range(10)], [(2500, 1000)] * 10, [torch.float32] * 10
    return synth.femnist_cnn_layout()


def run(K, rounds, which, workers, loader=None, async_ingress=False):
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    names, shapes, dtypes = _layout(which)
    model = synth.LayoutModule(names, shapes, dtypes)
    adapter = TorchModelAdapter(model, device="cuda:0")
    if workers or async_ingress:
        adapter.staging = None
        from fedscale_amd.bucket import ClientStaging

        adapter.staging = ClientStaging(adapter.layout, adapter.device, K, pack_workers=workers,
                                        async_ingress=async_ingress)
    agg = DeviceAggregator(adapter)
    rng = np.random.default_rng(0)
    pool = []
    for i in range(8):
        d = {}
        for n, t in model.state_dict().items():
            if t.dtype == torch.int64:
                d[n] = np.array(5 + i, dtype=np.int64).reshape(t.shape)
            else:
                d[n] = (t.numpy() + rng.standard_normal(t.shape, dtype=np.float32) * np.float32(0.01))
        pool.append(d)
    P = adapter.layout.P_full
    payloads = None
    if loader is not None:
        import pickle

        payloads = [pickle.dumps({"client_id": i, "moving_loss": 1.0, "trained_size": 200, "success": True,
                                  "utility": 1.0, "update_weight": d, "wall_duration": 0})
                    for i, d in enumerate(pool)]
        load = pickle.loads if loader == "pickle" else agg.deserialize_response
        t0 = time.perf_counter()
        for r in range(16):
            load(payloads[r % 8])
        t_load = (time.perf_counter() - t0) / 16
    res = []
    for r in range(rounds + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg.start_round(K)
        t_ing = 0.0
        if loader == "arrival":
            import collections
            import threading

            agg.server_events_queue = collections.deque()
            agg.device_decode_on_arrival = True
            th = threading.Thread(target=lambda: [agg.add_event_handler(k, "upload_model", None, payloads[k % 8])
                                                  for k in range(K)])
            th.start()
            done = 0
            while done < K:
                if agg.server_events_queue:
                    agg.on_result(agg.deserialize_response(agg.server_events_queue.popleft()[3]))
                    done += 1
                else:
                    time.sleep(0)
            th.join()
        for k in range(K if loader != "arrival" else 0):
            if payloads is not None:
                agg.on_result(load(payloads[k % 8]))
            else:
                agg.on_result({"client_id": k, "update_weight": pool[k % 8], "moving_loss": 1.0})
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        w = adapter.get_weights()
        t2 = time.perf_counter()
        if r > 0:  # first round warms up allocations
            res.append((t1 - t0, t2 - t1))
    t_round = float(np.median([a for a, _ in res]))
    t_egress = float(np.median([b for _, b in res]))
    out = {"layout": which, "K": K, "P": P, "round_s_incl_h2d": t_round, "egress_d2h_s": t_egress,
           "client_updates_per_s_incl_h2d": K / t_round,
           "client_updates_per_s_incl_h2d_d2h": K / (t_round + t_egress),
           "ingress_GBps": 4 * K * P / t_round / 1e9,
           "staging_capacity": adapter.staging.capacity, "pack_workers": adapter.staging.pack_workers,
           "from_payload": loader, "async_ingress": async_ingress, "loads_ms_per_update": (t_load * 1e3 if loader else None)}
    print(json.dumps(out), flush=True)
    return out


def egress(which, requests=8):
    """Egress per executor request (aggregator.py:788-804, 902-909): get_weights() + serialize_response.
    The reference pickles the weights again for every request; the mixin serves the bytes made once per
    model version."""
    import pickle

    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    names, shapes, dtypes = _layout(which)
    model = synth.LayoutModule(names, shapes, dtypes)
    adapter = TorchModelAdapter(model, device="cuda:0")
    agg = DeviceAggregator(adapter)
    rng = np.random.default_rng(1)
    upd = {n: (t.numpy() + np.float32(0.01) * rng.standard_normal(t.shape, dtype=np.float32)) if t.dtype != torch.int64
           else t.numpy() for n, t in model.state_dict().items()}
    times = {"cached": [], "reference": [], "handle": [], "get_weights": []}
    for r in range(3):
        agg.start_round(2)
        agg.on_result({"client_id": 0, "update_weight": upd, "moving_loss": 1.0})
        agg.on_result({"client_id": 1, "update_weight": upd, "moving_loss": 1.0})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(requests):
            agg.serialize_response(adapter.get_weights())
        t1 = time.perf_counter()
        for _ in range(requests):
            pickle.dumps(list(adapter.get_weights()))
        t2 = time.perf_counter()
        for _ in range(requests):  # the mixin's create_client_task path (EgressHandle)
            agg.serialize_response(adapter.egress_handle())
        t3 = time.perf_counter()
        for _ in range(requests):
            adapter.get_weights()
        t4 = time.perf_counter()
        if r > 0:
            times["cached"].append((t1 - t0) / requests)
            times["reference"].append((t2 - t1) / requests)
            times["handle"].append((t3 - t2) / requests)
            times["get_weights"].append((t4 - t3) / requests)
    out = {"egress": which, "requests_per_round": requests,
           "cached_ms_per_request": 1e3 * float(np.median(times["cached"])),
           "reference_pickle_ms_per_request": 1e3 * float(np.median(times["reference"])),
           "handle_ms_per_request": 1e3 * float(np.median(times["handle"])),
           "get_weights_clone_ms": 1e3 * float(np.median(times["get_weights"])),
           "bytes": len(agg.serialize_response(adapter.get_weights()))}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
