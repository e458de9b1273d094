"""Phase timing of BASELINE config 1's host round through the drop-in (bench.c1_host_round), median over
rounds: start_round, the first upload (begins the device round), the middle uploads, the last upload
(stages it and applies the round), get_weights (D2H + clone).  usage: python tools/c1_breakdown.py [rounds]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    K = 10
    names, shapes, _, ups = bench._c1_updates(0, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    agg = DeviceAggregator(TorchModelAdapter(model, device=dev))
    ph = {k: [] for k in ("start_round", "first_upload", "middle_uploads_each", "last_upload_and_apply",
                          "get_weights", "round")}
    for r in range(rounds + 10):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        agg.start_round(K)
        t1 = time.perf_counter()
        agg.on_result({"client_id": 0, "update_weight": ups[0], "moving_loss": 1.0})
        t2 = time.perf_counter()
        for k in range(1, K - 1):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        t3 = time.perf_counter()
        agg.on_result({"client_id": K - 1, "update_weight": ups[K - 1], "moving_loss": 1.0})
        t4 = time.perf_counter()
        agg.model_wrapper.get_weights()
        t5 = time.perf_counter()
        if r >= 10:
            for k, v in zip(ph, (t1 - t0, t2 - t1, (t3 - t2) / (K - 2), t4 - t3, t5 - t4, t5 - t0)):
                ph[k].append(v)
    print(json.dumps({k: round(float(np.median(v)) * 1e3, 4) for k, v in ph.items()} | {"unit": "ms", "rounds": rounds}))


if __name__ == "__main__":
    main()
