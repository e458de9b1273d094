"""Where config 1's host round goes (bench.c1_host_round: FEMNIST small-CNN, K = 10 host dicts through the drop-in,
then get_weights()): the median time of start_round, of the first K-1 on_result calls, of the last one (which
reduces and applies the round) and of get_weights(), then a cProfile of 300 rounds (top functions by own time)."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import synth  # noqa: E402
from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator  # noqa: E402
from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer  # noqa: E402
from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    job = bench.c1_job_conf()
    args = argparse.Namespace(**job["args"])
    K = args.num_participants
    names, shapes, base, ups = bench._c1_updates(1, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    agg = DeviceAggregator(TorchModelAdapter(model, optimizer=TorchServerOptimizer(args.gradient_policy, args, dev),
                                             device=dev), args)

    def one_round(rec=None):
        t0 = time.perf_counter()
        agg.start_round(K)
        t1 = time.perf_counter()
        for k in range(K - 1):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        t2 = time.perf_counter()
        agg.on_result({"client_id": K - 1, "update_weight": ups[K - 1], "moving_loss": 1.0})
        t3 = time.perf_counter()
        agg.model_wrapper.get_weights()
        t4 = time.perf_counter()
        if rec is not None:
            rec.append((t1 - t0, (t2 - t1) / (K - 1), t3 - t2, t4 - t3, t4 - t0))

    for _ in range(20):
        one_round()
    torch.cuda.synchronize(dev)
    rec = []
    for _ in range(300):
        one_round(rec)
    med = np.median(np.asarray(rec), axis=0) * 1e6
    print(json.dumps({"us": {"start_round": med[0], "on_result_each_of_first_K-1": med[1], "on_result_last": med[2],
                             "get_weights": med[3], "round": med[4]}, "K": K}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        one_round()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    print(s.getvalue())


if __name__ == "__main__":
    main()
