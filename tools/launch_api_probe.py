"""What the first HIP call after a kernel launch costs on the host (config 1's finish pays ~7 us for the event record
that follows its launch).  Launch config 1's fa_reduce_mirror (10 x 24,492 from pinned rows), then time ONE follow-up
call: torch's Event.record, a raw hipEventRecord through ctypes on an event made with hipEventCreateWithFlags
(disable-timing), hipStreamQuery, or a second launch; and, for comparison, each call with no launch before it.
Median microseconds of 300 rounds (20 untimed)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedscale_amd import _native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _native.load()
    hip = ctypes.CDLL("libamdhip64.so")
    K, P = 10, 24492
    ld = (P + 63) // 64 * 64
    hx = torch.randn(K, ld).pin_memory()
    out = torch.zeros(ld, device=dev)
    mir = torch.zeros(ld).pin_memory()
    s = torch.cuda.Stream(device=dev)
    st = s.cuda_stream
    tev = torch.cuda.Event()
    raw = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(raw), ctypes.c_uint(2)) == 0  # hipEventDisableTiming
    denom = float(np.float32(K))

    def launch():
        return lib.fa_reduce_mirror(hx.data_ptr(), ld, K, P, None, None, out.data_ptr(), mir.data_ptr(), denom, 2, st)

    tev.record(s)
    torch.cuda.synchronize(dev)
    nullst = torch.cuda.default_stream(dev)
    other = torch.cuda.Stream(device=dev)
    follow = {
        "null_stream_wait_event_torch": lambda: nullst.wait_event(tev),
        "null_stream_wait_event_raw": lambda: hip.hipStreamWaitEvent(ctypes.c_void_p(0), ctypes.c_void_p(tev.cuda_event), 0),
        "pool_stream_wait_event_torch": lambda: other.wait_event(tev),
        "torch_event_record": lambda: tev.record(s),
        "raw_hipEventRecord": lambda: hip.hipEventRecord(raw, ctypes.c_void_p(st)),
        "hipStreamQuery": lambda: hip.hipStreamQuery(ctypes.c_void_p(st)),
        "second_launch": launch,
    }
    res = {}
    for name, fn in follow.items():
        for after_launch in (True, False):
            ts = []
            for r in range(320):
                torch.cuda.synchronize(dev)
                if after_launch:
                    launch()
                    if "wait_event" in name:  # the event of that launch, as the adapter's join waits on
                        tev.record(s)
                t0 = time.perf_counter()
                fn()
                t1 = time.perf_counter()
                if r >= 20:
                    ts.append(t1 - t0)
            res[f"{name}{'_after_launch' if after_launch else '_idle'}"] = round(float(np.median(ts)) * 1e6, 2)
    ts = []
    for r in range(320):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        launch()
        t1 = time.perf_counter()
        if r >= 20:
            ts.append(t1 - t0)
    res["launch_idle"] = round(float(np.median(ts)) * 1e6, 2)
    print(json.dumps({"follow_up_call_us": res}), flush=True)


if __name__ == "__main__":
    main()
