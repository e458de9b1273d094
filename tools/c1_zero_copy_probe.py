"""Config 1's device floor with the client rows read straight out of the pinned staging mirror (zero-copy over
PCIe) and the model written straight into pinned host memory, against H2D + reduce + D2H (tools/c1_floor.py).
Every variant ends in one stream synchronize; median over rounds, milliseconds.  The pinned buffers' device
addresses come from hipHostGetDevicePointer, and nothing is launched unless it returns the host address (the
kernel then reads the same bytes the CPU wrote).  usage: python tools/c1_zero_copy_probe.py [rounds]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(ts):
    return round(float(np.median(ts)) * 1e3, 4)


def device_pointer(hip, t) -> int:
    dp = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(t.data_ptr()), 0)
    return dp.value if rc == 0 else -rc


def main():
    import torch

    from fedscale_amd import _native
    from fedscale_amd import kernels as kx
    from fedscale_amd._native import FA_FINALIZE
    from fedscale_amd.bucket import round_up
    from fedscale_amd.state import raw_stream

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    K, P = 10, 24492
    ld = round_up(P, 64)
    g = torch.Generator().manual_seed(1)
    hx = (torch.randn(K, ld, generator=g) * 0.05).pin_memory()
    x = torch.empty(K, ld, device=dev)
    out = torch.empty(ld, device=dev)
    hout = torch.zeros(ld).pin_memory()
    hout2 = torch.zeros(ld).pin_memory()
    denom = float(np.float32(K))
    st = torch.cuda.current_stream(dev)
    sp = raw_stream(0)
    res = {"hx_devptr_is_host_ptr": device_pointer(hip, hx) == hx.data_ptr(),
           "hout_devptr_is_host_ptr": device_pointer(hip, hout2) == hout2.data_ptr()}
    print(json.dumps(res), flush=True)
    if not (res["hx_devptr_is_host_ptr"] and res["hout_devptr_is_host_ptr"]):
        print(json.dumps({"skipped": "pinned buffers are not addressable by their host pointer"}))
        return

    def base():
        x.copy_(hx, non_blocking=True)
        kx.reduce(x, K, P, out, denom=denom, finalize=True)
        hout.copy_(out, non_blocking=True)

    def zc_in():  # rows read over PCIe by the kernel, model D2H as before
        _native.call("fa_reduce", hx.data_ptr(), ld, K, P, None, None, out.data_ptr(), denom, FA_FINALIZE, sp)
        hout2.copy_(out, non_blocking=True)

    def zc_both():  # rows read over PCIe, model written into pinned host memory by the kernel
        _native.call("fa_reduce", hx.data_ptr(), ld, K, P, None, None, hout2.data_ptr(), denom, FA_FINALIZE, sp)

    def reduce_only():
        kx.reduce(x, K, P, out, denom=denom, finalize=True)

    for name, fn in (("h2d_reduce_d2h", base), ("zero_copy_in_d2h", zc_in), ("zero_copy_in_out", zc_both),
                     ("reduce_only", reduce_only)):
        ts = []
        for r in range(rounds + 20):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            st.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = med(ts[20:])
        if name != "reduce_only":
            got = hout2 if name != "h2d_reduce_d2h" else hout
            res[name + "_bit_equal"] = bool(torch.equal(got[:P], hout[:P])) if name != "h2d_reduce_d2h" else True
    res.update(unit="ms", rounds=rounds, clients=K, params=P)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
