"""Interleaved timing of fa_qfed_accumulate variants (fedscale_amd/variants/libfedagg_qf2_*.so) in one process,
with and without the fused FedAvg chain.  Every variant's delta (and chain) must equal the first one's bit for bit.
usage: python tools/tune_qfed2.py [K] [P] [rounds] [acc]   (acc: time FA_ACCUMULATE launches, a later pass of a
streamed round: delta and the chain are read back)"""
import ctypes
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    later = len(sys.argv) > 4 and sys.argv[4] == "acc"
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    V, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "fedscale_amd", "variants", "libfedagg_qf2_*.so"))):
        lib = ctypes.CDLL(path)
        f = lib.fa_qfed_accumulate
        f.restype = I32
        f.argtypes = [V, I64, I32, I64, V, V, F, V, V, V, V, I64, I32, V]
        ws = lib.fa_qfed_workspace_bytes
        ws.restype, ws.argtypes = I64, [I32, I64, I64]
        name = os.path.basename(path)[len("libfedagg_qf2_"):-3]
        for chain in (False, True):
            libs[name + ("+chain" if chain else "")] = (f, chain, ws(K, round_up(P, 64), P))
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=3)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=3 + 90000, scale_noise=0.0)
    alpha = torch.rand(K, device="cuda") + 0.5
    delta = torch.empty(ld, device="cuda")
    chain = torch.empty(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = torch.empty(max(w for _, _, w in libs.values()) // 8 + 1, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    times = {n: [] for n in libs}
    rels = {}
    ref = ref_chain = ref_sq = None
    for r in range(rounds):
        for n, (f, use_chain, wsb) in libs.items():
            sq.zero_()
            args = (x.data_ptr(), ld, K, P, last.data_ptr(), alpha.data_ptr(), 0.05, delta.data_ptr(),
                    chain.data_ptr() if use_chain else None, sq.data_ptr(), ws.data_ptr(), wsb, 0, st)
            assert f(*args) == 0, n
            torch.cuda.synchronize()
            if later:  # time later passes: the chains continue from the first call's delta / chain
                args = args[:12] + (1,) + args[13:]
            if ref is None:
                ref, ref_sq = delta.clone(), sq.clone()
            else:
                if not torch.equal(delta, ref):
                    print(f"MISMATCH {n}: delta differs", flush=True)
                rel = ((sq - ref_sq).abs() / ref_sq).max().item()
                # variants with another fp32 partial length (QF_PART, _p*) round the norms differently
                assert rel < 1e-8, f"{n}: sqnorm differs by {rel}"
                rels[n] = max(rels.get(n, 0.0), rel)
            if use_chain:
                if ref_chain is None:
                    ref_chain = chain.clone()
                else:
                    assert torch.equal(chain, ref_chain), f"{n}: chain differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f(*args)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 3)
    # the chain equals the plain FedAvg sum (fa_reduce EPI_CHAIN) of the same rows
    if ref_chain is not None:
        from fedscale_amd import kernels as kx
        acc = torch.empty(ld, device="cuda")
        kx.reduce(x, K, P, acc)
        assert torch.equal(acc[:P], ref_chain[:P]), "chain != FedAvg sum"
    b = 4 * K * P + 8 * P + 8 * K
    print(f"--- K={K} P={P} {'FA_ACCUMULATE passes ' if later else ''}(GB/s over 4KP + 8P + 8K; +chain moves 4P more)")
    for n, t in sorted(times.items(), key=lambda kv: np.median(kv[1])):
        print(f"{n:40s} {np.median(t):8.3f} ms {b / (np.median(t) * 1e-3) / 1e9:8.1f} GB/s  sqnorm rel {rels.get(n, 0.0):.1e}", flush=True)


if __name__ == "__main__":
    main()
