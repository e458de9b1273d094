"""One rank of the SPMD RCCL probe, run as a child process with a deadline (``state.spmd_rccl_probe``).

    python -m fedscale_amd.rccl_probe --nranks N --rank R --device D --id <hex of the 128-byte ncclUniqueId>

Opens a communicator of its own over the N ranks (fa_rccl_init_rank: ncclCommInitRank, which blocks until every
rank has joined), asks RCCL for its rank count, rank and device (fa_rccl_comm_info), closes it and prints one JSON
line.  Running it in a child lets the parent rank give up after a deadline: a rank whose init fails, or that never
starts, cannot leave the others blocked in ncclCommInitRank.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--id", required=True)
    a = ap.parse_args(argv)
    out = {"rank": a.rank, "device": a.device}
    try:
        from . import _native
        from .state import comm_info

        raw = bytes.fromhex(a.id)
        if len(raw) != 128:
            raise ValueError(f"the unique id has {len(raw)} bytes, not 128")
        idbuf = (ctypes.c_char * 128).from_buffer_copy(raw)
        h = ctypes.c_void_p()
        _native.call("fa_rccl_init_rank", a.nranks, idbuf, a.rank, a.device, ctypes.byref(h))
        try:
            info = comm_info(h, 1)
        finally:
            _native.call("fa_rccl_destroy", h)
        out.update({"ok": True, "count": info["count"], "user_rank": info["ranks"][0], "cu_device": info["devices"][0]})
    except Exception as e:  # reported to the parent, which exchanges it with the other ranks
        out.update({"ok": False, "error": f"{type(e).__name__}: {e}"})
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
