"""How libfedagg.so is built, and the build id that ties a binary to the sources it was built from.

The id is the first 16 hex digits of SHA-256 over (the compiler flags, any extra -D definitions, and every
source and header file of the library, by relative path and content).  The build embeds it in the library
(``-DFA_BUILD_ID``, returned by ``fa_build_id()`` and also present in the binary as the marker
``FA_BUILD_ID=<id>``), together with the extra definitions (``fa_build_defs()``).  ``_native.load()``
recomputes the id from the sources in the tree it is loaded from and refuses a library whose id differs, so
the binary a test or benchmark ran is provably the one those sources produce; ``__graft_entry__.build()``
rebuilds whenever the embedded id differs from the tree's (not by file time).

    python -m fedscale_amd.buildinfo                 # print the tree's id
    python -m fedscale_amd.buildinfo --out X.so --defs "-DQF_MAXK=1024"   # build a variant (tools/build_ab.sh)
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
#: translation units of libfedagg.so, relative to the repository root (compiled in this order)
SRCS = ("fedscale_amd/csrc/fedagg.hip", "fedscale_amd/csrc/client_update.hip", "fedscale_amd/csrc/ingress_host.cpp",
        "fedscale_amd/csrc/ingress_dma.cpp", "fedscale_amd/csrc/rccl_comm.cpp")
#: headers they include (every #include "..." of the library)
HDRS = ("fedscale_amd/csrc/fa_device.h", "include/fedagg.h", "include/fedclient.h")
FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall")
LIB = os.path.join(ROOT, "fedscale_amd", "libfedagg.so")
MARKER = b"FA_BUILD_ID="
_ID_RE = re.compile(rb"FA_BUILD_ID=([0-9a-f]{16})")


def source_id(defs: str = "", root: str = ROOT) -> str:
    """The build id of the sources under ``root`` built with FLAGS plus ``defs`` (extra -D options)."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode() + b"\0" + " ".join(defs.split()).encode() + b"\0")
    for rel in SRCS + HDRS:
        with open(os.path.join(root, rel), "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


def embedded_id(lib_path: str):
    """The id a built library carries (read from the file; nothing is loaded), or None."""
    try:
        with open(lib_path, "rb") as f:
            m = _ID_RE.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def build_cmd(out: str, defs: str = "", hipcc: str = None) -> list:
    hipcc = hipcc or os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    d = " ".join(defs.split())
    return ([hipcc] + list(FLAGS) + d.split() +
            [f"-DFA_BUILD_ID=\"{source_id(d)}\"", f"-DFA_BUILD_DEFS=\"{d}\"", "-o", out] +
            [os.path.join(ROOT, s) for s in SRCS])


def build(out: str = LIB, defs: str = "", force: bool = False) -> bool:
    """Compile ``out`` unless it already carries the tree's id for ``defs``; True when it compiled.  The library
    is written to a temporary name and renamed into place, so a process that has the old one loaded keeps a
    valid mapping."""
    want = source_id(defs)
    if not force and embedded_id(out) == want:
        return False
    tmp = out + ".tmp%d" % os.getpid()
    cmd = build_cmd(tmp, defs)
    print("[build]", " ".join(cmd), flush=True)
    try:
        subprocess.run(cmd, check=True, cwd="/tmp")
        if embedded_id(tmp) != want:
            raise RuntimeError(f"{tmp}: the build does not carry the id {want}")
        os.replace(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return True


# ---- the host staging extension (fedscale_amd/_hoststage: CPython C API, gcc) ------------------------------------
HOST_SRC = "fedscale_amd/csrc/hoststage.c"
HOST_FLAGS = ("-O2", "-shared", "-fPIC", "-Wall", "-Werror", "-std=c11")


def host_module_path() -> str:
    import sysconfig

    return os.path.join(ROOT, "fedscale_amd", "_hoststage" + sysconfig.get_config_var("EXT_SUFFIX"))


def host_source_id(root: str = ROOT) -> str:
    """Build id of the host staging extension: SHA-256 over its flags and source (as ``source_id`` does for the
    HIP library)."""
    h = hashlib.sha256()
    h.update(" ".join(HOST_FLAGS).encode() + b"\0")
    with open(os.path.join(root, HOST_SRC), "rb") as f:
        data = f.read()
    h.update(HOST_SRC.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


def build_host(out: str = None, force: bool = False) -> bool:
    """Compile the host staging extension unless it already carries the source's id; True when it compiled."""
    import sysconfig

    import numpy as np

    out = out or host_module_path()
    want = host_source_id()
    if not force and embedded_id(out) == want:
        return False
    tmp = out + ".tmp%d" % os.getpid()
    cmd = ([os.environ.get("CC", "gcc")] + list(HOST_FLAGS) +
           ["-I" + sysconfig.get_paths()["include"], "-I" + np.get_include(),
            f"-DHS_BUILD_ID=\"FA_BUILD_ID={want}\"", "-o", tmp, os.path.join(ROOT, HOST_SRC)])
    print("[build]", " ".join(cmd), flush=True)
    try:
        subprocess.run(cmd, check=True, cwd="/tmp")
        if embedded_id(tmp) != want:
            raise RuntimeError(f"{tmp}: the build does not carry the id {want}")
        os.replace(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return True


def main(argv=None) -> int:
    import argparse

    p = argparse.ArgumentParser()
    p.add_argument("--out", default=None, help="build this library (default: print the tree's id)")
    p.add_argument("--defs", default="", help="extra -D options of a tuning / A/B variant")
    p.add_argument("--force", action="store_true")
    a = p.parse_args(argv)
    if a.out is None:
        print(source_id(a.defs))
        return 0
    build(os.path.abspath(a.out), a.defs, a.force)
    print(f"{a.out}: {embedded_id(a.out)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
