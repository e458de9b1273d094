"""The binary is tied to the sources (fedscale_amd/buildinfo.py): the library carries a hash of every source, header
and flag it was built from, the loader recomputes it from the tree and refuses any other library, and build()
rebuilds by that hash, not by file time.  CPU only (loading the library makes no GPU call)."""
import os
import shutil

import pytest

from fedscale_amd import _native, buildinfo


def _tree_copy(tmp_path):
    for rel in buildinfo.SRCS + buildinfo.HDRS:
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(os.path.join(buildinfo.ROOT, rel), dst)
    return tmp_path


def test_shipped_library_carries_the_trees_build_id():
    info = _native.build_info()
    assert info["build_id"] == buildinfo.source_id() == buildinfo.embedded_id(_native.LIB_PATH)
    assert info["defs"] == ""
    assert len(info["build_id"]) == 16 and int(info["build_id"], 16) >= 0


def test_unchanged_copy_of_the_sources_verifies(tmp_path):
    tree = _tree_copy(tmp_path)
    assert buildinfo.source_id(root=str(tree)) == buildinfo.source_id()
    _native.load(tree=str(tree))  # accepted


@pytest.mark.parametrize("rel", [buildinfo.SRCS[0], buildinfo.HDRS[0], "include/fedagg.h"])
def test_stale_library_is_rejected(tmp_path, rel):
    """One changed byte in any source or header: the shipped library no longer matches and load() refuses it."""
    tree = _tree_copy(tmp_path)
    with open(tree / rel, "ab") as f:
        f.write(b"\n// changed\n")
    assert buildinfo.source_id(root=str(tree)) != buildinfo.source_id()
    with pytest.raises(_native.FedAggError, match="stale"):
        _native.load(tree=str(tree))


def test_flags_and_defs_enter_the_id():
    assert buildinfo.source_id("-DQF_MAXK=1024") != buildinfo.source_id()
    assert buildinfo.source_id("-DQF_MAXK=1024") == buildinfo.source_id("  -DQF_MAXK=1024 ")


def test_missing_sources_cannot_be_verified(tmp_path):
    with pytest.raises(_native.FedAggError, match="cannot verify"):
        _native.load(tree=str(tmp_path))


def test_build_is_a_no_op_when_the_id_matches(monkeypatch):
    calls = []
    monkeypatch.setattr(buildinfo.subprocess, "run", lambda *a, **k: calls.append(a))
    assert buildinfo.build(_native.LIB_PATH) is False
    assert calls == []


def test_build_recompiles_a_library_without_the_trees_id(tmp_path, monkeypatch):
    """A library whose embedded id differs (here: a file with an old id) is rebuilt: the compiler runs on a
    temporary name and the result replaces the file only if it carries the tree's id."""
    lib = tmp_path / "libfedagg.so"
    lib.write_bytes(b"\0FA_BUILD_ID=0123456789abcdef\0")
    ran = []

    def fake_run(cmd, check, cwd):
        out = cmd[cmd.index("-o") + 1]
        ran.append(cmd)
        idarg = [c for c in cmd if c.startswith("-DFA_BUILD_ID=")][0]
        with open(out, "wb") as f:
            f.write(b"FA_BUILD_ID=" + idarg.split('"')[1].encode())

    monkeypatch.setattr(buildinfo.subprocess, "run", fake_run)
    assert buildinfo.build(str(lib)) is True
    assert len(ran) == 1 and buildinfo.embedded_id(str(lib)) == buildinfo.source_id()
    assert not [p for p in os.listdir(tmp_path) if ".tmp" in p]
