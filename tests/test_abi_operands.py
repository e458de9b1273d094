"""The C ABI's device scope and operand checks (fedscale_amd/csrc/fa_device.h) on the CPU: the header is
compiled with g++ against a mock HIP runtime of 8 GPUs (tests/csrc/mock_hip), so the multi-device cases the
one-GPU box cannot stage run here — an input on another GPU than the call's (stream- or output-selected),
pageable and pinned host memory, extents past an allocation, pointer tables (one query per allocation).
tests/test_gpu_abi_operands.py runs the same checks through the real library on the GPU."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_devscope_operand_checks_against_a_mock_runtime(tmp_path):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / "devscope_test")
    src = os.path.join(HERE, "csrc", "devscope_test.cpp")
    subprocess.run([cxx, "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(HERE, "csrc", "mock_hip"), "-o", exe,
                    src], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED: 0 failure(s)" in r.stdout
    assert sum(line.startswith("ok ") for line in r.stdout.splitlines()) >= 19
