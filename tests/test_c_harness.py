"""The C ABI from C++ (tests/c/abi_harness.cpp): compiled with g++ against include/zgpu.h and linked
to libzgpu.so, as a cgo / JNI / Rust FFI binding would use it. CPU: argument checks, status names,
clean failure without a device. GPU: decodes through the C ABI only, bit-exact, with the reference's
error statuses (incl. UnexpectedChunkDecodedSize lengths and an empty inner chunk of a shard)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "zarrs_amd", "lib")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("abi") / "abi_harness")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-o", exe,
                           os.path.join(ROOT, "tests", "c", "abi_harness.cpp"), "-L" + LIB, "-lzgpu",
                           "-Wl,-rpath," + LIB])
    return exe


def _run(exe):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_c_harness_cpu_part(harness):
    out = _run(harness)
    assert "PASS" in out


@pytest.mark.gpu
def test_c_harness_gpu_part(harness):
    out = _run(harness)
    assert "gpu: ran" in out and "PASS" in out
