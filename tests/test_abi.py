"""CPU checks of the drop-in boundary: libzgpu.so loads and exports every symbol include/zgpu.h
declares; the ctypes mirror matches the header (no compute calls: there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zgpu.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(zgpu_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from zarrs_amd import _lib as L
    lib = L.load()
    decl = declared_functions()
    assert len(decl) >= 14
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(L.EXPORTS) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (zgpu_\w+)", out))
    assert set(decl) <= exported


def test_desc_struct_layout_matches_header():
    from zarrs_amd import _lib as L
    # const void*, uint64, 4 x uint64[8]
    assert C.sizeof(L.ChunkDesc) == 8 + 8 + 4 * 8 * 8
    assert L.ChunkDesc.chunk_shape.offset == 16


def test_status_names_and_version():
    from zarrs_amd import _lib as L
    lib = L.load()
    for i, n in enumerate(L.STATUS_NAMES):
        assert lib.zgpu_status_name(i).decode() == n
    assert b"gfx950" in lib.zgpu_version()


def test_kernels_built_for_gfx950():
    from zarrs_amd import _lib as L
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", L.LIB_PATH],
                         capture_output=True, text=True, cwd="/tmp")
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_ctx_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from zarrs_amd import Context, ZgpuError
    with pytest.raises(ZgpuError):
        Context(0)
