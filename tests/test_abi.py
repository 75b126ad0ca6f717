"""CPU checks of the C-ABI boundary: the library loads and exports every declared symbol."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "md2.h")
LIB = os.path.join(ROOT, "monodepth2.jl_amd", "lib", "libmd2hip.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(md2_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_symbols():
    syms = declared_symbols()
    assert "md2_loss_fwd_bwd" in syms and "md2_abi_version" in syms


def test_library_exports_all_symbols():
    assert os.path.exists(LIB), "build libmd2hip.so first (make -C monodepth2.jl_amd/csrc)"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    lib.md2_abi_version.restype = ctypes.c_int
    assert lib.md2_abi_version() == 2
    lib.md2_last_error.restype = ctypes.c_char_p
    assert lib.md2_last_error() is not None
