"""CPU tests of the C-ABI boundary: the library loads, exports every symbol include/uno_kkt.h
declares, and fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "uno_kkt.h")).read()
    return sorted(set(re.findall(r"\b(uno_kkt_[a-z_]+)\s*\(", txt)))


def test_header_declares_the_plugin_surface():
    syms = declared_symbols()
    for s in ["uno_kkt_create", "uno_kkt_analyze", "uno_kkt_factorize", "uno_kkt_inertia", "uno_kkt_solve",
              "uno_kkt_destroy", "uno_kkt_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from uno_amd import kkt
    lib = kkt.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(declared_symbols()) == set(kkt.EXPORTED_SYMBOLS)
    assert b"gfx950" in lib.uno_kkt_version()


def test_library_is_gfx950_code_object():
    so = open(os.path.join(ROOT, "uno_amd", "libuno_kkt.so"), "rb").read()
    assert b"gfx950" in so


def test_no_silent_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from uno_amd import HipKKT, KKTError
    with pytest.raises(KKTError):
        HipKKT(0)
