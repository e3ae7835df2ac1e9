"""CPU-side checks of the C ABI boundary: libsfx.so loads and exports every symbol that
include/sfx.h declares, with the ctypes signatures the Python layer binds.  No compute."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sfx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sfx_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("sfx_create", "sfx_gpi", "sfx_update", "sfx_update_all", "sfx_select_action"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from sfx import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # every declared function is bound with a signature in the Python layer
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_version_and_error_strings():
    from sfx import _lib

    assert "gfx950" in _lib.version()
    # a failing call (bad geometry) reports through sfx_last_error without touching a GPU
    h = ctypes.c_void_p()
    rc = _lib.lib.sfx_create(ctypes.byref(h), 0, 1, 1, 0, None, 1, 1, 1, 0, None)
    assert rc != 0
    assert b"geometry" in _lib.lib.sfx_last_error()


def test_kernels_compiled_for_gfx950():
    from sfx import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
