"""CPU: libmvpose.so loads and exports every symbol include/mvpose.h declares;
argument validation fails loudly before any device work."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mvpose.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mvp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "mvp_triangulate" in syms and "mvp_last_error" in syms


def test_library_exports_every_declared_symbol():
    from mvpose import _lib
    missing = [s for s in declared_symbols() if not hasattr(_lib.lib, s)]
    assert not missing, f"libmvpose.so lacks {missing}"
    # and the ctypes table covers the header exactly
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_abi_version():
    from mvpose import _lib
    assert _lib.lib.mvp_abi_version() == 1


def test_argument_errors_are_reported():
    from mvpose import _lib
    ci = (ctypes.c_int * 2)(0, 5)
    rc = _lib.lib.mvp_triangulate(None, 10, 2, None, 2, ci, 2, 0, None, None, None)
    assert rc == -1
    assert "cam_idx[1]=5" in _lib.last_error()
    with pytest.raises(_lib.MvposeError):
        _lib.call("mvp_triangulate", None, 10, 2, None, 2, ci, 2, 7, None, None, None)


def test_camera_pack_matches_numpy():
    import numpy as np
    from mvpose import _lib, ops, synthetic as syn
    c = syn.make_rig(2, seed=3)[1]
    out = np.zeros(40)
    P = ctypes.POINTER(ctypes.c_double)
    args = [np.ascontiguousarray(a, dtype=np.float64) for a in (c["K"], c["dist"], c["R"], c["T"])]
    _lib.call("mvp_camera_pack", *[a.ctypes.data_as(P) for a in args], out.ctypes.data_as(P))
    ref = ops.pack_camera(c["K"], c["R"], c["T"], c["dist"])
    np.testing.assert_allclose(out, ref, rtol=1e-15, atol=1e-9)
