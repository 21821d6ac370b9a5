"""The C-ABI library loads and exports every symbol include/ptyx.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

from ptyrad_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ptyx.h")).read()
    return sorted(set(re.findall(r"\b(ptyx_[a-z_]+)\s*\(", src)))


def test_header_matches_python_exports():
    assert sorted(_lib.EXPORTS) == header_symbols()


def test_library_loads_and_exports_all_symbols():
    lib = _lib.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.ptyx_version() >= 100
    assert lib.ptyx_last_error() == b""


def test_struct_layouts_match_header():
    # sizes of the C structs (all 4-byte fields / 8-byte pointers, no padding surprises)
    assert ctypes.sizeof(_lib.Dims) == 9 * 4
    assert ctypes.sizeof(_lib.Inputs) == 10 * 8 + 8     # + float dz, padded to pointer alignment
    assert ctypes.sizeof(_lib.Grads) == 7 * 8
    assert ctypes.sizeof(_lib.LossCfg) == 12 * 4
    assert ctypes.sizeof(_lib.ObjConstraints) == 19 * 4


def test_plan_create_rejects_bad_dims_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    d = _lib.Dims(100, 1, 1, 1, 200, 200, 4, 4, 0)   # N=100 unsupported -> checked before any HIP call
    rc = lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0)
    assert rc == _lib.PTYX_EUNSUPPORTED
    assert b"N must be" in lib.ptyx_last_error()
    d = _lib.Dims(128, 1, 9, 1, 200, 200, 4, 4, 0)   # too many object modes
    assert lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0) == _lib.PTYX_EUNSUPPORTED
    d = _lib.Dims(128, 1, 1, 1, 100, 200, 4, 4, 0)   # object smaller than the window
    assert lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0) == _lib.PTYX_EINVAL
    assert lib.ptyx_plan_create(None, ctypes.byref(d), 0) == _lib.PTYX_EINVAL


def test_constraint_entry_points_validate_without_gpu():
    lib = _lib.load()
    assert lib.ptyx_constraints_ws_bytes() >= 8 * 8
    assert lib.ptyx_constraints_evals_offset() < lib.ptyx_constraints_ws_bytes()
    # argument checks happen before any HIP call
    assert lib.ptyx_obj_rblur(None, None, None, 1, 32, 32, 4, 1.0) == _lib.PTYX_EUNSUPPORTED   # even kernel
    assert lib.ptyx_obj_rblur(None, None, None, 1, 2, 32, 5, 1.0) == _lib.PTYX_EINVAL          # reflect pad
    assert lib.ptyx_probe_ortho(None, None, 17, 32, None) == _lib.PTYX_EUNSUPPORTED             # > 16 modes
    c = _lib.ObjConstraints()
    c.zblur_a, c.zblur_ks, c.zblur_std = 1, 6, 1.0
    assert lib.ptyx_obj_constrain(None, ctypes.c_void_p(8), ctypes.c_void_p(8), 1, 2, 4, 4, ctypes.byref(c),
                                  None) == _lib.PTYX_EUNSUPPORTED
    assert b"odd" in lib.ptyx_last_error()


def test_stage_entry_points_validate_without_gpu():
    lib = _lib.load()
    vp = ctypes.c_void_p(8)
    assert lib.ptyx_blur_adjoint(None, vp, vp, 1, 32, 32, 4, 1.0) == _lib.PTYX_EUNSUPPORTED     # even kernel
    assert lib.ptyx_blur_adjoint(None, vp, vp, 1, 2, 32, 5, 1.0) == _lib.PTYX_EINVAL            # reflect pad
    assert lib.ptyx_blur_adjoint(None, vp, vp, 1, 32, 32, 5, 0.0) == _lib.PTYX_EINVAL           # sigma
    assert lib.ptyx_blur_adjoint(None, vp, vp, 0, 32, 32, 5, 1.0) == _lib.PTYX_OK               # empty
    assert lib.ptyx_patch_gather(None, vp, 1, 1, 16, 16, vp, vp, 2, 32, vp) == _lib.PTYX_EINVAL  # N > object
    assert b"larger than the object" in lib.ptyx_last_error()
    assert lib.ptyx_patch_gather(None, vp, 1, 1, 64, 64, vp, vp, 70000, 32, vp) == _lib.PTYX_EUNSUPPORTED
    assert lib.ptyx_patch_scatter_add(None, vp, 1, 1, 64, 64, None, vp, 3, 32, vp) == _lib.PTYX_EINVAL
    assert lib.ptyx_patch_scatter_add(None, vp, 1, 1, 64, 64, None, None, 0, 32, None) == _lib.PTYX_OK

