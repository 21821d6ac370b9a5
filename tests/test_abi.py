"""The C-ABI library loads and exports every symbol include/ptyx.h declares (no GPU needed)."""
import ctypes
import os
import re
import subprocess

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


STRUCT_C = {"Dims": "ptyx_dims", "Inputs": "ptyx_inputs", "Grads": "ptyx_grads", "LossCfg": "ptyx_loss_cfg",
            "KernelStat": "ptyx_kernel_stat", "ObjConstraints": "ptyx_obj_constraints", "MeasProc": "ptyx_meas_proc"}


def c_layout(tmp_path, classes):
    """{struct: (sizeof, {field: offsetof})} from the C compiler on include/ptyx.h."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ptyx.h"', "int main(void) {"]
    for py, cs in classes.items():
        lines.append(f'  printf("S {py} %zu\\n", sizeof({cs}));')
        for f, _ in getattr(_lib, py)._fields_:
            lines.append(f'  printf("F {py} {f} %zu\\n", offsetof({cs}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n"):
        parts = ln.split()
        if parts and parts[0] == "S":
            out.setdefault(parts[1], [0, {}])[0] = int(parts[2])
        elif parts and parts[0] == "F":
            out.setdefault(parts[1], [0, {}])[1][parts[2]] = int(parts[3])
    return out


def py_layout(cls):
    return ctypes.sizeof(cls), {f: getattr(cls, f).offset for f, _ in cls._fields_}


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror in ptyrad_amd/_lib.py has the C header's size and field offsets, and
    names every C field (gcc on include/ptyx.h), and the library agrees on the sizes."""
    c = c_layout(tmp_path, STRUCT_C)
    hdr = open(os.path.join(ROOT, "include", "ptyx.h")).read()
    for py, cs in STRUCT_C.items():
        size, offs = py_layout(getattr(_lib, py))
        assert c[py][0] == size, (py, c[py][0], size)
        assert c[py][1] == offs, py
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cs, cs), hdr, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        cnames = re.findall(r"\*?\s*(\w+)\s*(?:\[\d+\])?\s*[,;]", body)
        assert sorted(cnames) == sorted(offs), (py, cnames)
    lib = _lib.load()          # load() itself checks ptyx_abi_struct_sizes against the mirrors
    sizes = (ctypes.c_size_t * 7)()
    assert lib.ptyx_abi_struct_sizes(sizes, 7) == 7
    assert list(sizes) == [c[py][0] for py in STRUCT_C]


def integration_stub():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.search(r"## 1\. Minimal ctypes stub.*?```python\n(.*?)```", text, re.S).group(1)


def test_integration_stub_matches_header_and_library(tmp_path, monkeypatch):
    """The binding INTEGRATION.md shows PtyRAD maintainers, executed as written: its structs have
    the header's layout field for field, check_abi() passes against libptyx.so, and a plan request
    travels through its Dims (abi_version included) to the library's validation."""
    monkeypatch.setenv("PTYX_LIB", _lib.LIB_PATH)
    _lib.load()
    ns = {}
    exec(compile(integration_stub(), "INTEGRATION.md", "exec"), ns)
    c = c_layout(tmp_path, {k: STRUCT_C[k] for k in ("Dims", "Inputs", "Grads", "LossCfg")})
    for py in ("Dims", "Inputs", "Grads", "LossCfg"):
        assert py_layout(ns[py]) == (c[py][0], c[py][1]), py
    ns["check_abi"]()

    class M:   # N = 88 (8·11) is rejected by ptyx_plan_create before any HIP call
        opt_obja = __import__("torch").zeros((1, 1, 200, 200))
        opt_probe = __import__("torch").zeros((1, 88, 88, 2))
        crop_pos = __import__("torch").zeros((4, 2), dtype=__import__("torch").int32)
        shift_probes = True
    with pytest.raises(RuntimeError, match="N must be"):
        ns["make_plan"](M, 4)


def test_plan_create_rejects_stale_abi_version():
    lib = _lib.load()
    h = ctypes.c_void_p()
    d = _lib.Dims(128, 1, 1, 1, 200, 200, 4, 4, 0, 101)
    assert lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0) == _lib.PTYX_EINVAL
    assert b"abi_version" in lib.ptyx_last_error()


def test_plan_create_rejects_bad_dims_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    d = _lib.Dims(88, 1, 1, 1, 200, 200, 4, 4, 0)    # N=88 = 8·11 unsupported -> checked before any HIP call
    rc = lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0)
    assert rc == _lib.PTYX_EUNSUPPORTED
    assert b"N must be" in lib.ptyx_last_error()
    for n in (16, 121, 264, 540, 1024):    # below 32, 11², 8·3·11, above 512
        d = _lib.Dims(n, 1, 1, 1, 600, 600, 4, 4, 0)
        assert lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(d), 0) == _lib.PTYX_EUNSUPPORTED, n
    d = _lib.Dims(128, 1, 33, 1, 200, 200, 4, 4, 0)  # too many object modes (> 32)
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
    assert lib.ptyx_probe_ortho(None, None, 65, 32, None) == _lib.PTYX_EUNSUPPORTED             # > 64 modes
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
    assert lib.ptyx_simlar_std(None, vp, 33, 4, 16, vp, vp) == _lib.PTYX_EUNSUPPORTED          # O > 32
    assert lib.ptyx_simlar_std(None, vp, 0, 4, 16, vp, vp) == _lib.PTYX_EINVAL                 # no modes
    assert lib.ptyx_simlar_std(None, None, 2, 4, 16, vp, vp) == _lib.PTYX_EINVAL               # null x
    assert lib.ptyx_simlar_std(None, None, 2, 0, 16, None, None) == _lib.PTYX_OK               # empty
    assert lib.ptyx_simlar_std_grad(None, vp, 2, 4, 16, vp, vp, vp) == _lib.PTYX_EINVAL        # gx aliases x
    assert lib.ptyx_simlar_std_grad(None, None, 2, 0, 16, None, None, None) == _lib.PTYX_OK




def test_tuning_keys_round_trip_without_gpu():
    """Every key _lib.TUNING_KEYS names (the GPU tests' tuning fixture resets exactly these) is a
    library key that takes -1 (the measured default) and reads back; unknown keys are refused."""
    for k in _lib.TUNING_KEYS:
        before = _lib.get_tuning(k)
        _lib.set_tuning(k, -1)
        assert _lib.get_tuning(k) == -1, k
        _lib.set_tuning(k, before)
    lib = _lib.load()
    assert lib.ptyx_set_tuning(b"no_such_key", 1) == _lib.PTYX_EINVAL
    assert lib.ptyx_get_tuning(b"no_such_key") == -2


def test_plan_set_adam_validates_without_gpu():
    """ptyx_plan_set_adam (ABI 209) refuses a null plan and null arrays before touching the device;
    a PTYX_PREP_FUSED_ADAM call needs a registered step (checked in tests/test_gpu_stepgraph.py)."""
    lib = _lib.load()
    rc = lib.ptyx_plan_set_adam(None, 0, None, None, None, None, None, None, None, 0.9, 0.999, 1e-8, 0.0, 0,
                                None, 0, None, None, None)
    assert rc == _lib.PTYX_EINVAL and b"plan is null" in lib.ptyx_last_error()
    assert _lib.PTYX_PREP_FUSED_ADAM == 32
    assert _lib.get_tuning("fuse_adam") == -1


def test_plan_set_select_validates_without_gpu():
    """ptyx_plan_set_select (ABI 210) refuses a null plan before touching the device."""
    lib = _lib.load()
    rc = lib.ptyx_plan_set_select(None, None, None, None, None, 0, None, 0)
    assert rc == _lib.PTYX_EINVAL and b"plan is null" in lib.ptyx_last_error()
    assert _lib.PTYX_PREP_SELECT == 64 and _lib.get_tuning("sel_fold") == -1
