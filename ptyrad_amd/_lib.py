"""ctypes binding of libptyx.so (include/ptyx.h).  The HIP library is REQUIRED.

There is no CPU fallback: if the shared library is missing or fails to load, every entry
point raises.  torch is imported first so that its HIP runtime (libamdhip64.so.7) is the one
that libptyx.so binds to.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libptyx)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTYX_LIB", os.path.join(_HERE, "lib", "libptyx.so"))

PTYX_ABI_VERSION = 210     # include/ptyx.h
PTYX_PREP_CALL, PTYX_PREP_FULL, PTYX_PREP_REUSE = 0, 1, 2
PTYX_PREP_DEFER_PROBE = 4  # flag bit: the probe-gradient reduction may wait for a later piece
PTYX_PREP_DEFER_GATHER = 8  # flag bit (_begin / _end): keep the object-gradient slots for the slot exchange
PTYX_PREP_GRAD_STORE = 16  # flag bit: the call overwrites d_obja / d_objp (no zeroing needed before)
PTYX_PREP_FUSED_ADAM = 32  # flag bit: the call ends with the step ptyx_plan_set_adam registered
PTYX_PREP_SELECT = 64      # flag bit: the call begins with the selection ptyx_plan_set_select registered
PTYX_SLOT_META = 8         # floats per table row of a slot-exchange rank block
PTYX_BATCH_SUMS = 37      # doubles per mini-batch of ptyx_forward_loss_grad_begin / _end
PTYX_OK, PTYX_EINVAL, PTYX_ENOMEM, PTYX_EHIP, PTYX_EUNSUPPORTED = 0, 1, 2, 3, 4
PTYX_SHIFT_PROBES = 1
PTYX_MEAS_F16 = 2
PTYX_PROP_GRAD = 4

_ERRNAMES = {1: "EINVAL", 2: "ENOMEM", 3: "EHIP", 4: "EUNSUPPORTED"}

# every symbol include/ptyx.h declares (checked by tests/test_abi.py)
EXPORTS = ("ptyx_plan_create", "ptyx_plan_destroy", "ptyx_forward", "ptyx_forward_loss_grad",
           "ptyx_forward_loss_grad_begin", "ptyx_forward_loss_grad_end", "ptyx_set_tuning", "ptyx_get_tuning",
           "ptyx_adjoint_dldi", "ptyx_profile_begin", "ptyx_profile_end", "ptyx_plan_workspace_bytes",
           "ptyx_last_error", "ptyx_version", "ptyx_constraints_ws_bytes", "ptyx_constraints_evals_offset",
           "ptyx_meas_gather", "ptyx_pacbed_ws_bytes", "ptyx_loss_pacbed", "ptyx_obj_rblur", "ptyx_blur_adjoint", "ptyx_patch_gather", "ptyx_patch_scatter_add", "ptyx_simlar_std", "ptyx_simlar_std_grad",
           "ptyx_obj_constrain", "ptyx_probe_fix_int", "ptyx_probe_ortho",
           "ptyx_plan_register_capacity", "ptyx_abi_struct_sizes", "ptyx_build_id", "ptyx_raw_read", "ptyx_meas_stats_len", "ptyx_meas_ws_bytes", "ptyx_meas_stats", "ptyx_meas_finish",
           "ptyx_meas_mean", "ptyx_meas_mean_seq", "ptyx_meas_pad_background", "ptyx_meas_pad_resample",
           "ptyx_step_select", "ptyx_step_store", "ptyx_adam_step", "ptyx_adam_step_store", "ptyx_plan_set_adam", "ptyx_plan_set_select", "ptyx_plan_check",
           "ptyx_plan_slot_floats", "ptyx_slot_block_floats", "ptyx_plan_slot_target", "ptyx_slots_export", "ptyx_obj_gather_slots",
           "ptyx_obj_gather_slots_adam")


class PtyxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ptyx {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class Dims(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("P", ctypes.c_int32), ("O", ctypes.c_int32),
                ("Nz", ctypes.c_int32), ("Ny", ctypes.c_int32), ("Nx", ctypes.c_int32),
                ("n_scans", ctypes.c_int32), ("max_patterns", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("abi_version", ctypes.c_int32)]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if len(args) < 10 and "abi_version" not in kw:
            self.abi_version = PTYX_ABI_VERSION


class Inputs(ctypes.Structure):
    _fields_ = [("obja", ctypes.c_void_p), ("objp", ctypes.c_void_p), ("probe", ctypes.c_void_p),
                ("shifts", ctypes.c_void_p), ("H", ctypes.c_void_p), ("omode_occu", ctypes.c_void_p),
                ("crop_pos", ctypes.c_void_p), ("meas", ctypes.c_void_p), ("obj_tilts", ctypes.c_void_p),
                ("kvec", ctypes.c_void_p), ("dz", ctypes.c_float), ("meas_rows", ctypes.c_void_p),
                ("meas_row_count", ctypes.c_int32)]


class Grads(ctypes.Structure):
    _fields_ = [("d_obja", ctypes.c_void_p), ("d_objp", ctypes.c_void_p),
                ("d_probe", ctypes.c_void_p), ("d_shifts", ctypes.c_void_p), ("d_H", ctypes.c_void_p),
                ("d_tilts", ctypes.c_void_p), ("d_dz", ctypes.c_void_p)]


class LossCfg(ctypes.Structure):
    _fields_ = [("single_on", ctypes.c_int32), ("single_w", ctypes.c_float), ("single_q", ctypes.c_float),
                ("poissn_on", ctypes.c_int32), ("poissn_w", ctypes.c_float), ("poissn_q", ctypes.c_float),
                ("poissn_eps", ctypes.c_float),
                ("sparse_on", ctypes.c_int32), ("sparse_w", ctypes.c_float), ("sparse_n", ctypes.c_int32),
                ("grad_scale", ctypes.c_float), ("max_batch", ctypes.c_int32), ("prep", ctypes.c_int32)]


class ObjConstraints(ctypes.Structure):
    _fields_ = [("zblur_a", ctypes.c_int32), ("zblur_p", ctypes.c_int32), ("zblur_ks", ctypes.c_int32),
                ("zblur_std", ctypes.c_float),
                ("cr_a", ctypes.c_int32), ("cr_p", ctypes.c_int32), ("cr_alpha1", ctypes.c_float),
                ("cr_alpha2", ctypes.c_float),
                ("mir_on", ctypes.c_int32), ("mir_relax", ctypes.c_float), ("mir_scale", ctypes.c_float),
                ("mir_power", ctypes.c_float),
                ("thr_on", ctypes.c_int32), ("thr_relax", ctypes.c_float), ("thr_lo", ctypes.c_float),
                ("thr_hi", ctypes.c_float),
                ("pos_on", ctypes.c_int32), ("pos_subtract_min", ctypes.c_int32), ("pos_relax", ctypes.c_float)]


class MeasProc(ctypes.Structure):
    _fields_ = [("flipud", ctypes.c_int32), ("fliplr", ctypes.c_int32), ("transpose", ctypes.c_int32),
                ("crop_ky0", ctypes.c_int32), ("crop_ky1", ctypes.c_int32), ("crop_kx0", ctypes.c_int32),
                ("crop_kx1", ctypes.c_int32), ("neg_mode", ctypes.c_int32), ("neg_force", ctypes.c_int32),
                ("neg_value", ctypes.c_float), ("norm_mode", ctypes.c_int32), ("norm_value", ctypes.c_float)]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int32), ("total_ms", ctypes.c_float)]


_lib = None


def load(path: str | None = None):
    """Load libptyx.so once and declare the prototypes.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"libptyx.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(there is no CPU fallback)")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    lib.ptyx_plan_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(Dims), ctypes.c_int]
    lib.ptyx_plan_destroy.argtypes = [vp]
    lib.ptyx_forward.argtypes = [vp, vp, ctypes.POINTER(Inputs), vp, i32, vp]
    lib.ptyx_forward_loss_grad.argtypes = [vp, vp, ctypes.POINTER(Inputs), vp, vp, i32, i32,
                                           ctypes.POINTER(LossCfg), vp, vp, ctypes.POINTER(Grads)]
    lib.ptyx_forward_loss_grad_begin.argtypes = [vp, vp, ctypes.POINTER(Inputs), vp, vp, i32, i32,
                                                 ctypes.POINTER(LossCfg), vp, ctypes.POINTER(Grads), vp]
    lib.ptyx_forward_loss_grad_end.argtypes = [vp, vp, vp, vp]
    lib.ptyx_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.ptyx_get_tuning.argtypes = [ctypes.c_char_p]
    lib.ptyx_get_tuning.restype = ctypes.c_int64
    lib.ptyx_adjoint_dldi.argtypes = [vp, vp, ctypes.POINTER(Inputs), vp, i32, vp, f32,
                                      ctypes.POINTER(Grads)]
    lib.ptyx_profile_begin.argtypes = [vp]
    lib.ptyx_profile_end.argtypes = [vp, ctypes.POINTER(KernelStat), i32, ctypes.POINTER(i32)]
    lib.ptyx_profile_begin.restype = ctypes.c_int
    lib.ptyx_profile_end.restype = ctypes.c_int
    lib.ptyx_plan_workspace_bytes.argtypes = [vp]
    lib.ptyx_plan_workspace_bytes.restype = ctypes.c_size_t
    lib.ptyx_plan_check.argtypes = [vp]
    lib.ptyx_plan_register_capacity.argtypes = [vp]
    lib.ptyx_plan_register_capacity.restype = ctypes.c_int64
    lib.ptyx_last_error.restype = ctypes.c_char_p
    lib.ptyx_version.restype = ctypes.c_int
    lib.ptyx_abi_struct_sizes.argtypes = [ctypes.POINTER(ctypes.c_size_t), i32]
    lib.ptyx_abi_struct_sizes.restype = ctypes.c_int
    lib.ptyx_build_id.restype = ctypes.c_char_p
    lib.ptyx_constraints_ws_bytes.restype = ctypes.c_size_t
    lib.ptyx_constraints_evals_offset.restype = ctypes.c_size_t
    lib.ptyx_obj_rblur.argtypes = [vp, vp, vp, i32, i32, i32, i32, f32]
    lib.ptyx_pacbed_ws_bytes.argtypes = [i32, i32]
    lib.ptyx_pacbed_ws_bytes.restype = ctypes.c_size_t
    lib.ptyx_loss_pacbed.argtypes = [vp, vp, vp, i32, vp, vp, i32, i32, i32, f32, f32, f32, vp, vp, vp]
    lib.ptyx_meas_gather.argtypes = [vp, vp, i32, i32, i32, vp, i32, vp, i32, i32, i32, i32,
                                     ctypes.c_double, ctypes.c_double, i32, i32, vp]
    lib.ptyx_blur_adjoint.argtypes = [vp, vp, vp, i32, i32, i32, i32, f32]
    lib.ptyx_patch_gather.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, i32, i32, vp]
    lib.ptyx_patch_scatter_add.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, i32, i32, vp]
    lib.ptyx_obj_constrain.argtypes = [vp, vp, vp, i32, i32, i32, i32, ctypes.POINTER(ObjConstraints), vp]
    lib.ptyx_probe_fix_int.argtypes = [vp, vp, i32, i32, vp, vp]
    lib.ptyx_probe_ortho.argtypes = [vp, vp, i32, i32, vp]
    i64 = ctypes.c_int64
    lib.ptyx_raw_read.argtypes = [vp, ctypes.c_char_p, i64, i32, i32, i32, i64, i64, i64, vp]
    lib.ptyx_meas_stats_len.argtypes = [i32, i32]
    lib.ptyx_meas_stats_len.restype = ctypes.c_size_t
    lib.ptyx_meas_ws_bytes.argtypes = [i32, i32]
    lib.ptyx_meas_ws_bytes.restype = ctypes.c_size_t
    lib.ptyx_meas_stats.argtypes = [vp, vp, i64, i32, i32, ctypes.POINTER(MeasProc), vp, vp]
    lib.ptyx_meas_finish.argtypes = [vp, vp, i64, i32, i32, ctypes.POINTER(MeasProc), vp, vp, vp, i32]
    lib.ptyx_meas_mean.argtypes = [vp, i32, i32, ctypes.POINTER(MeasProc), vp, vp, vp]
    lib.ptyx_meas_mean_seq.argtypes = [vp, vp, i64, i32, i32, ctypes.POINTER(MeasProc), vp, vp, i32, vp]
    lib.ptyx_meas_pad_background.argtypes = [vp, vp, i32, i32, i32, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                             i32, i32, i32, i32, vp]
    lib.ptyx_meas_pad_resample.argtypes = [vp, vp, i32, i64, i32, i32, vp, i32, i32, i32, i32, i32, i32, vp, i32]
    lib.ptyx_step_select.argtypes = [vp, vp, vp, vp, i32, vp, vp, i64, vp, i32]
    lib.ptyx_simlar_std.argtypes = [vp, vp, i32, i64, i32, vp, vp]
    lib.ptyx_simlar_std_grad.argtypes = [vp, vp, i32, i64, i32, vp, vp, vp]
    lib.ptyx_step_store.argtypes = [vp, vp, i32, vp, vp, vp]
    d64 = ctypes.c_double
    lib.ptyx_adam_step.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, d64, d64, d64, d64, i32]
    lib.ptyx_adam_step_store.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, d64, d64, d64, d64, i32, vp, i32, vp, vp, vp]
    lib.ptyx_plan_set_adam.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, d64, d64, d64, d64, i32, vp, i32, vp, vp, vp]
    lib.ptyx_plan_set_select.argtypes = [vp, vp, vp, vp, vp, i64, vp, i32]
    lib.ptyx_plan_slot_floats.argtypes = [vp]
    lib.ptyx_plan_slot_floats.restype = ctypes.c_int64
    lib.ptyx_plan_slot_target.argtypes = [vp, vp, i32]
    lib.ptyx_slot_block_floats.argtypes = [vp, i32]
    lib.ptyx_slot_block_floats.restype = ctypes.c_int64
    lib.ptyx_slots_export.argtypes = [vp, vp, i32, i32, vp, vp]
    lib.ptyx_obj_gather_slots.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp, i32, vp]
    lib.ptyx_obj_gather_slots_adam.argtypes = lib.ptyx_obj_gather_slots.argtypes
    for name in ("ptyx_plan_slot_target", "ptyx_slots_export", "ptyx_obj_gather_slots", "ptyx_obj_gather_slots_adam", "ptyx_plan_check", "ptyx_adam_step", "ptyx_adam_step_store", "ptyx_plan_set_adam", "ptyx_plan_set_select", "ptyx_step_select", "ptyx_step_store", "ptyx_plan_create", "ptyx_plan_destroy", "ptyx_forward", "ptyx_forward_loss_grad",
                 "ptyx_forward_loss_grad_begin", "ptyx_forward_loss_grad_end", "ptyx_set_tuning",
                 "ptyx_adjoint_dldi", "ptyx_meas_gather", "ptyx_loss_pacbed", "ptyx_obj_rblur", "ptyx_blur_adjoint", "ptyx_patch_gather",
                 "ptyx_patch_scatter_add", "ptyx_obj_constrain", "ptyx_probe_fix_int",
                 "ptyx_probe_ortho", "ptyx_raw_read", "ptyx_meas_stats", "ptyx_meas_finish",
                 "ptyx_meas_mean", "ptyx_meas_mean_seq", "ptyx_meas_pad_background", "ptyx_meas_pad_resample",
                 "ptyx_simlar_std", "ptyx_simlar_std_grad"):
        getattr(lib, name).restype = ctypes.c_int
    _check_abi(lib)
    _lib = lib
    return lib


STRUCTS = ("Dims", "Inputs", "Grads", "LossCfg", "KernelStat", "ObjConstraints", "MeasProc")   # header order


def _check_abi(lib):
    """The library's ABI version and C struct sizes must match these ctypes mirrors, and its build
    id the sources next to it (PTYX_LIB pointing elsewhere, e.g. a variant build, skips that)."""
    if "PTYX_LIB" not in os.environ:
        from .csrc import build as _build
        want, got = _build.source_hash(), lib.ptyx_build_id().decode()
        if got != want:
            raise ImportError(f"libptyx.so was built from other sources (build id {got[:12]} != {want[:12]}): "
                              "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    if lib.ptyx_version() != PTYX_ABI_VERSION:
        raise ImportError(f"libptyx.so ABI {lib.ptyx_version()} != {PTYX_ABI_VERSION}: rebuild the library")
    sizes = (ctypes.c_size_t * len(STRUCTS))()
    lib.ptyx_abi_struct_sizes(sizes, len(STRUCTS))
    for name, sz in zip(STRUCTS, sizes):
        if ctypes.sizeof(globals()[name]) != sz:
            raise ImportError(f"ctypes {name} is {ctypes.sizeof(globals()[name])} B, libptyx.so says {sz} B")


def set_tuning(key: str, value: int) -> None:
    """ptyx_set_tuning: select an engine variant (tests / A/B runs; -1 = the measured default)."""
    check(load().ptyx_set_tuning(key.encode(), int(value)))


TUNING_KEYS = ("s3_hold", "s_psi0", "s_gather", "s_defer_groups", "gather_split", "gen_wg_per_cu", "gather_rows", "fmm_hold_h", "fuse_adam", "tail_fin", "small_spec", "sel_fold", "rows_hu", "psi_hold", "gadam_lead")   # ptyx_set_tuning's keys


def get_tuning(key: str) -> int:
    return int(load().ptyx_get_tuning(key.encode()))


def check(rc: int):
    if rc != PTYX_OK:
        raise PtyxError(rc, _lib.ptyx_last_error().decode(errors="replace"))
