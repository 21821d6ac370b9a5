"""PtyRAD's constraint_params schema defaults (src/ptyrad/params/constraint_params.py:6-106), as data.
Shared by make_golden_constraints.py and the GPU constraint tests (which cannot import the reference)."""

DEFAULTS = {
    "ortho_pmode": {"freq": 1},
    "probe_mask_k": {"freq": None, "radius": 0.22, "width": 0.05, "power_thresh": 0.95},
    "fix_probe_int": {"freq": 1},
    "obj_rblur": {"freq": None, "obj_type": "both", "kernel_size": 5, "std": 0.5},
    "obj_zblur": {"freq": 1, "obj_type": "both", "kernel_size": 5, "std": 1.0},
    "kr_filter": {"freq": None, "obj_type": "both", "radius": 0.15, "width": 0.05},
    "kz_filter": {"freq": None, "obj_type": "both", "beta": 1.0, "alpha": 1.0},
    "complex_ratio": {"freq": None, "obj_type": "both", "alpha1": 1.0, "alpha2": 0.0},
    "mirrored_amp": {"freq": 1, "relax": 0.1, "scale": 0.03, "power": 4.0},
    "obja_thresh": {"freq": 1, "relax": 0.0, "thresh": [0.98, 1.02]},
    "objp_postiv": {"freq": 1, "relax": 0.0, "mode": "clip_neg"},
    "tilt_smooth": {"freq": None, "std": 2.0},
}

