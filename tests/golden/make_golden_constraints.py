"""Golden fixtures for the on-device constraints, made by running the
reference's own CombinedConstraint (src/ptyrad/constraints.py:227-246).

Run here (build container) only:  python tests/golden/make_golden_constraints.py
Writes tests/golden/cons_<case>.npz with the inputs (obja, objp, probe, probe_int_sum, niter,
constraint_params as JSON) and the reference's outputs (out_obja, out_objp, out_probe).

obj_rblur calls torchvision.transforms.functional.gaussian_blur, which is absent from this image.
For the one case that switches it on (cons_rblur) the stub is given torchvision's published
algorithm restated in torch (_tv_gaussian_blur below), so that fixture pins the reference's call
site (axes, order, parameters) but not torchvision itself: "parity unpinned" for that kernel.
Every other case runs with gaussian_blur stubbed to raise.  Data only; no reference source is
copied.
"""
import copy
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from refimport import REF_SRC, import_reference  # noqa: E402

import_reference()
import ptyrad.constraints as cons  # noqa: E402

from constraint_defaults import DEFAULTS  # noqa: E402


def _tv_gaussian_blur(img, kernel_size, sigma):
    """torchvision.transforms.functional.gaussian_blur restated (tensor input, float32)."""
    ks = [kernel_size, kernel_size] if isinstance(kernel_size, int) else list(kernel_size)
    sg = [float(sigma), float(sigma)] if not isinstance(sigma, (list, tuple)) else [float(s) for s in sigma]

    def k1d(k, s):
        half = (k - 1) * 0.5
        x = torch.linspace(-half, half, steps=k)
        pdf = torch.exp(-0.5 * (x / s).pow(2))
        return pdf / pdf.sum()

    kx, ky = k1d(ks[0], sg[0]), k1d(ks[1], sg[1])
    k2 = torch.mm(ky[:, None], kx[None, :]).to(img.dtype)
    shape = img.shape
    x = img.reshape(-1, 1, shape[-2], shape[-1])
    x = torch.nn.functional.pad(x, [ks[0] // 2, ks[0] // 2, ks[1] // 2, ks[1] // 2], mode="reflect")
    y = torch.nn.functional.conv2d(x, k2[None, None])
    return y.reshape(shape)


def make_state(O, Nz, Ny, Nx, P, N, seed):
    rng = np.random.default_rng(seed)
    obja = (1.0 + 0.04 * rng.standard_normal((O, Nz, Ny, Nx))).astype(np.float32)
    objp = (0.05 + 0.1 * rng.standard_normal((O, Nz, Ny, Nx))).astype(np.float32)
    yy, xx = np.mgrid[:N, :N] - N / 2
    base = np.exp(-(yy ** 2 + xx ** 2) / (2 * (N / 8) ** 2))
    probe = np.stack([base * (0.6 ** p) * np.exp(1j * (p + 1) * 0.3 * (xx + 0.5 * yy) / N)
                      + 0.05 * (rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
                      for p in range(P)]).astype(np.complex64)
    return obja, objp, probe


class _Model:
    """The attributes CombinedConstraint reads (constraints.py:34-224)."""

    def __init__(self, obja, objp, probe, probe_int_sum):
        self.opt_obja = torch.nn.Parameter(torch.tensor(obja))
        self.opt_objp = torch.nn.Parameter(torch.tensor(objp))
        self.opt_probe = torch.nn.Parameter(torch.view_as_real(torch.tensor(probe)).contiguous())
        self.opt_obj_tilts = torch.nn.Parameter(torch.zeros(1, 2))
        self.probe_int_sum = torch.tensor(probe_int_sum, dtype=torch.float32)
        self.device = "cpu"
        self.N_scan_slow = self.N_scan_fast = 1

    def get_complex_probe_view(self):
        return torch.view_as_complex(self.opt_probe)


def run_case(name, cp_over, shape, niter=1, seed=0, rblur=False, int_scale=1.1):
    cp = copy.deepcopy(DEFAULTS)
    for k, v in cp_over.items():
        cp[k].update(v)
    O, Nz, Ny, Nx, P, N = shape
    obja, objp, probe = make_state(O, Nz, Ny, Nx, P, N, seed)
    probe_int_sum = float((np.abs(probe.astype(np.complex128)) ** 2).sum() * int_scale)
    m = _Model(obja, objp, probe, probe_int_sum)
    tvf = sys.modules["torchvision.transforms.functional"]
    saved = cons.gaussian_blur
    if rblur:
        cons.gaussian_blur = _tv_gaussian_blur
    try:
        cons.CombinedConstraint(cp, device="cpu", verbose=False)(m, niter)
    finally:
        cons.gaussian_blur = saved
    out = os.path.join(HERE, f"cons_{name}.npz")
    np.savez_compressed(out, obja=obja, objp=objp, probe=probe, probe_int_sum=np.float32(probe_int_sum),
                        niter=np.int64(niter), constraint_params=json.dumps(cp),
                        rblur_torchvision_restated=np.bool_(rblur),
                        out_obja=m.opt_obja.detach().numpy(), out_objp=m.opt_objp.detach().numpy(),
                        out_probe=torch.view_as_complex(m.opt_probe.detach()).numpy())
    print("wrote", out, os.path.getsize(out), "bytes")
    del tvf


def main():
    torch.manual_seed(0)
    # schema defaults (obj_rblur needs torchvision: see cons_rblur), single mode, c2-like
    run_case("default_p1", {}, (1, 1, 70, 90, 1, 32), seed=1)
    # mixed state + multislice: ortho_pmode over 4 modes, z-blur across 6 slices, 2 object modes
    run_case("default_p4o2z6", {}, (2, 6, 48, 56, 4, 32), seed=2)
    # relaxed / alternative branches and the reductions (complex_ratio Cbar, subtract_min)
    run_case("options", {"obj_zblur": {"obj_type": "amplitude", "kernel_size": 3, "std": 0.8},
                         "complex_ratio": {"freq": 1, "alpha1": 0.7, "alpha2": 0.2},
                         "mirrored_amp": {"relax": 0.5, "scale": 0.5, "power": 2.0},
                         "obja_thresh": {"relax": 0.3, "thresh": [0.95, 1.03]},
                         "objp_postiv": {"relax": 0.2, "mode": "subtract_min"},
                         "ortho_pmode": {"freq": None}},
             (1, 3, 40, 44, 2, 32), seed=3)
    # frequency gating: niter 3 with freq 2 (skipped) and 3 (applied)
    run_case("freq", {"obj_zblur": {"freq": 2}, "mirrored_amp": {"freq": 3, "relax": 0.0},
                      "obja_thresh": {"freq": 2}, "objp_postiv": {"freq": 3, "relax": 0.5},
                      "fix_probe_int": {"freq": 2}},
             (1, 2, 36, 40, 3, 32), niter=3, seed=4)
    # Fourier-space filters (torch-on-device path): kr, kz, probe mask
    run_case("fourier", {"kr_filter": {"freq": 1, "obj_type": "phase", "radius": 0.3, "width": 0.05},
                         "kz_filter": {"freq": 1, "obj_type": "both", "beta": 0.5, "alpha": 2.0},
                         "probe_mask_k": {"freq": 1, "radius": 0.5, "width": 0.05, "power_thresh": 0.9}},
             (1, 4, 40, 48, 3, 32), seed=5)
    # lateral blur (torchvision restated, see module docstring)
    run_case("rblur", {"obj_rblur": {"freq": 1, "obj_type": "both", "kernel_size": 5, "std": 0.5}},
             (2, 2, 33, 47, 1, 32), seed=6, rblur=True)
    run_case("rblur_k7", {"obj_rblur": {"freq": 1, "obj_type": "phase", "kernel_size": 7, "std": 1.3},
                          "obj_zblur": {"freq": None}},
             (1, 1, 64, 64, 1, 32), seed=7, rblur=True)


if __name__ == "__main__":
    assert os.path.isdir(REF_SRC), "the reference is needed to (re)generate fixtures"
    main()
