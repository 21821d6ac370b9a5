"""CombinedConstraint on the device — drop-in for src/ptyrad/constraints.py:CombinedConstraint.

Same constructor (constraint_params, device, verbose), same forward(model, niter) and the same
order of application (constraints.py:227-246).  The default-on constraints and the options that
are plain point-wise / reduction work run as HIP kernels of libptyx.so (ptyx_constraints.hpp):

  ortho_pmode    ptyx_probe_ortho    (Gram matrix, fp64 complex Jacobi, V^H M; no host sync)
  fix_probe_int  ptyx_probe_fix_int
  obj_rblur      ptyx_obj_rblur      (torchvision gaussian_blur, reflect padding)
  obj_zblur, complex_ratio, mirrored_amp, obja_thresh, objp_postiv
                 ptyx_obj_constrain  (one fused pass over the object in the default chain)
  tilt_smooth    ptyx_obj_rblur on the (2, N_scan_slow, N_scan_fast) tilt maps

The Fourier-space filters that are off by default (probe_mask_k, kr_filter, kz_filter) run as
torch-ROCm FFT ops on the same device, restating the reference's arithmetic.  There is no CPU
path: the HIP entry points raise if libptyx.so is missing.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _on(cp, name, niter):
    c = cp.get(name) or {}
    f = c.get("freq")
    return f is not None and niter % f == 0


def object_footprint(cp, niter):
    """What iteration ``niter``'s object constraints read (constraints.py:83-208): 'global' for the
    Fourier filters (kr / kz), the lateral blur, objp_postiv's subtract_min (the global minimum)
    and complex_ratio (its Cbar = Σ|ln A| / Σ|φ| sums the whole object, constraints.py:352);
    'pointwise' when only per-pixel ones run (obj_zblur acts along z at one (y, x), mirrored_amp,
    obja_thresh, objp_postiv clip_neg); else 'none'.  The band exchange refreshes the whole object
    before a 'global' iteration only."""
    blur = cp.get("obj_rblur") or {}
    pos = cp.get("objp_postiv") or {}
    if _on(cp, "kr_filter", niter) or _on(cp, "kz_filter", niter) or _on(cp, "complex_ratio", niter) or \
            (_on(cp, "obj_rblur", niter) and blur.get("std", 0) != 0) or \
            (_on(cp, "objp_postiv", niter) and pos.get("mode", "clip_neg") == "subtract_min"):
        return "global"
    if any(_on(cp, k, niter) for k in ("obj_zblur", "mirrored_amp", "obja_thresh", "objp_postiv")):
        return "pointwise"
    return "none"


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream) if t.is_cuda else ctypes.c_void_p(0)


def _vprint(msg, verbose):
    if verbose:
        print(msg, flush=True)


# --------------------------------------------------------------- torch-on-device filters (rare options)
def _sigmoid_mask(Npix, radius, width, device):
    """utils/math_ops.py:52-95 (make_sigmoid_mask, centre Npix // 2)."""
    k = torch.arange(Npix, dtype=torch.float32, device=device)
    gy, gx = torch.meshgrid(k, k, indexing="ij")
    kR = torch.sqrt((gy - Npix // 2) ** 2 + (gx - Npix // 2) ** 2)
    return 1 / (1 + torch.exp((kR - Npix * radius / 2) / (width * Npix) * 10))


def _sort_by_mode_int(modes):
    """constraints.py:249-253."""
    w = modes.abs().pow(2).sum(tuple(range(1, modes.ndim)))
    return modes[torch.sort(w, descending=True).indices]


def kr_filter(obj, radius, width):
    """constraints.py:293-304."""
    Ny, Nx = obj.shape[-2:]
    mask = _sigmoid_mask(min(Ny, Nx), radius, width, obj.device)
    W = torch.fft.ifftshift(torch.nn.functional.interpolate(mask[None, None], size=(Ny, Nx)), dim=(-2, -1)).squeeze()
    return torch.real(torch.fft.ifft2(torch.fft.fft2(obj) * W[None, None]))


def kz_filter(obj, beta, alpha, obj_type):
    """constraints.py:306-331."""
    Nz, Ny, Nx = obj.shape[-3:]
    kz, ky, kx = (torch.fft.fftfreq(n).to(obj.device) for n in (Nz, Ny, Nx))
    gz, gy, gx = torch.meshgrid(kz, ky, kx, indexing="ij")
    W = 1 - torch.atan((beta * torch.abs(gz) / torch.sqrt(gx ** 2 + gy ** 2 + 1e-3)) ** 2) / (torch.pi / 2)
    Wa = W * torch.exp(-alpha * (gx ** 2 + gy ** 2))
    f = torch.real(torch.fft.ifftn(torch.fft.fftn(obj, dim=(-3, -2, -1)) * Wa[None], dim=(-3, -2, -1)))
    return 1 + 0.9 * (f - 1) if obj_type == "amplitude" else f


def probe_mask_k(probe, radius, width, power_thresh):
    """constraints.py:43-68."""
    Npix = probe.size(-1)
    powers = probe.abs().pow(2).sum((-2, -1)) / probe.abs().pow(2).sum()
    idx = int((powers.cumsum(0) > power_thresh).nonzero()[0].item())
    mask = torch.ones_like(probe, dtype=torch.float32)
    mask[:idx + 1] = _sigmoid_mask(Npix, radius, width, probe.device)
    sh = lambda x: torch.fft.fftshift(x, dim=(-2, -1))    # noqa: E731
    ish = lambda x: torch.fft.ifftshift(x, dim=(-2, -1))  # noqa: E731
    pk = sh(torch.fft.fft2(ish(probe), norm="ortho"))
    pr = sh(torch.fft.ifft2(ish(mask * pk), norm="ortho"))
    return _sort_by_mode_int(pr), idx


# --------------------------------------------------------------- the module
class CombinedConstraint(torch.nn.Module):
    """constraints.py:15-246 on the device (see the module docstring)."""

    def __init__(self, constraint_params, device="cuda", verbose=True):
        super().__init__()
        self.device = device
        self.constraint_params = constraint_params
        self.verbose = verbose
        self._lib = _lib.load()
        self._ws = {}

    def _workspace(self, dev):
        key = str(dev)
        if key not in self._ws:
            n = int(self._lib.ptyx_constraints_ws_bytes())
            self._ws[key] = torch.zeros((n + 7) // 8, dtype=torch.float64, device=dev)
        return self._ws[key]

    # ---- probe
    def apply_ortho_pmode(self, model, niter):
        """constraints.py:34-41."""
        if not _on(self.constraint_params, "ortho_pmode", niter):
            return
        pr = model.opt_probe.data
        P, N = pr.shape[0], pr.shape[1]
        if P > 1:   # one mode: V = [1], the reference's matmul returns the probe unchanged
            _lib.check(self._lib.ptyx_probe_ortho(_stream(pr), _ptr(pr), P, N, _ptr(self._workspace(pr.device))))
        if self.verbose:
            pint = model.get_complex_probe_view().abs().pow(2)
            pw = (pint.sum((1, 2)) / pint.sum()).detach().cpu().numpy().round(3)
            _vprint(f"Apply ortho pmode constraint at iter {niter}, relative pmode power = {pw}, "
                    f"probe int sum = {pint.sum():.4f}", True)

    def apply_probe_mask_k(self, model, niter):
        """constraints.py:43-68 (torch FFT on the device)."""
        if not _on(self.constraint_params, "probe_mask_k", niter):
            return
        c = self.constraint_params["probe_mask_k"]
        pr, idx = probe_mask_k(model.get_complex_probe_view(), c["radius"], c["width"], c["power_thresh"])
        model.opt_probe.data = torch.view_as_real(pr).contiguous()
        _vprint(f"Apply Fourier-space probe amplitude constraint at iter {niter}, pmode_index = {idx} when "
                f"power_thresh = {c['power_thresh']}", self.verbose)

    def apply_fix_probe_int(self, model, niter):
        """constraints.py:70-81."""
        if not _on(self.constraint_params, "fix_probe_int", niter):
            return
        pr = model.opt_probe.data
        target = torch.as_tensor(model.probe_int_sum, dtype=torch.float32, device=pr.device).reshape(1).contiguous()
        _lib.check(self._lib.ptyx_probe_fix_int(_stream(pr), _ptr(pr), pr.shape[0], pr.shape[1], _ptr(target),
                                                _ptr(self._workspace(pr.device))))
        if self.verbose:
            _vprint(f"Apply fix probe int constraint at iter {niter}, probe int sum = "
                    f"{model.get_complex_probe_view().abs().pow(2).sum():.4f}", True)

    # ---- object
    def _rblur(self, t, ks, std):
        out = torch.empty_like(t)
        Ny, Nx = t.shape[-2:]
        _lib.check(self._lib.ptyx_obj_rblur(_stream(t), _ptr(t), _ptr(out), t.numel() // (Ny * Nx), Ny, Nx, int(ks),
                                            float(std)))
        return out

    def apply_obj_rblur(self, model, niter):
        """constraints.py:83-98."""
        c = self.constraint_params.get("obj_rblur") or {}
        if not (_on(self.constraint_params, "obj_rblur", niter) and c.get("std", 0) != 0):
            return
        if c["obj_type"] in ("amplitude", "both"):
            model.opt_obja.data = self._rblur(model.opt_obja.data.contiguous(), c["kernel_size"], c["std"])
            _vprint(f"Apply lateral (y,x) Gaussian blur with std = {c['std']} px on obja at iter {niter}", self.verbose)
        if c["obj_type"] in ("phase", "both"):
            model.opt_objp.data = self._rblur(model.opt_objp.data.contiguous(), c["kernel_size"], c["std"])
            _vprint(f"Apply lateral (y,x) Gaussian blur with std = {c['std']} px on objp at iter {niter}", self.verbose)

    def _obj_cfg(self, niter, zblur, pointwise):
        cp, c = self.constraint_params, _lib.ObjConstraints()
        z = cp.get("obj_zblur") or {}
        if zblur and _on(cp, "obj_zblur", niter) and z.get("std", 0) != 0:
            c.zblur_a = int(z["obj_type"] in ("amplitude", "both"))
            c.zblur_p = int(z["obj_type"] in ("phase", "both"))
            c.zblur_ks, c.zblur_std = int(z["kernel_size"]), float(z["std"])
        if not pointwise:
            return c
        if _on(cp, "complex_ratio", niter):
            r = cp["complex_ratio"]
            c.cr_a = int(r["obj_type"] in ("amplitude", "both"))
            c.cr_p = int(r["obj_type"] in ("phase", "both"))
            c.cr_alpha1, c.cr_alpha2 = float(r["alpha1"]), float(r["alpha2"])
        if _on(cp, "mirrored_amp", niter):
            m = cp["mirrored_amp"]
            c.mir_on, c.mir_relax, c.mir_scale, c.mir_power = 1, float(m["relax"]), float(m["scale"]), float(m["power"])
        if _on(cp, "obja_thresh", niter):
            t = cp["obja_thresh"]
            c.thr_on, c.thr_relax, c.thr_lo, c.thr_hi = 1, float(t["relax"]), float(t["thresh"][0]), float(t["thresh"][1])
        if _on(cp, "objp_postiv", niter):
            p = cp["objp_postiv"]
            c.pos_on, c.pos_relax = 1, float(p["relax"])
            c.pos_subtract_min = int(p.get("mode", "clip_neg") == "subtract_min")
        return c

    def _constrain(self, model, cfg):
        a, p = model.opt_obja.data, model.opt_objp.data
        if not (a.is_contiguous() and p.is_contiguous()):
            a, p = a.contiguous(), p.contiguous()
            model.opt_obja.data, model.opt_objp.data = a, p
        O, Nz, Ny, Nx = a.shape
        _lib.check(self._lib.ptyx_obj_constrain(_stream(a), _ptr(a), _ptr(p), O, Nz, Ny, Nx, ctypes.byref(cfg),
                                                _ptr(self._workspace(a.device))))

    def apply_object_chain(self, model, niter):
        """obj_zblur (:100-114) → kr_filter (:116-130) → kz_filter (:132-145) → complex_ratio
        (:147-163) → mirrored_amp (:165-179) → obja_thresh (:181-190) → objp_postiv (:192-208).
        Without the Fourier filters this is one fused kernel pass."""
        cp = self.constraint_params
        kr, kz = _on(cp, "kr_filter", niter), _on(cp, "kz_filter", niter)
        if kr or kz:
            self._constrain(model, self._obj_cfg(niter, zblur=True, pointwise=False))
            if kr:
                c = cp["kr_filter"]
                if c["obj_type"] in ("amplitude", "both"):
                    model.opt_obja.data = kr_filter(model.opt_obja, c["radius"], c["width"]).contiguous()
                if c["obj_type"] in ("phase", "both"):
                    model.opt_objp.data = kr_filter(model.opt_objp, c["radius"], c["width"]).contiguous()
            if kz:
                c = cp["kz_filter"]
                if c["obj_type"] in ("amplitude", "both"):
                    model.opt_obja.data = kz_filter(model.opt_obja, c["beta"], c["alpha"], "amplitude").contiguous()
                if c["obj_type"] in ("phase", "both"):
                    model.opt_objp.data = kz_filter(model.opt_objp, c["beta"], c["alpha"], "phase").contiguous()
            self._constrain(model, self._obj_cfg(niter, zblur=False, pointwise=True))
        else:
            self._constrain(model, self._obj_cfg(niter, zblur=True, pointwise=True))
        if self.verbose:
            a, p = model.opt_obja, model.opt_objp
            _vprint(f"Applied object constraints at iter {niter}: obja range ({a.min().item():.3f}, "
                    f"{a.max().item():.3f}), objp range ({p.min().item():.3f}, {p.max().item():.3f})", True)

    def apply_tilt_smooth(self, model, niter):
        """constraints.py:210-225 (the same reflect-padded Gaussian as obj_rblur, kernel 5)."""
        c = self.constraint_params.get("tilt_smooth") or {}
        if not (_on(self.constraint_params, "tilt_smooth", niter) and c.get("std", 0) != 0):
            return
        if model.opt_obj_tilts.shape[0] == 1:
            _vprint("`tilt_smooth` constraint requires `tilt_type':'each'`, skip this constraint", self.verbose)
            return
        t = model.opt_obj_tilts.data.reshape(model.N_scan_slow, model.N_scan_fast, 2).permute(2, 0, 1).contiguous()
        model.opt_obj_tilts.data = self._rblur(t, 5, c["std"]).permute(1, 2, 0).reshape(-1, 2).contiguous()

    def object_footprint(self, niter):
        """'none' / 'pointwise' / 'global': what this iteration's object constraints read (the
        band exchange keeps only a rank's own rows current; recon_step syncs before 'global')."""
        return object_footprint(self.constraint_params, niter)

    def forward(self, model, niter):
        """constraints.py:227-246."""
        with torch.no_grad():
            self.apply_ortho_pmode(model, niter)
            self.apply_probe_mask_k(model, niter)
            self.apply_fix_probe_int(model, niter)
            self.apply_obj_rblur(model, niter)
            self.apply_object_chain(model, niter)
            self.apply_tilt_smooth(model, niter)
