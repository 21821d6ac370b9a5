"""CPU oracle for PtyRAD's iteration-wise constraints.

TEST INFRASTRUCTURE ONLY: imported by tests/, never by ptyrad_amd (the product path runs the
HIP kernels of ptyrad_amd/csrc/ptyx_constraints.hpp and fails loudly without them).

NumPy restatement, float64 by default, of src/ptyrad/constraints.py (reference @ 0.1.0b9):

  CombinedConstraint.forward order            constraints.py:227-246
  ortho_pmode  / orthogonalize_modes_vec      :34-41, :255-291 (+ sort_by_mode_int :249-253)
  probe_mask_k                                :43-68  (make_sigmoid_mask utils/math_ops.py:52-95)
  fix_probe_int                               :70-81
  obj_rblur (torchvision gaussian_blur)       :83-98
  obj_zblur (gaussian_blur_1d)                :100-114 (utils/image_proc.py:435-455)
  kr_filter / kz_filter                       :116-145, :293-331
  complex_ratio                               :147-163, :333-358
  mirrored_amp                                :165-179
  obja_thresh                                 :181-190
  objp_postiv                                 :192-208

Pinning: tests/golden/make_golden_constraints.py runs the reference CombinedConstraint itself
and stores inputs/outputs (tests/golden/cons_*.npz); tests/test_constraints_oracle.py checks
this module against them.  obj_rblur calls torchvision.transforms.functional.gaussian_blur,
which is absent from this image: its restatement here follows torchvision's published
algorithm (1-D kernel exp(-x²/2σ²) on linspace(-(k-1)/2, (k-1)/2, k), f32, normalised; 2-D
kernel = outer product; reflect padding) and is "parity unpinned" against the reference.
"""
from __future__ import annotations

import numpy as np


# ------------------------------------------------------------------ kernels
def gaussian1d_scipy(size, std):
    """utils/image_proc.py:435-441 (scipy.signal.windows.gaussian, norm=True), f64 → f32 like :449."""
    n = np.arange(size, dtype=np.float64) - (size - 1) / 2.0
    k = np.exp(-0.5 * (n / std) ** 2)
    return (k / k.sum()).astype(np.float32)


def gaussian1d_torchvision(size, sigma):
    """torchvision.transforms.functional._get_gaussian_kernel1d (f32)."""
    half = (size - 1) * 0.5
    x = np.linspace(-half, half, size, dtype=np.float32)
    pdf = np.exp(-0.5 * (x / np.float32(sigma)) ** 2).astype(np.float32)
    return (pdf / pdf.sum(dtype=np.float32)).astype(np.float32)


# ------------------------------------------------------------------ object constraints
def obj_rblur(obj, ks, std):
    """constraints.py:83-98: torchvision gaussian_blur over the last two axes, reflect padding."""
    k = gaussian1d_torchvision(ks, std).astype(np.float64)
    k2 = np.outer(k.astype(np.float32), k.astype(np.float32)).astype(np.float64)
    h = ks // 2
    pad = [(0, 0)] * (obj.ndim - 2) + [(h, h), (h, h)]
    x = np.pad(obj.astype(np.float64), pad, mode="reflect")
    Ny, Nx = obj.shape[-2:]
    out = np.zeros(obj.shape, np.float64)
    for i in range(ks):
        for j in range(ks):
            out += k2[i, j] * x[..., i:i + Ny, j:j + Nx]
    return out


def obj_zblur(obj, ks, std):
    """constraints.py:100-114 → gaussian_blur_1d (image_proc.py:443-455): conv1d 'same' along z,
    replicate padding, kernel from get_gaussian1d(norm=True) cast to the tensor dtype."""
    k = gaussian1d_scipy(ks, std).astype(np.float64)
    h = ks // 2
    Nz = obj.shape[1]
    x = obj.astype(np.float64)
    out = np.zeros(obj.shape, np.float64)
    for j in range(ks):
        zs = np.clip(np.arange(Nz) + j - h, 0, Nz - 1)
        out += k[j] * x[:, zs]
    return out


def sigmoid_mask(Npix, radius, width):
    """utils/math_ops.py:52-95 (make_sigmoid_mask, centre Npix//2)."""
    ky = np.arange(Npix, dtype=np.float32)
    gy, gx = np.meshgrid(ky, ky, indexing="ij")
    c = Npix // 2
    kR = np.sqrt((gy - c) ** 2 + (gx - c) ** 2)
    with np.errstate(over="ignore"):
        return 1.0 / (1.0 + np.exp((kR - Npix * radius / 2) / (width * Npix) * 10))


def kr_filter(obj, radius, width):
    """constraints.py:293-304: sigmoid top-hat in (ky, kx), nearest-resized to (Ny, Nx)."""
    Ny, Nx = obj.shape[-2:]
    n = min(Ny, Nx)
    m = sigmoid_mask(n, radius, width)
    iy = np.floor(np.arange(Ny) * (n / Ny)).astype(int)     # F.interpolate mode='nearest'
    ix = np.floor(np.arange(Nx) * (n / Nx)).astype(int)
    W = np.fft.ifftshift(m[iy][:, ix], axes=(-2, -1))
    return np.real(np.fft.ifft2(np.fft.fft2(obj) * W))


def kz_filter(obj, beta, alpha, obj_type):
    """constraints.py:306-331."""
    Nz, Ny, Nx = obj.shape[-3:]
    kz, ky, kx = (np.fft.fftfreq(n) for n in (Nz, Ny, Nx))
    gz, gy, gx = np.meshgrid(kz, ky, kx, indexing="ij")
    W = 1 - np.arctan((beta * np.abs(gz) / np.sqrt(gx ** 2 + gy ** 2 + 1e-3)) ** 2) / (np.pi / 2)
    Wa = W * np.exp(-alpha * (gx ** 2 + gy ** 2))
    f = np.real(np.fft.ifftn(np.fft.fftn(obj, axes=(-3, -2, -1)) * Wa[None], axes=(-3, -2, -1)))
    if obj_type == "amplitude":
        f = 1 + 0.9 * (f - 1)
    return f


def complex_ratio(obja, objp, alpha1, alpha2):
    """constraints.py:333-358; returns (objac, objpc, Cbar)."""
    la = np.log(obja.astype(np.float64))
    cbar = np.abs(la).sum() / (np.abs(objp.astype(np.float64)).sum() + 1e-8)
    objac = np.exp((1 - alpha1) * la - alpha1 * cbar * objp)
    objpc = (1 - alpha2) * objp - alpha2 / (cbar + 1e-8) * la
    return objac, objpc, cbar


def mirrored_amp(obja, objp, relax, scale, power):
    """constraints.py:165-179."""
    amp_new = 1 - scale * np.power(np.maximum(objp, 0.0), power)
    return relax * obja + (1 - relax) * amp_new


def obja_thresh(obja, relax, lo, hi):
    """constraints.py:181-190."""
    return relax * obja + (1 - relax) * np.clip(obja, lo, hi)


def objp_postiv(objp, relax, mode="clip_neg"):
    """constraints.py:192-208."""
    mod = objp - objp.min() if mode == "subtract_min" else np.maximum(objp, 0.0)
    return relax * objp + (1 - relax) * mod


# ------------------------------------------------------------------ probe constraints
def sort_by_mode_int(modes):
    """constraints.py:249-253 (descending intensity)."""
    w = (np.abs(modes) ** 2).reshape(modes.shape[0], -1).sum(1)
    return modes[np.argsort(-w, kind="stable")]


def orthogonalize_modes(modes, sort=True):
    """constraints.py:255-291: A = M M^H, eigenvectors V, ortho = V^H M (then sorted).
    Eigenvectors follow LAPACK geev's normalisation (unit norm, largest component real > 0)."""
    P = modes.shape[0]
    M = modes.reshape(P, -1).astype(np.complex128)
    A = M @ M.conj().T
    _, V = np.linalg.eig(A)
    for i in range(P):
        v = V[:, i] / np.linalg.norm(V[:, i])
        k = int(np.argmax(np.abs(v) ** 2))
        V[:, i] = v * (np.conj(v[k]) / abs(v[k]))
    ortho = (V.conj().T @ M).reshape(modes.shape)
    return sort_by_mode_int(ortho) if sort else ortho


def fix_probe_int(probe, probe_int_sum):
    """constraints.py:70-81."""
    cur = np.sqrt((np.abs(probe.astype(np.complex128)) ** 2).sum())
    return probe * (np.sqrt(probe_int_sum) / cur)


def probe_mask_k(probe, radius, width, power_thresh):
    """constraints.py:43-68 (fftshift2(fft2(ifftshift2(.), ortho)) sandwich)."""
    Npix = probe.shape[-1]
    pw = (np.abs(probe) ** 2).sum((-2, -1)) / (np.abs(probe) ** 2).sum()
    idx = int(np.nonzero(np.cumsum(pw) > power_thresh)[0][0])
    mask = np.ones(probe.shape, np.float64)
    mask[:idx + 1] = sigmoid_mask(Npix, radius, width)
    sh = lambda x: np.fft.fftshift(x, axes=(-2, -1))     # noqa: E731
    ish = lambda x: np.fft.ifftshift(x, axes=(-2, -1))   # noqa: E731
    pk = sh(np.fft.fft2(ish(probe), norm="ortho"))
    pr = sh(np.fft.ifft2(ish(mask * pk), norm="ortho"))
    return sort_by_mode_int(pr)


# ------------------------------------------------------------------ CombinedConstraint.forward
def _on(cp, name, niter):
    f = cp.get(name, {}).get("freq")
    return f is not None and niter % f == 0


def combined(cp, state, niter):
    """constraints.py:227-246 on a dict state {obja, objp, probe (complex), probe_int_sum}; returns
    the updated state (float64 / complex128)."""
    a = state["obja"].astype(np.float64)
    p = state["objp"].astype(np.float64)
    pr = state["probe"].astype(np.complex128)
    if _on(cp, "ortho_pmode", niter):
        pr = orthogonalize_modes(pr, sort=True)
    if _on(cp, "probe_mask_k", niter):
        c = cp["probe_mask_k"]
        pr = probe_mask_k(pr, c["radius"], c["width"], c["power_thresh"])
    if _on(cp, "fix_probe_int", niter):
        pr = fix_probe_int(pr, float(state["probe_int_sum"]))
    c = cp.get("obj_rblur", {})
    if _on(cp, "obj_rblur", niter) and c.get("std", 0) != 0:
        if c["obj_type"] in ("amplitude", "both"):
            a = obj_rblur(a, c["kernel_size"], c["std"])
        if c["obj_type"] in ("phase", "both"):
            p = obj_rblur(p, c["kernel_size"], c["std"])
    c = cp.get("obj_zblur", {})
    if _on(cp, "obj_zblur", niter) and c.get("std", 0) != 0:
        if c["obj_type"] in ("amplitude", "both"):
            a = obj_zblur(a, c["kernel_size"], c["std"])
        if c["obj_type"] in ("phase", "both"):
            p = obj_zblur(p, c["kernel_size"], c["std"])
    if _on(cp, "kr_filter", niter):
        c = cp["kr_filter"]
        if c["obj_type"] in ("amplitude", "both"):
            a = kr_filter(a, c["radius"], c["width"])
        if c["obj_type"] in ("phase", "both"):
            p = kr_filter(p, c["radius"], c["width"])
    if _on(cp, "kz_filter", niter):
        c = cp["kz_filter"]
        if c["obj_type"] in ("amplitude", "both"):
            a = kz_filter(a, c["beta"], c["alpha"], "amplitude")
        if c["obj_type"] in ("phase", "both"):
            p = kz_filter(p, c["beta"], c["alpha"], "phase")
    if _on(cp, "complex_ratio", niter):
        c = cp["complex_ratio"]
        ac, pc, _ = complex_ratio(a, p, c["alpha1"], c["alpha2"])
        if c["obj_type"] in ("amplitude", "both"):
            a = ac
        if c["obj_type"] in ("phase", "both"):
            p = pc
    if _on(cp, "mirrored_amp", niter):
        c = cp["mirrored_amp"]
        a = mirrored_amp(a, p, c["relax"], c["scale"], c["power"])
    if _on(cp, "obja_thresh", niter):
        c = cp["obja_thresh"]
        a = obja_thresh(a, c["relax"], c["thresh"][0], c["thresh"][1])
    if _on(cp, "objp_postiv", niter):
        c = cp["objp_postiv"]
        p = objp_postiv(p, c["relax"], c.get("mode", "clip_neg"))
    return {"obja": a, "objp": p, "probe": pr}
