"""ptyx ORACLE — CPU restatement of PtyRAD's per-mini-batch hot path.  TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``ptyrad_amd``) never routes through it and fails loudly without the HIP library.

What it restates (NumPy, written from the equations, not from the reference code):

* patch gather        — ``src/ptyrad/models.py:251-265``  (get_obj_ROI)
* sub-px probe shift  — ``src/ptyrad/utils/image_proc.py:495-537`` (imshift_batch) with the
                        grid ``arange(N)/N`` of ``models.py:179``
* forward model       — ``src/ptyrad/forward.py:20-80`` (multislice_forward_model_vec_all)
* loss terms          — ``src/ptyrad/losses.py:36-104, 143-155`` (single / poissn / sparse)
* gradients           — the hand-derived adjoint of all of the above, i.e. what
                        ``loss.backward()`` (``reconstruction.py:753``) produces by autograd.
* optional stages     — detector blur ``models.py:375-382`` and object pre-blur ``models.py:267-284``
                        (torchvision ``gaussian_blur``: f32 1-D kernel exp(-x²/2σ²) on
                        linspace(-(k-1)/2, (k-1)/2, k), normalised, outer product, reflect padding)
                        and their transposes.

Parity pinning: the oracle is checked against golden vectors produced by running the
reference itself in the build container (``tests/golden/make_golden.py``,
``tests/test_oracle_golden.py``).

Conventions: F = unnormalised fft2, F^-1 = ifft2, F_o = ortho fft2, S = fftshift2.
Complex gradients follow torch's real-view convention g = dL/dRe + i dL/dIm.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass

import numpy as np

LOSS_NAMES = ("loss_single", "loss_poissn", "loss_pacbed", "loss_sparse", "loss_simlar")


def _fft2(x):
    return np.fft.fft2(x, axes=(-2, -1))


def _ifft2(x):
    return np.fft.ifft2(x, axes=(-2, -1))


def shift_grid(n: int) -> np.ndarray:
    """Effective k grid of the probe shift ramp after ifftshift: ((k + N/2) mod N) / N.

    imshift_batch multiplies fftshift2(F P) by exp(-2πi s·g) with g = arange(N)/N
    (models.py:179, image_proc.py:531), then ifftshifts, so in FFT order the grid is g[(k+N/2)%N].
    """
    return ((np.arange(n) + n // 2) % n) / n


def shift_ramp(shifts: np.ndarray, n: int, cdt=np.complex128) -> np.ndarray:
    """W_b[ky,kx] = exp(-2πi (s_y g[ky] + s_x g[kx]))   (image_proc.py:531)."""
    g = shift_grid(n)
    sy = shifts[:, 0, None, None].astype(np.float64)
    sx = shifts[:, 1, None, None].astype(np.float64)
    return np.exp(-2j * np.pi * (sy * g[None, :, None] + sx * g[None, None, :])).astype(cdt)


def gaussian_kernel1d(ks, sigma):
    """torchvision _get_gaussian_kernel1d in f32 (the kernel gaussian_blur builds)."""
    half = (ks - 1) * 0.5
    x = np.linspace(-half, half, ks, dtype=np.float32)
    pdf = np.exp(-0.5 * (x / np.float32(sigma)) ** 2).astype(np.float32)
    return (pdf / pdf.sum(dtype=np.float32)).astype(np.float32)


def gaussian_blur(x, sigma, ks=5):
    """torchvision gaussian_blur over the last two axes (reflect padding), float64."""
    k = gaussian_kernel1d(ks, sigma)
    k2 = np.outer(k, k).astype(np.float32).astype(np.float64)
    h = ks // 2
    xp = np.pad(np.asarray(x, np.float64), [(0, 0)] * (x.ndim - 2) + [(h, h), (h, h)], mode="reflect")
    Ny, Nx = x.shape[-2:]
    out = np.zeros(x.shape, np.float64)
    for i in range(ks):
        for j in range(ks):
            out += k2[i, j] * xp[..., i:i + Ny, j:j + Nx]
    return out


def gaussian_blur_adjoint(g, sigma, ks=5):
    """Transpose of gaussian_blur: spread each output over its taps, then fold the reflected pad."""
    k = gaussian_kernel1d(ks, sigma)
    k2 = np.outer(k, k).astype(np.float32).astype(np.float64)
    h = ks // 2
    Ny, Nx = g.shape[-2:]
    gp = np.zeros(g.shape[:-2] + (Ny + 2 * h, Nx + 2 * h), np.float64)
    for i in range(ks):
        for j in range(ks):
            gp[..., i:i + Ny, j:j + Nx] += k2[i, j] * g
    for r in range(h):                       # padded row r ↔ row h - r; row h+Ny+r ↔ Ny-2-r
        gp[..., 2 * h - r, :] += gp[..., r, :]
        gp[..., h + Ny - 2 - r, :] += gp[..., h + Ny + r, :]
    gp = gp[..., h:h + Ny, :]
    for c in range(h):
        gp[..., :, 2 * h - c] += gp[..., :, c]
        gp[..., :, h + Nx - 2 - c] += gp[..., :, h + Nx + c]
    return gp[..., :, h:h + Nx]


def otf_measurements(meas, idx, canvas=None, pad_idx=None, scale=None):
    """PtychoAD.get_measurements(indices) with on-the-fly padding / resampling (models.py:384-412):
    paste each frame into the canvas at pad_idx = (h1, h2, w1, w2), then
    interpolate(scale_factor, 'bilinear', align_corners=False) (aten: source index
    s·(i+0.5)-0.5 clamped at 0 with s = f32(1/scale), i1 = min(i0+1, in-1)) and divide by
    scale_y·scale_x.  float64 arithmetic on the f32 inputs."""
    frames = np.asarray(meas, np.float64)[np.asarray(idx)]
    if canvas is not None:
        h1, h2, w1, w2 = (int(v) for v in pad_idx)
        c = np.broadcast_to(np.asarray(canvas, np.float64), (len(frames),) + np.shape(canvas)).copy()
        c[:, h1:h2, w1:w2] = frames
        frames = c
    if scale is None or all(f == 1 for f in scale):
        return frames
    B, Hp, Wp = frames.shape
    sy, sx = float(scale[0]), float(scale[1])
    Ho, Wo = int(np.floor(Hp * sy)), int(np.floor(Wp * sx))

    def src(n_out, n_in, s):
        inv = np.float32(1.0 / s)
        real = (inv * (np.arange(n_out, dtype=np.float32) + np.float32(0.5)) - np.float32(0.5)).astype(np.float64)
        real = np.maximum(real, 0.0)
        i0 = np.minimum(np.floor(real).astype(np.int64), n_in - 1)
        l1 = np.clip(real - i0, 0.0, 1.0)
        i1 = i0 + (i0 < n_in - 1)
        return i0, i1, l1

    y0, y1, ly = src(Ho, Hp, sy)
    x0, x1, lx = src(Wo, Wp, sx)
    ly, lx = ly[:, None], lx[None, :]
    f = frames
    out = ((1 - ly) * ((1 - lx) * f[:, y0][:, :, x0] + lx * f[:, y0][:, :, x1]) +
           ly * ((1 - lx) * f[:, y1][:, :, x0] + lx * f[:, y1][:, :, x1]))
    return out / np.float64(np.float32(sy * sx))


def get_patches(obja, objp, crop_pos, idx, n):
    """(B,O,Nz,N,N) amplitude and phase patches at integer crop positions (models.py:251-265)."""
    B = len(idx)
    O, Nz = obja.shape[:2]
    amp = np.empty((B, O, Nz, n, n), obja.dtype)
    ph = np.empty((B, O, Nz, n, n), objp.dtype)
    for i, s in enumerate(idx):
        cy, cx = int(crop_pos[s, 0]), int(crop_pos[s, 1])
        amp[i] = obja[:, :, cy:cy + n, cx:cx + n]
        ph[i] = objp[:, :, cy:cy + n, cx:cx + n]
    return amp, ph


def get_probes(probe, shifts_b, shift_probes, cdt=np.complex128):
    """(B,P,N,N) probes: F^-1(F(P) ⊙ W_b) if shift_probes else broadcast (models.py:286-298)."""
    n = probe.shape[-1]
    P = probe.astype(cdt)
    if not shift_probes:
        return np.broadcast_to(P, (len(shifts_b),) + P.shape).copy()
    W = shift_ramp(shifts_b, n, cdt)
    return _ifft2(_fft2(P)[None] * W[:, None]).astype(cdt)


@dataclass
class ForwardCache:
    probes: np.ndarray     # (B,P,N,N)
    O: np.ndarray          # (B,Om,Nz,N,N) complex object patches
    psis: list             # psis[n] = wave entering slice n, (B,P,Om,N,N)
    Psi: np.ndarray        # (B,P,Om,N,N) far field, fftshifted
    dp: np.ndarray         # (B,N,N)
    X: list = None         # X[n] = F(ψⁿ ⊙ Oⁿ), n < Nz-1 (ψ^{n+1} = F⁻¹(H Xⁿ))


def forward(amp, ph, probes, H, occu, eps=1e-10, cdt=np.complex128) -> ForwardCache:
    """multislice_forward_model_vec_all (forward.py:20-80)."""
    Ocplx = (amp * np.exp(1j * ph.astype(np.float64))).astype(cdt)   # torch.polar  (forward.py:53)
    Nz = Ocplx.shape[2]
    psi = probes[:, :, None].astype(cdt)                               # (B,P,1,N,N)  (forward.py:57)
    psi = np.broadcast_to(psi, probes.shape[:2] + (Ocplx.shape[1],) + probes.shape[2:]).copy()
    psis, X = [], []
    Hc = H.astype(cdt)
    for n in range(Nz - 1):                                            # (forward.py:60-63)
        psis.append(psi)
        X.append(_fft2(psi * Ocplx[:, None, :, n]).astype(cdt))
        psi = _ifft2(Hc * X[-1]).astype(cdt)
    psis.append(psi)
    psi_out = psi * Ocplx[:, None, :, Nz - 1]                          # (forward.py:66-67)
    nn = psi_out.shape[-1]
    Psi = np.fft.fftshift(_fft2(psi_out) / nn, axes=(-2, -1)).astype(cdt)   # ortho + fftshift2
    dp = (np.abs(Psi) ** 2 * occu[None, None, :, None, None]).sum(axis=(1, 2)) + eps   # (forward.py:79)
    return ForwardCache(probes, Ocplx, psis, Psi, dp, X)


def loss_terms(dp, meas, ph, occu, lp):
    """CombinedLoss.forward (losses.py:143-155) → [single, poissn, pacbed, sparse, simlar] and dL/dI.

    Returns (terms, dLdI (B,N,N), dL/dφ_patch (B,O,Nz,N,N)).
    """
    B = dp.shape[0]
    K = dp.size
    terms = np.zeros(5)
    dLdI = np.zeros_like(dp, dtype=np.float64)
    I = dp.astype(np.float64)
    M = meas.astype(np.float64)
    s = lp["loss_single"]
    if s["state"]:                                                     # losses.py:36-50
        q = s.get("dp_pow", 0.5)
        Iq, Mq = I ** q, M ** q
        mu = Mq.mean()
        S = ((Iq - Mq) ** 2).sum()
        rmse = math.sqrt(S / K)
        terms[0] = s["weight"] * rmse / mu
        if rmse > 0:
            dLdI += s["weight"] / (mu * K * rmse) * (Iq - Mq) * q * I ** (q - 1)
    p = lp["loss_poissn"]
    if p["state"]:                                                     # losses.py:52-75
        q = p.get("dp_pow", 1.0)
        e = p.get("eps", 1e-6)
        Iq, Mq = I ** q, M ** q
        mu = Mq.mean()
        terms[1] = -p["weight"] * (Mq * np.log(Iq + e) - Iq).mean() / mu
        dLdI += -p["weight"] / (mu * K) * (Mq / (Iq + e) - 1.0) * q * I ** (q - 1)
    pb = lp["loss_pacbed"]
    if pb["state"]:                                                    # losses.py:77-89
        q = pb.get("dp_pow", 0.2)
        Ib, Mb = I.mean(axis=0), M.mean(axis=0)
        d = Ib ** q - Mb ** q
        mu = (M ** q).mean()
        rmse = math.sqrt((d * d).mean())
        terms[2] = pb["weight"] * rmse / mu
        if rmse > 0:
            dLdI += pb["weight"] / (mu * d.size * rmse * B) * d * q * Ib ** (q - 1)

    sp = lp["loss_sparse"]
    dph = np.zeros(ph.shape, np.float64)
    if sp["state"]:                                                    # losses.py:91-104
        nord = sp["ln_order"]
        a = np.abs(ph.astype(np.float64))
        cnt = ph.shape[0] * ph.shape[2] * ph.shape[3] * ph.shape[4]
        m = (a ** nord).sum(axis=(0, 2, 3, 4)) / cnt                  # per object mode
        terms[3] = sp["weight"] * (m ** (1.0 / nord) * occu).sum()
        for o in range(ph.shape[1]):
            coef = sp["weight"] * occu[o] * (m[o] ** (1.0 / nord - 1.0) if m[o] > 0 else 0.0) / cnt
            dph[:, o] = coef * a[:, o] ** (nord - 1) * np.sign(ph[:, o])
    return terms, dLdI, dph


def simlar_term(amp, ph, occu, lp):
    """loss_simlar (losses.py:106-141): w Σ_{amp,phase} mean(std_o(blur(x)·occ_o)) over the
    (B,O,Nz,N,N) patches; returns (term, dL/damp, dL/dph).  Area resampling (scale ≠ 1) is not
    restated (the schema default is 1)."""
    p = lp.get("loss_simlar", {"state": False})
    if not p["state"]:
        return 0.0, 0.0, 0.0
    if p.get("scale_factor") is not None and any(f != 1 for f in p["scale_factor"]):
        raise NotImplementedError("loss_simlar area resampling is not restated")
    std, O = p.get("blur_std"), amp.shape[1]
    term, grads = 0.0, []
    for x, kinds in ((amp, ("amplitude", "both")), (ph, ("phase", "both"))):
        if p.get("obj_type", "both") not in kinds:
            grads.append(0.0)
            continue
        xb = gaussian_blur(x, std) if std else np.asarray(x, np.float64)
        y = xb * occu[None, :, None, None, None]
        s = y.std(axis=1, ddof=1)
        term += p["weight"] * s.mean()
        gy = p["weight"] / s.size * (y - y.mean(axis=1, keepdims=True)) / ((O - 1) * np.where(s > 0, s, np.inf))[:, None]
        gx = gy * occu[None, :, None, None, None]
        grads.append(gaussian_blur_adjoint(gx, std) if std else gx)
    return term, grads[0], grads[1]


def adjoint(cache: ForwardCache, dLdI, dph_sparse, amp, ph, probe, shifts_b, H, occu, shift_probes,
            cdt=np.complex128):
    """Hand-derived adjoint of forward().

    Returns per-pattern gradients: dA, dφ (B,O,Nz,N,N), dprobe (P,N,N) complex, dshift (B,2).
    """
    B, P = cache.probes.shape[:2]
    Om, Nz = amp.shape[1], amp.shape[2]
    n = amp.shape[-1]
    Oc = cache.O
    Hc = H.astype(cdt)
    # g_Ψ = 2 occ Ψ ∂L/∂I, un-shift, ortho adjoint = ortho inverse
    gPsi = 2.0 * occu[None, None, :, None, None] * cache.Psi * dLdI[:, None, None]
    g = np.fft.ifft2(np.fft.ifftshift(gPsi, axes=(-2, -1)), axes=(-2, -1), norm="ortho").astype(cdt)
    gO = np.zeros((B, Om, Nz, n, n), cdt)
    dH = np.zeros((n, n), np.complex128)
    for sl in range(Nz - 1, -1, -1):
        if sl < Nz - 1:                                 # adjoint of F^-1 H F is F^-1 conj(H) F
            G = _fft2(g)
            dHb = (np.conj(cache.X[sl]) * G).sum(axis=(1, 2)) / (n * n)      # per pattern (B,N,N)
            cache.dHb = dHb if sl == Nz - 2 else cache.dHb + dHb
            dH += dHb.sum(axis=0)                                              # dL/dH (real-view convention)
            g = _ifft2(np.conj(Hc) * G).astype(cdt)
        gO[:, :, sl] = (np.conj(cache.psis[sl]) * g).sum(axis=1)   # Σ_p conj(ψ^n) g
        g = g * np.conj(Oc[:, None, :, sl])
    gPb = g.sum(axis=2)                                 # (B,P,N,N): Σ_o
    # O = A e^{iφ}: dA = Re(g_O e^{-iφ}), dφ = Im(conj(O) g_O)
    e = np.exp(-1j * ph.astype(np.float64))
    dA = np.real(gO * e)
    dP = np.imag(np.conj(Oc) * gO) + dph_sparse
    if shift_probes:
        W = shift_ramp(shifts_b, n, cdt)                              # (B,N,N)
        Fp = _fft2(probe.astype(cdt))                                  # (P,N,N)
        dprobe = _ifft2(np.conj(W)[:, None] * _fft2(gPb)).sum(axis=0)
        gg = shift_grid(n)
        dshift = np.zeros((B, 2))
        for ax, gvec in ((0, gg[:, None]), (1, gg[None, :])):
            dPb = _ifft2(Fp[None] * (W[:, None] * (-2j * np.pi) * gvec))     # ∂P_b/∂s
            dshift[:, ax] = np.real((np.conj(gPb) * dPb).sum(axis=(1, 2, 3)))
    else:
        dprobe = gPb.sum(axis=0)
        dshift = np.zeros((B, 2))
    cache.dH = dH
    return dA, dP, dprobe, dshift


def tilt_ramps(tilts_b, n, dx, dz):
    """Per-position propagator factor exp(i dz (Ky tan θy + Kx tan θx)) (models.py:330-356),
    (B,N,N), and the k grid (create_grids models.py:163-171)."""
    g = (np.arange(-n // 2, n // 2) + 0.5) / n
    k1 = np.fft.ifftshift(2 * np.pi * g / dx)
    t = np.asarray(tilts_b, np.float64) / 1e3
    ph = dz * (k1[None, :, None] * np.tan(t[:, 0, None, None]) + k1[None, None, :] * np.tan(t[:, 1, None, None]))
    return np.exp(1j * ph), k1


def forward_loss_grad(obja, objp, probe, shifts, crop_pos, H, occu, meas, batches, loss_params,
                      shift_probes=True, grad_scale=1.0, cdt=np.complex128, detector_blur_std=None,
                      obj_preblur_std=None, tilts=None, dx=None, dz=None):
    """Oracle of ptyx_forward_loss_grad: per-mini-batch losses, gradients accumulated over batches.

    batches: list of index arrays (each its own NRMSE normalisation, losses.py:45-47);
    grad_scale: the 1/grad_accumulation factor of reconstruction.py:750.
    Returns (terms (n_batches,5), dp list, grads dict).
    """
    if isinstance(loss_params, str):
        loss_params = json.loads(loss_params)
    n = probe.shape[-1]
    g_obja = np.zeros(obja.shape, np.float64)
    g_objp = np.zeros(objp.shape, np.float64)
    g_probe = np.zeros(probe.shape, np.complex128)
    g_shifts = np.zeros(shifts.shape, np.float64)
    g_H = np.zeros(probe.shape[-2:], np.complex128)
    g_tilts = None if tilts is None else np.zeros(np.shape(tilts), np.float64)
    g_dz_ramp, g_H_base = 0.0, np.zeros(probe.shape[-2:], np.complex128)
    all_terms, dps = [], []
    for idx in batches:
        idx = np.asarray(idx)
        amp, ph = get_patches(obja, objp, crop_pos, idx, n)
        if obj_preblur_std:                                        # models.py:275-284
            amp, ph = gaussian_blur(amp, obj_preblur_std), gaussian_blur(ph, obj_preblur_std)
        probes = get_probes(probe, shifts[idx], shift_probes, cdt)
        Hx = H
        if tilts is not None:                                      # per-position tilts (tilt_type 'each')
            ramp, k1 = tilt_ramps(np.asarray(tilts)[idx], n, dx, dz)
            Hx = (np.asarray(H, np.complex128)[None] * ramp)[:, None, None]
        cache = forward(amp, ph, probes, Hx, occu, cdt=cdt)
        dp = gaussian_blur(cache.dp, detector_blur_std) if detector_blur_std else cache.dp   # :379-380
        terms, dLdI, dph = loss_terms(dp, meas[idx], ph, occu, loss_params)
        if detector_blur_std:
            dLdI = gaussian_blur_adjoint(dLdI, detector_blur_std)
        st, sdA, sdP = simlar_term(amp, ph, occu, loss_params)
        terms[4] = st
        dA, dP, dprobe, dshift = adjoint(cache, dLdI, dph, amp, ph, probe, shifts[idx], Hx, occu,
                                         shift_probes, cdt)
        dA, dP = dA + sdA, dP + sdP
        if tilts is not None and amp.shape[2] > 1:                # dL/dθ_b = Re Σ conj(g_Hb) ∂H_b/∂θ_b
            Hb = Hx[:, 0, 0]
            t = np.asarray(tilts, np.float64)[idx] / 1e3
            w = np.real(np.conj(cache.dHb) * 1j * Hb)
            g_tilts[idx, 0] += grad_scale * dz * (w * k1[None, :, None]).sum(axis=(1, 2)) / np.cos(t[:, 0]) ** 2 / 1e3
            g_tilts[idx, 1] += grad_scale * dz * (w * k1[None, None, :]).sum(axis=(1, 2)) / np.cos(t[:, 1]) ** 2 / 1e3
            T = k1[None, :, None] * np.tan(t[:, 0, None, None]) + k1[None, None, :] * np.tan(t[:, 1, None, None])
            g_dz_ramp += grad_scale * float((w * T).sum())                       # ∂/∂dz of the ramps
            g_H_base += grad_scale * (np.conj(ramp) * cache.dHb).sum(axis=0)     # Σ_b conj(r_b) g_Hb
        if obj_preblur_std:
            dA, dP = gaussian_blur_adjoint(dA, obj_preblur_std), gaussian_blur_adjoint(dP, obj_preblur_std)
        for i, s in enumerate(idx):
            cy, cx = int(crop_pos[s, 0]), int(crop_pos[s, 1])
            g_obja[:, :, cy:cy + n, cx:cx + n] += grad_scale * dA[i]
            g_objp[:, :, cy:cy + n, cx:cx + n] += grad_scale * dP[i]
            g_shifts[s] += grad_scale * dshift[i]
        g_probe += grad_scale * dprobe
        g_H += grad_scale * cache.dH
        all_terms.append(terms)
        dps.append(dp)
    grads = dict(obja=g_obja, objp=g_objp, probe=g_probe, shifts=g_shifts, H=g_H, tilts=g_tilts,
                 dz_ramp=g_dz_ramp, H_base=g_H_base)
    return np.array(all_terms), dps, grads


N_BATCH_SUMS = 37   # include/ptyx.h PTYX_BATCH_SUMS


def batch_sums(dp, meas, ph, lp):
    """The additive sums behind the loss terms of one (part of a) mini-batch, in the engine's
    PTYX_BATCH_SUMS layout: [count, Σ(I^q-M^q)², ΣM^q (loss_single), Σ(M^q log(I^q+ε)-I^q), ΣM^q
    (loss_poissn), Σ|φ|^n per object mode (8 slots)] — losses.py:45-47, 70-72, 101 before the means."""
    out = np.zeros(N_BATCH_SUMS)
    out[0] = dp.shape[0]
    I, M = dp.astype(np.float64), meas.astype(np.float64)
    s, p, sp = lp["loss_single"], lp["loss_poissn"], lp["loss_sparse"]
    if s["state"]:
        q = s.get("dp_pow", 0.5)
        out[1], out[2] = ((I ** q - M ** q) ** 2).sum(), (M ** q).sum()
    if p["state"]:
        q, e = p.get("dp_pow", 1.0), p.get("eps", 1e-6)
        Mq, Iq = M ** q, I ** q
        out[3], out[4] = (Mq * np.log(Iq + e) - Iq).sum(), Mq.sum()
    if sp["state"]:
        a = np.abs(ph.astype(np.float64)) ** sp["ln_order"]
        out[5:5 + ph.shape[1]] = a.sum(axis=(0, 2, 3, 4))
    return out


def terms_from_sums(sums, n, Nz, occu, lp):
    """Loss terms and adjoint coefficients of a WHOLE mini-batch from its summed batch_sums
    (losses.py:36-104): terms (5,), (c_single, c_poissn), c_sparse per object mode."""
    B = sums[0]
    K = B * n * n
    terms = np.zeros(5)
    c1 = c2 = 0.0
    s, p, sp = lp["loss_single"], lp["loss_poissn"], lp["loss_sparse"]
    if s["state"] and B > 0:
        mu, rmse = sums[2] / K, math.sqrt(sums[1] / K)
        terms[0] = s["weight"] * rmse / mu
        c1 = s["weight"] / (mu * K * rmse) if rmse > 0 else 0.0
    if p["state"] and B > 0:
        mu = sums[4] / K
        terms[1] = -p["weight"] * (sums[3] / K) / mu
        c2 = -p["weight"] / (mu * K)
    csp = np.zeros(len(occu))
    if sp["state"] and B > 0:
        nord, cnt = sp["ln_order"], B * Nz * n * n
        m = sums[5:5 + len(occu)] / cnt
        terms[3] = sp["weight"] * float((m ** (1.0 / nord) * occu).sum())
        for o in range(len(occu)):
            csp[o] = sp["weight"] * occu[o] * (m[o] ** (1.0 / nord - 1.0) if m[o] > 0 else 0.0) / cnt
    return terms, (c1, c2), csp


def forward_loss_grad_parts(obja, objp, probe, shifts, crop_pos, H, occu, meas, parts, loss_params, reduce,
                            shift_probes=True, grad_scale=1.0, cdt=np.complex128):
    """Oracle of ptyx_forward_loss_grad_begin → all-reduce → _end for ONE rank: ``parts[m]`` is this
    rank's share (possibly empty) of mini-batch m, ``reduce(sums)`` sums the (n_batches, N_BATCH_SUMS) batch
    sums over the ranks in place.  Returns (terms of the whole mini-batches, grads of this rank's
    patterns); summed over the ranks the gradients equal forward_loss_grad over the whole batches."""
    if isinstance(loss_params, str):
        loss_params = json.loads(loss_params)
    n = probe.shape[-1]
    Nz = obja.shape[1]
    sums = np.zeros((len(parts), N_BATCH_SUMS))
    fw = []
    for m, idx in enumerate(parts):
        idx = np.asarray(idx, dtype=np.int64)
        if idx.size == 0:
            fw.append(None)
            continue
        amp, ph = get_patches(obja, objp, crop_pos, idx, n)
        cache = forward(amp, ph, get_probes(probe, shifts[idx], shift_probes, cdt), H, occu, cdt=cdt)
        sums[m] = batch_sums(cache.dp, meas[idx], ph, loss_params)
        fw.append((idx, amp, ph, cache))
    reduce(sums)
    g = dict(obja=np.zeros(obja.shape), objp=np.zeros(objp.shape), probe=np.zeros(probe.shape, np.complex128),
             shifts=np.zeros(shifts.shape))
    all_terms = []
    for m, f in enumerate(fw):
        terms, (c1, c2), csp = terms_from_sums(sums[m], n, Nz, occu, loss_params)
        all_terms.append(terms)
        if f is None:
            continue
        idx, amp, ph, cache = f
        I, M = cache.dp.astype(np.float64), meas[idx].astype(np.float64)
        dLdI = np.zeros_like(I)
        s, p, sp = loss_params["loss_single"], loss_params["loss_poissn"], loss_params["loss_sparse"]
        if s["state"]:
            q = s.get("dp_pow", 0.5)
            dLdI += c1 * (I ** q - M ** q) * q * I ** (q - 1)
        if p["state"]:
            q, e = p.get("dp_pow", 1.0), p.get("eps", 1e-6)
            dLdI += c2 * (M ** q / (I ** q + e) - 1.0) * q * I ** (q - 1)
        dph = np.zeros(ph.shape)
        if sp["state"]:
            a = np.abs(ph.astype(np.float64))
            for o in range(ph.shape[1]):
                dph[:, o] = csp[o] * a[:, o] ** (sp["ln_order"] - 1) * np.sign(ph[:, o])
        dA, dP, dprobe, dshift = adjoint(cache, dLdI, dph, amp, ph, probe, shifts[idx], H, occu, shift_probes, cdt)
        for i, sidx in enumerate(idx):
            cy, cx = int(crop_pos[sidx, 0]), int(crop_pos[sidx, 1])
            g["obja"][:, :, cy:cy + n, cx:cx + n] += grad_scale * dA[i]
            g["objp"][:, :, cy:cy + n, cx:cx + n] += grad_scale * dP[i]
            g["shifts"][sidx] += grad_scale * dshift[i]
        g["probe"] += grad_scale * dprobe
    return np.array(all_terms), g


def propagator_param_grads(gH, H, dz, tilts, dx, lambd, case):
    """Chain rule from dL/dH to the optimised slice thickness / global tilts (get_propagators
    cases 1, 2A, 3, models.py:339-356): dL/dθ = Re Σ conj(gH) ∂H/∂θ, with ∂H/∂θ = i (∂φ/∂θ) H for
    the H the forward actually used (its phase dz·Kz ≈ 300 rad is rounded in f32, and the
    constant part dz·k of that phase cancels only against the same H).  Returns (d_dz, d_tilts)."""
    n = gH.shape[-1]
    g = (np.arange(-n // 2, n // 2) + 0.5) / n
    k1 = np.fft.ifftshift(2 * np.pi * g / dx)
    Ky, Kx = np.meshgrid(k1, k1, indexing="ij")
    k = 2 * np.pi / lambd
    Kz = np.sqrt(k ** 2 - Kx ** 2 - Ky ** 2)
    ty, tx = tilts[0] / 1e3, tilts[1] / 1e3
    T = Ky * np.tan(ty) + Kx * np.tan(tx)
    H = np.asarray(H, np.complex128)
    if case == 1:
        dHdz = 1j * (Kz + T) * H
    elif case == 2:
        dHdz = 1j * T * H
    else:
        dHdz = 1j * Kz * H
    dHty = 1j * dz * Ky / np.cos(ty) ** 2 / 1e3 * H
    dHtx = 1j * dz * Kx / np.cos(tx) ** 2 / 1e3 * H
    re = lambda a: float(np.real(np.sum(np.conj(gH) * a)))   # noqa: E731
    return re(dHdz), np.array([re(dHty), re(dHtx)])


def forward_dp(obja, objp, probe, shifts, crop_pos, H, occu, idx, shift_probes=True, cdt=np.complex128,
               detector_blur_std=None, obj_preblur_std=None):
    """Oracle of ptyx_forward (PtychoAD.forward, models.py:422-436): (B,N,N) dp."""
    n = probe.shape[-1]
    amp, ph = get_patches(obja, objp, crop_pos, np.asarray(idx), n)
    if obj_preblur_std:
        amp, ph = gaussian_blur(amp, obj_preblur_std), gaussian_blur(ph, obj_preblur_std)
    probes = get_probes(probe, shifts[np.asarray(idx)], shift_probes, cdt)
    dp = forward(amp, ph, probes, H, occu, cdt=cdt).dp
    return gaussian_blur(dp, detector_blur_std) if detector_blur_std else dp


def adam_step(params, grads, state, lrs, t, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam default update (used at reconstruction.py:759), in the params' dtype.

    Complex parameters are handled through their real view, as PtyRAD's probe is a
    view_as_real parameter (models.py:103).
    """
    b1, b2 = betas
    for k in params:
        if grads.get(k) is None or lrs.get(k, 0) == 0:
            continue
        g = grads[k].astype(params[k].dtype)
        m, v = state.get(k, (np.zeros_like(g), np.zeros_like(g)))
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        state[k] = (m, v)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        params[k] = params[k] - (lrs[k] / bc1) * m / (np.sqrt(v) / math.sqrt(bc2) + eps)
    return params
