"""Synthetic, seeded 4D-STEM inputs for the ptyx hot path.

This is one-time input preparation (NumPy, host side), the analogue of what
PtyRAD's ``Initializer.init_all`` (``src/ptyrad/initialization.py:590-605``)
produces as ``init_variables``.  It is *not* part of the HIP hot path.  The
physics follows the textbook formulas that PtyRAD also uses:

* electron wavelength, aperture-limited probe with defocus
  (cf. ``utils/physics.py:219-305`` make_stem_probe),
* incoherent probe modes (cf. ``utils/physics.py:382-472`` make_mixed_probe),
* Fresnel angular-spectrum propagator with the half-bin k grid
  (cf. ``utils/physics.py:475-489`` near_field_evolution),
* raster scan with jitter, integer crop positions + sub-px remainders
  (cf. ``initialization.py:352-359``).

All arrays are returned in the layouts the C-ABI takes (see include/ptyx.h).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

STEP_ANG = 0.429       # tBL_WSe2 scan step (demo/params/tBL_WSe2_reconstruct.yml)
DX_ANG = 0.1494        # fixed calibration used by SURVEY §8c
KV = 80.0
CONV_MRAD = 24.9


def electron_wavelength(kv: float) -> float:
    """Relativistic electron wavelength in Angstrom for an accelerating voltage in kV."""
    v = kv * 1e3
    # h / sqrt(2 m e V (1 + eV / 2mc^2)), with constants folded (Angstrom, volts)
    return 12.2643 / math.sqrt(v * (1.0 + 0.97845e-6 * v))


def stem_probe(n: int, dx: float = DX_ANG, kv: float = KV, conv_mrad: float = CONV_MRAD,
               defocus: float = 0.0) -> np.ndarray:
    """Aperture-limited STEM probe (complex64, (n, n)), unit total intensity, centred."""
    lam = electron_wavelength(kv)
    fk = np.fft.fftfreq(n, d=dx)                      # 1/Angstrom, FFT order
    ky, kx = np.meshgrid(fk, fk, indexing="ij")
    k2 = kx * kx + ky * ky
    aperture = np.sqrt(k2) <= (conv_mrad * 1e-3 / lam)
    chi = -math.pi * lam * defocus * k2                # defocus aberration phase
    pupil = aperture * np.exp(-1j * chi)
    probe = np.fft.fftshift(np.fft.ifft2(pupil))
    probe /= np.sqrt(np.sum(np.abs(probe) ** 2))
    return probe.astype(np.complex64)


def mixed_probe(base: np.ndarray, n_modes: int, weights=(0.02,)) -> np.ndarray:
    """Orthogonal incoherent modes built from the base probe times low-order polynomials."""
    n = base.shape[-1]
    if n_modes == 1:
        return base[None].astype(np.complex64)
    y, x = np.meshgrid(np.arange(n) - n / 2, np.arange(n) - n / 2, indexing="ij")
    y = y / (n / 4)
    x = x / (n / 4)
    polys = [np.ones_like(x), x, y, x * y, x * x - 1, y * y - 1, x * x * y, x * y * y,
             x ** 3, y ** 3, x * x * y * y]
    modes = []
    for m in range(n_modes):
        v = base * polys[m % len(polys)].astype(np.complex128)
        for u in modes:
            v = v - np.vdot(u, v) * u
        v = v / np.sqrt(np.vdot(v, v).real)
        modes.append(v)
    modes = np.stack(modes)
    w = np.empty(n_modes)
    w[0] = 1.0
    rest = list(weights) + [weights[-1]] * n_modes
    for m in range(1, n_modes):
        w[m] = rest[m - 1]
    w = w / w.sum()
    modes = modes * np.sqrt(w)[:, None, None]
    return modes.astype(np.complex64)


def fresnel_propagator(n: int, dx: float, dz: float, kv: float = KV) -> np.ndarray:
    """Angular-spectrum propagator on the half-bin grid, zero frequency at the corner (complex64)."""
    lam = electron_wavelength(kv)
    g = (np.arange(-(n // 2), n - n // 2) + 0.5) / n
    kvec = 2.0 * math.pi * g / dx
    ky, kx = np.meshgrid(kvec, kvec, indexing="ij")
    k0 = 2.0 * math.pi / lam
    h = np.exp(1j * dz * np.sqrt(k0 * k0 - kx * kx - ky * ky))
    return np.fft.ifftshift(h).astype(np.complex64)


def object_side(scan: int, n: int, step_px: float) -> int:
    return int(1.2 * math.ceil((scan - 1) * step_px + n))


@dataclass
class Scan:
    crop_pos: np.ndarray       # (n_scans, 2) int32, top-left corner (y, x)
    shifts: np.ndarray         # (n_scans, 2) float32 sub-px remainders (y, x)
    obj_shape: tuple           # (Ny, Nx)
    n_slow: int
    n_fast: int


def raster_scan(n_slow: int, n_fast: int, n: int, step_px: float = STEP_ANG / DX_ANG,
                jitter: float = 0.15, seed: int = 0, obj_shape=None) -> Scan:
    """Raster positions centred in the object canvas, + Gaussian jitter (px)."""
    rng = np.random.default_rng(seed)
    if obj_shape is None:
        obj_shape = (object_side(n_slow, n, step_px), object_side(n_fast, n, step_px))
    ny, nx = obj_shape
    iy, ix = np.meshgrid(np.arange(n_slow), np.arange(n_fast), indexing="ij")
    py = iy.reshape(-1) * step_px
    px = ix.reshape(-1) * step_px
    py = py + (ny - ((n_slow - 1) * step_px + n)) / 2.0
    px = px + (nx - ((n_fast - 1) * step_px + n)) / 2.0
    pos = np.stack([py, px], -1) + rng.normal(0.0, jitter, size=(py.size, 2))
    crop = np.round(pos)
    crop[:, 0] = np.clip(crop[:, 0], 0, ny - n)
    crop[:, 1] = np.clip(crop[:, 1], 0, nx - n)
    shifts = (pos - crop).astype(np.float32)
    return Scan(crop.astype(np.int32), shifts, (ny, nx), n_slow, n_fast)


def atom_phase_object(obj_shape, n_slices: int = 1, n_omodes: int = 1, spacing_px: float = 3.3 / DX_ANG,
                      sigma: float = 1.5, peak: float = 0.3, seed: int = 1):
    """Ground-truth object: unit amplitude, Gaussian 'atoms' on a hexagonal lattice in phase."""
    rng = np.random.default_rng(seed)
    ny, nx = obj_shape
    phase = np.zeros((n_omodes, n_slices, ny, nx), np.float32)
    yy = np.arange(ny)[:, None]
    xx = np.arange(nx)[None, :]
    for s in range(n_slices):
        off = rng.uniform(0, spacing_px, size=2)
        a1 = np.array([0.0, spacing_px])
        a2 = np.array([spacing_px * math.sqrt(3) / 2, spacing_px / 2])
        basis = np.stack([a1, a2])
        inv = np.linalg.inv(basis.T)
        # fractional lattice coordinates of every pixel, distance to nearest lattice point
        fy = yy - off[0]
        fx = xx - off[1]
        c = np.einsum("ij,jyx->iyx", inv, np.stack(np.broadcast_arrays(fy, fx)))
        c = c - np.round(c)
        d = np.einsum("ij,jyx->iyx", basis.T, c)
        r2 = d[0] ** 2 + d[1] ** 2
        phase[:, s] = (peak / n_slices) * np.exp(-r2 / (2 * sigma * sigma))
    amp = np.ones_like(phase)
    return amp, phase


def recon_init_object(obj_shape, n_slices: int, n_omodes: int, seed: int = 2):
    """exp(1j * 1e-8 * U) start (cf. initialization.py:1629), as (amplitude, phase) f32."""
    rng = np.random.default_rng(seed)
    z = np.exp(1j * 1e-8 * rng.random((n_omodes, n_slices) + tuple(obj_shape)))
    return np.abs(z).astype(np.float32), np.angle(z).astype(np.float32)


def omode_occupancy(n_omodes: int) -> np.ndarray:
    if n_omodes == 1:
        return np.ones(1, np.float32)
    w = np.linspace(1.0, 0.5, n_omodes)
    return (w / w.sum()).astype(np.float32)


@dataclass
class Problem:
    """All hot-path inputs for one synthetic configuration."""
    obja: np.ndarray
    objp: np.ndarray
    probe: np.ndarray          # (P, N, N) complex64
    H: np.ndarray              # (N, N) complex64
    occu: np.ndarray           # (O,) f32
    crop_pos: np.ndarray
    shifts: np.ndarray
    meas: np.ndarray           # (n_scans, N, N) f32 (or f16)
    n_slow: int
    n_fast: int
    dz: float = 2.0
    extra: dict = field(default_factory=dict)


def random_problem(n: int, n_slow: int, n_fast: int, P: int = 1, O: int = 1, Nz: int = 1,
                   seed: int = 0, meas_dtype=np.float32, meas: str = "uniform") -> Problem:
    """Throughput/parity problem: realistic probe + geometry, random object and DPs.

    meas='uniform' draws U[0,1) DPs (acceptable for throughput runs).
    """
    rng = np.random.default_rng(seed)
    scan = raster_scan(n_slow, n_fast, n, seed=seed)
    probe = mixed_probe(stem_probe(n), P)
    H = fresnel_propagator(n, DX_ANG, 2.0)
    obja = (1.0 + 0.05 * rng.standard_normal((O, Nz) + scan.obj_shape)).astype(np.float32)
    objp = (0.1 * rng.standard_normal((O, Nz) + scan.obj_shape)).astype(np.float32)
    n_scans = n_slow * n_fast
    if meas == "uniform":
        m = rng.random((n_scans, n, n), dtype=np.float32).astype(meas_dtype)
    elif meas == "zeros":
        m = np.zeros((n_scans, n, n), meas_dtype)
    else:                      # "none": caller provides measurements (e.g. generated on the GPU)
        m = None
    return Problem(obja, objp, probe, H, omode_occupancy(O), scan.crop_pos, scan.shifts,
                   m, n_slow, n_fast)


# BASELINE.json configs[1..4] as bench.py runs them (SURVEY §8d geometry): probe side N, modes,
# slices, DP storage, the full raster side and how it is divided over the ranks
BENCH_CONFIGS = {
    "c2": dict(N=128, P=1, O=1, Nz=1, f16=False, scan=256, mode="weak"),
    "c2-strong": dict(N=128, P=1, O=1, Nz=1, f16=False, scan=256, mode="strong"),
    "c3": dict(N=256, P=8, O=2, Nz=1, f16=False, scan=512, mode="block"),
    "c4": dict(N=128, P=1, O=1, Nz=16, f16=False, scan=1024, mode="strong"),
    "c5": dict(N=256, P=4, O=1, Nz=1, f16=True, scan=4096, mode="block"),
}


def bench_geometry(config: str, world: int = 1, rank: int = 0, patterns: int = 16384, scan: int | None = None):
    """The positions one rank of a bench.py job processes.

    c2: a scan x scan raster per rank (weak scaling: the global raster is (scan·world) x scan);
    c2-strong / c4: the config's raster split by rows over the ranks (strong scaling);
    c3 / c5: a block of `patterns` positions of the config's raster, starting at the rank's first
    row of the full raster (the full c5 shard is 275 GB of DPs per GPU).
    Returns (crop_pos, shifts, (Ny, Nx), description, total positions of the job's global scan or None).
    """
    cfg = BENCH_CONFIGS[config]
    N = cfg["N"]
    step_px = STEP_ANG / DX_ANG
    if config == "c2":
        S = scan or cfg["scan"]
        sc = raster_scan(S * world, S, N, seed=0)
        sl = slice(rank * S * S, (rank + 1) * S * S)
        return (sc.crop_pos[sl], sc.shifts[sl], sc.obj_shape,
                f"c2: synthetic 4D-STEM, {S}x{S} scan per GPU (weak scaling), 128x128 DP, P=O=Nz=1", None)
    if cfg["mode"] == "strong":
        S = cfg["scan"] if config == "c4" else (scan or cfg["scan"])
        sc = raster_scan(S, S, N, seed=0)
        r0, r1 = S * rank // world, S * (rank + 1) // world
        sl = slice(r0 * S, r1 * S)
        return (sc.crop_pos[sl], sc.shifts[sl], sc.obj_shape,
                f"{config}: {S}x{S} scan split over {world} GPU(s) (rows {r0}-{r1} here), {N}x{N} DP, "
                f"P={cfg['P']}, O={cfg['O']}, Nz={cfg['Nz']}", sc.crop_pos.shape[0])
    S = cfg["scan"]
    side = object_side(S, N, step_px)
    n_fast = min(S, patterns)
    n_slow = max(1, patterns // n_fast)
    rows_per_rank = S // max(1, world)
    blk = raster_scan(n_slow, n_fast, N, obj_shape=(side, side), seed=rank)
    full_y0 = (side - ((S - 1) * step_px + N)) / 2.0
    blk_y0 = (side - ((n_slow - 1) * step_px + N)) / 2.0
    dy = int(round(full_y0 + rank * rows_per_rank * step_px - blk_y0))
    crop_pos = blk.crop_pos.copy()
    crop_pos[:, 0] = np.clip(crop_pos[:, 0] + dy, 0, side - N)
    return (crop_pos, blk.shifts, (side, side),
            f"{config}: {n_slow}x{n_fast} block of the {S}x{S} scan per GPU (rank shard rows from "
            f"{rank * rows_per_rank}), object {side}x{side}, {N}x{N} DP, P={cfg['P']}, O={cfg['O']}, "
            f"Nz={cfg['Nz']}{', fp16 DP storage' if cfg['f16'] else ''}", None)
