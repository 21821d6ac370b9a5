"""Measurement ingest into HBM — drop-in for load_raw (src/ptyrad/load.py:19-49) and
Initializer._process_meas (src/ptyrad/initialization.py:709-752) on EMPAD-style raw stacks.

    meas, info = ingest_raw(path, init_params, device, file_shape=(N, H, W), offset=0, gap=1024)

reads the file straight into device memory (libptyx ptyx_raw_read: pinned double buffers,
strided DMA that drops the per-frame gaps), applies meas_flipT, meas_crop,
meas_remove_neg_values and meas_normalization on the device (ptyx_meas_stats /
ptyx_meas_finish) and returns the (N', Npix_y, Npix_x) stack the model consumes, f32 or f16
(fp16 storage for the large-field configs).  Sharded use: each rank passes rank/world and gets
its contiguous block of scan rows; the normalisation statistics are all-reduced (one MIN and
one SUM) so every rank divides by the global constant, exactly like a single-rank run.

A single rank holding the whole stack takes the normalisation constant from the reference's own
f32 mean pattern (ptyx_meas_mean_seq: numpy's sequential f32 meas.mean(0), bit for bit), so the
stored stack is the reference's meas / const exactly; sharded ingest uses the f64 statistics
(summable over ranks, ≈ 1e-6).

meas_pad (initialization.py:956-1048: constant / edge / linear_ramp / exp / power backgrounds,
'precompute' or 'on_the_fly') and meas_resample (:1050-1102: 'precompute' bilinear zoom, or
'on_the_fly' scale factors) follow the normalisation: the mean pattern is again the reference's
f32 one (single rank) or comes from the statistics (ptyx_meas_mean, global across ranks), the
2-parameter background fit of
image_proc.py:458-492 runs on the host (scipy.optimize.curve_fit, the reference's own solver,
on Ho·Wo values), the background is built on the device (ptyx_meas_pad_background) and a
precomputed pad and / or resample is ONE fused paste + zoom pass (ptyx_meas_pad_resample).
On-the-fly options return the model's init_variables (on_the_fly_meas_padded, _idx,
on_the_fly_meas_scale_factors), which PtychoHIP consumes through ptyx_meas_gather.

Not supported here (NotImplementedError, run the reference's host path for them): meas_permute,
meas_reshape and the simulation options meas_add_source_size / meas_add_detector_blur /
meas_add_poisson_noise (each when enabled; None, and 0 for the two blurs, are off as in the
reference).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib

_NEG = {"clip_neg": 0, "subtract_min": 1, "clip_value": 2, "subtract_value": 3}
_NORM = {"max_at_one": 0, "mean_at_one": 1, "sum_to_one": 2, "divide_const": 3}
_UNSUPPORTED = ("meas_permute", "meas_reshape", "meas_add_source_size", "meas_add_detector_blur",
                "meas_add_poisson_noise")
_PAD_TYPES = {"constant": 0, "edge": 1, "linear_ramp": 2, "exp": 3, "power": 4}
_MODES = ("on_the_fly", "precompute")


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def proc_from_params(init_params: dict, H: int, W: int) -> _lib.MeasProc:
    """The ptyx_meas_proc of init_params (flipT, ky/kx crop, negative values, normalisation)."""
    for k in _UNSUPPORTED:
        v = init_params.get(k)
        if v is not None and not (k in ("meas_add_source_size", "meas_add_detector_blur") and v == 0):
            raise NotImplementedError(f"{k} is not supported by the device ingest path")
    p = _lib.MeasProc()
    f = init_params.get("meas_flipT")
    if f is not None:
        if not isinstance(f, (list, tuple)) or len(f) != 3:
            raise ValueError(f"Expected flipT_axes to be a list of 3 values, got: {f}")
        p.flipud, p.fliplr, p.transpose = (int(v) for v in f)
    Ht, Wt = (W, H) if p.transpose else (H, W)
    c = init_params.get("meas_crop")
    p.crop_ky0 = p.crop_ky1 = p.crop_kx0 = p.crop_kx1 = -1
    if c is not None:
        if len(c) != 4:
            raise ValueError(f"Expected 4 crop ranges [N_slow, N_fast, ky, kx], got {c}")
        if c[2] is not None:
            p.crop_ky0, p.crop_ky1 = _bounds(c[2], Ht)
        if c[3] is not None:
            p.crop_kx0, p.crop_kx1 = _bounds(c[3], Wt)
    neg = init_params.get("meas_remove_neg_values") or {}
    mode = neg.get("mode", "clip_neg")
    if mode not in _NEG:
        raise ValueError(f"Unsupported mode '{mode}' for handling negative values.")
    if mode in ("clip_value", "subtract_value") and neg.get("value") is None:
        raise KeyError(f"Mode '{mode}' requires a non-None 'value'.")
    p.neg_mode, p.neg_force = _NEG[mode], int(bool(neg.get("force", False)))
    p.neg_value = float(neg.get("value") or 0.0)
    norm = init_params.get("meas_normalization") or {}
    nm = norm.get("mode", "max_at_one")
    if nm not in _NORM:
        raise ValueError(f"Unsupported normalization mode '{nm}'.")
    if nm == "divide_const" and norm.get("value") is None:
        raise KeyError("Mode 'divide_const' requires a non-None 'norm_const'.")
    p.norm_mode, p.norm_value = _NORM[nm], float(norm.get("value") or 0.0)
    return p


def _bounds(b, n):
    s = slice(b[0], b[1]).indices(n)
    return s[0], s[1]


def _out_shape(p, H, W):
    Ht, Wt = (W, H) if p.transpose else (H, W)
    ky = (0, Ht) if p.crop_ky1 < 0 else (p.crop_ky0, p.crop_ky1)
    kx = (0, Wt) if p.crop_kx1 < 0 else (p.crop_kx0, p.crop_kx1)
    return ky[1] - ky[0], kx[1] - kx[0]


def load_raw(file_path, shape, offset=0, gap=1024, device="cuda", first=0, count=None):
    """load.py:19-49 into device memory: frames [first, first+count) of (N, H, W) f32."""
    lib = _lib.load()
    N, H, W = (int(v) for v in shape)
    count = N - first if count is None else int(count)
    dev = torch.device(device)
    out = torch.empty((count, H, W), dtype=torch.float32, device=dev)
    _lib.check(lib.ptyx_raw_read(_stream(dev), str(file_path).encode(), int(offset), H, W, int(gap), N, int(first),
                                 count, _p(out)))
    return out


def meas_stats(raw: torch.Tensor, p, chunk_frames=None) -> torch.Tensor:
    """ptyx_meas_stats over a device (n, H, W) f32 stack, optionally in frame chunks."""
    lib = _lib.load()
    n, H, W = raw.shape
    Ho, Wo = _out_shape(p, H, W)
    dev = raw.device
    stats = torch.zeros(int(lib.ptyx_meas_stats_len(Ho, Wo)), dtype=torch.float64, device=dev)
    stats[0] = math.inf
    ws = _ws(lib, Ho, Wo, dev)
    step = max(int(chunk_frames or n), 1)
    for f0 in range(0, n, step):
        part = raw[f0:f0 + step]
        _lib.check(lib.ptyx_meas_stats(_stream(dev), _p(part), part.shape[0], H, W, ctypes.byref(p), _p(stats),
                                       _p(ws)))
    return stats


def allreduce_stats(stats: torch.Tensor):
    """Rank reduction of ptyx_meas_stats: MIN of the minimum, SUM of the count and pixel sums."""
    import torch.distributed as tdist
    mn = stats[:1].clone()
    tdist.all_reduce(mn, op=tdist.ReduceOp.MIN)
    rest = stats[1:].clone()
    tdist.all_reduce(rest)
    stats[0] = mn[0]
    stats[1:] = rest
    return stats


def meas_finish(raw: torch.Tensor, p, stats: torch.Tensor, out_f16=False) -> torch.Tensor:
    """ptyx_meas_finish: the processed (n, Ho, Wo) stack given complete statistics."""
    lib = _lib.load()
    n, H, W = raw.shape
    Ho, Wo = _out_shape(p, H, W)
    dev = raw.device
    out = torch.empty((n, Ho, Wo), dtype=torch.float16 if out_f16 else torch.float32, device=dev)
    _lib.check(lib.ptyx_meas_finish(_stream(dev), _p(raw), n, H, W, ctypes.byref(p), _p(stats),
                                    _p(_ws(lib, Ho, Wo, dev)), _p(out), int(bool(out_f16))))
    return out


def _ws(lib, Ho, Wo, dev):
    return torch.empty((int(lib.ptyx_meas_ws_bytes(Ho, Wo)) + 7) // 8, dtype=torch.float64, device=dev)


def pad_config(init_params: dict):
    """meas_pad (initialization.py:973-982, 1041-1042): None, or a dict whose 'mode' is None, is off."""
    cfg = init_params.get("meas_pad")
    if cfg is None or cfg.get("mode") is None:
        return None
    mode, ptype = cfg["mode"], cfg["padding_type"]
    if ptype not in _PAD_TYPES:
        raise ValueError(f"Unsupported padding_type = '{ptype}'")
    if mode not in _MODES:
        raise ValueError(f"meas_pad does not support mode = '{mode}', please choose from 'on_the_fly', 'precompute', or null")
    return {"mode": mode, "type": ptype, "target": int(cfg["target_Npix"]), "value": cfg.get("value", 10),
            "threshold": cfg.get("threshold", 70)}


def resample_config(init_params: dict, otf_pad: bool):
    """meas_resample (initialization.py:1055-1095): off for None / mode None; unequal scale factors
    become their minimum; an on-the-fly pad forces an on-the-fly resample."""
    cfg = init_params.get("meas_resample")
    if cfg is None or cfg.get("mode") is None:
        return None
    if "scale_factors" not in cfg:
        raise KeyError("Missing required configuration field: 'scale_factors'")
    sf = cfg["scale_factors"]
    if len(sf) != 2:
        raise ValueError("scale_factors for resample must be a list or tuple of two elements.")
    s = min(sf) if sf[0] != sf[1] else sf[0]
    mode = "on_the_fly" if otf_pad else cfg["mode"]
    if mode not in _MODES:
        raise ValueError(f"meas_resample does not support mode = '{mode}', please choose from 'on_the_fly', 'precompute', or null")
    return {"mode": mode, "scale": s}


def pad_geometry(Ho, Wo, pad):
    """Canvas (Hp, Wp) and frame origin (h1, w1) of meas_pad (initialization.py:990-998): the
    frame centred with the odd pixel after it; exp / power evaluate on target_Npix²."""
    T = pad["target"]
    py, px = max(0, T - Ho), max(0, T - Wo)
    if pad["type"] in ("exp", "power"):
        if Ho > T or Wo > T:
            raise ValueError(f"meas_pad: target_Npix {T} is smaller than the measurement ({Ho}, {Wo})")
        Hp = Wp = T
    else:
        Hp, Wp = Ho + py, Wo + px
    return Hp, Wp, py // 2, px // 2


def fit_background(amp: np.ndarray, percentile, fit_type):
    """(a, b) of the radial background of image_proc.py:458-492: pixels at or below the given
    percentile of the amplitude, fitted by a·exp(-b·r) or a·r^-b with r measured from the
    (H//2, W//2) centre, a, b ≥ 0, by scipy.optimize.curve_fit (the reference's solver: TRF under
    bounds, maxfev 10000, started at (max, 0.1) / (max, 1))."""
    from scipy.optimize import curve_fit
    keep = amp <= np.percentile(amp, percentile)
    yy, xx = np.indices(amp.shape)
    cy, cx = amp.shape[0] // 2, amp.shape[1] // 2
    r = np.sqrt((xx - cx) ** 2 + (yy - cy) ** 2) + 1e-10
    rr, vv = r[keep], amp[keep]
    if fit_type == "exp":
        def model(x, a, b):
            return a * np.exp(-b * x)
        start = [np.max(vv), 0.1]
    else:
        def model(x, a, b):
            return a * x ** -b
        start = [np.max(vv), 1]
    popt, _ = curve_fit(model, rr, vv, p0=start, bounds=([0, 0], [np.inf, np.inf]), maxfev=10000)
    return float(popt[0]), float(popt[1])


def meas_mean(p, stats: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """ptyx_meas_mean: the (Ho, Wo) f64 mean of the processed stack, from its statistics."""
    lib = _lib.load()
    Ho, Wo = _out_shape(p, H, W)
    dev = stats.device
    mean = torch.empty((Ho, Wo), dtype=torch.float64, device=dev)
    _lib.check(lib.ptyx_meas_mean(_stream(dev), H, W, ctypes.byref(p), _p(stats), _p(_ws(lib, Ho, Wo, dev)),
                                  _p(mean)))
    return mean


def meas_mean_seq(raw: torch.Tensor, p, stats: torch.Tensor, normalized: bool) -> torch.Tensor:
    """ptyx_meas_mean_seq: numpy's f32 meas.mean(0) of the stack after the negative-value rule
    (normalized False) or after normalisation by p's constant (True), bit for bit: (Ho, Wo) f32."""
    lib = _lib.load()
    n, H, W = raw.shape
    Ho, Wo = _out_shape(p, H, W)
    mean = torch.empty((Ho, Wo), dtype=torch.float32, device=raw.device)
    _lib.check(lib.ptyx_meas_mean_seq(_stream(raw.device), _p(raw), n, H, W, ctypes.byref(p), _p(stats),
                                      _p(_ws(lib, Ho, Wo, raw.device)), int(bool(normalized)), _p(mean)))
    return mean


def reference_normalization(raw: torch.Tensor, p, stats: torch.Tensor):
    """The proc with the reference's own f32 normalisation constant (initialization.py:928-944:
    max / mean / sum of the f32 mean pattern, computed by numpy on exactly that pattern), as a
    divide_const: the stored stack is then bit-identical to the reference's meas / const."""
    if p.norm_mode == _NORM["divide_const"]:
        return p
    m = meas_mean_seq(raw, p, stats, False).cpu().numpy()
    const = {0: m.max(), 1: m.mean(), 2: m.sum()}[p.norm_mode]
    q = _lib.MeasProc()
    ctypes.memmove(ctypes.byref(q), ctypes.byref(p), ctypes.sizeof(p))
    q.norm_mode, q.norm_value = _NORM["divide_const"], float(const)
    return q


def pad_background(mean: torch.Tensor, pad: dict):
    """The padded background canvas (initialization.py:986-1025) on the device from the mean
    pattern (f32: the reference's own, or f64 from the statistics): (bg (Hp, Wp) f64,
    (Hp, Wp, h1, w1), (a, b))."""
    lib = _lib.load()
    Ho, Wo = mean.shape
    Hp, Wp, h1, w1 = pad_geometry(Ho, Wo, pad)
    a = b = 0.0
    if pad["type"] in ("exp", "power"):
        amp = np.sqrt(mean.cpu().numpy().astype(np.float32))   # the reference's f32 amp_avg
        a, b = fit_background(amp, pad["threshold"], pad["type"])
    mean = mean.double()
    value = float(pad["value"]) if pad["type"] in ("constant", "linear_ramp") else 0.0
    bg = torch.empty((Hp, Wp), dtype=torch.float64, device=mean.device)
    _lib.check(lib.ptyx_meas_pad_background(_stream(mean.device), _p(mean), Ho, Wo, _PAD_TYPES[pad["type"]], a, b,
                                            value, Hp, Wp, h1, w1, _p(bg)))
    return bg, (Hp, Wp, h1, w1), (a, b)


def pad_resample(meas: torch.Tensor, bg, geom, out_hw, out_f16=False) -> torch.Tensor:
    """ptyx_meas_pad_resample: paste every frame of meas (n, Hm, Wm) into the background canvas
    (bg None = no padding) and zoom it to out_hw (order-1 spline, scipy's grid), in one pass."""
    lib = _lib.load()
    n, Hm, Wm = meas.shape
    Hp, Wp, h1, w1 = geom if bg is not None else (Hm, Wm, 0, 0)
    Ho, Wo = out_hw
    out = torch.empty((n, Ho, Wo), dtype=torch.float16 if out_f16 else torch.float32, device=meas.device)
    _lib.check(lib.ptyx_meas_pad_resample(_stream(meas.device), _p(meas), int(meas.dtype == torch.float16), n, Hm, Wm,
                                          None if bg is None else _p(bg), Hp, Wp, h1, w1, Ho, Wo, _p(out),
                                          int(bool(out_f16))))
    return out


def process_meas_ex(raw: torch.Tensor, init_params: dict, out_f16=False, reduce_across_ranks=False,
                    chunk_frames=None):
    """_process_meas (initialization.py:709-752) on a device-resident (n, H, W) f32 stack: flipT,
    ky/kx crop, negative values, normalisation, meas_pad, meas_resample, final clip.  Returns
    (meas, extras); extras holds what the reference leaves in init_variables / init_params:
    on_the_fly_meas_padded ((1, Hp, Wp) f64 device tensor or None), on_the_fly_meas_padded_idx,
    on_the_fly_meas_scale_factors, meas_Npix, and pad_int_sum (the on-the-fly background's
    intensity that init_measurements adds to meas_avg_sum, :107-112)."""
    n, H, W = raw.shape
    p = proc_from_params(init_params, H, W)
    pad = pad_config(init_params)
    rs = resample_config(init_params, otf_pad=pad is not None and pad["mode"] == "on_the_fly")
    stats = meas_stats(raw, p, chunk_frames)
    if reduce_across_ranks:
        allreduce_stats(stats)
    # one rank holding the whole stack: the reference's f32 normalisation constant and mean
    # pattern exactly (a sequential f32 pass); sharded / chunked: the f64 statistics (≈ 1e-6)
    exact = not reduce_across_ranks and n > 0
    if exact:
        p = reference_normalization(raw, p, stats)
    Ho, Wo = _out_shape(p, H, W)
    extras = {"on_the_fly_meas_padded": None, "on_the_fly_meas_padded_idx": None,
              "on_the_fly_meas_scale_factors": None, "meas_Npix": Wo, "pad_int_sum": 0.0, "pad_fit": None}
    bg, geom, cur = None, None, (Ho, Wo)
    if pad is not None:
        mean = meas_mean_seq(raw, p, stats, True) if exact else meas_mean(p, stats, H, W)
        bg, geom, extras["pad_fit"] = pad_background(mean, pad)
        extras["meas_Npix"] = geom[1]
        if pad["mode"] == "on_the_fly":
            Hp, Wp, h1, w1 = geom
            extras["on_the_fly_meas_padded"] = bg[None]
            extras["on_the_fly_meas_padded_idx"] = [h1, h1 + Ho, w1, w1 + Wo]
            extras["pad_int_sum"] = float(bg.sum())
        else:
            cur = geom[:2]
    out_hw = cur
    if rs is not None:
        s = rs["scale"]
        if rs["mode"] == "precompute":
            out_hw = (int(round(cur[0] * float(s))), int(round(cur[1] * float(s))))   # scipy.ndimage.zoom's shape
            extras["meas_Npix"] = out_hw[1]
        else:
            extras["meas_Npix"] = math.floor(extras["meas_Npix"] * s)
            extras["on_the_fly_meas_scale_factors"] = [s, s]
    precompute_pad = pad is not None and pad["mode"] == "precompute"
    if not precompute_pad and out_hw == (Ho, Wo):
        return meas_finish(raw, p, stats, out_f16), extras
    m32 = meas_finish(raw, p, stats, False)
    meas = pad_resample(m32, bg if precompute_pad else None, geom, out_hw, out_f16)
    del m32
    return meas, extras


def process_meas(raw: torch.Tensor, init_params: dict, out_f16=False, reduce_across_ranks=False, chunk_frames=None):
    """process_meas_ex without the extras: the processed stack only."""
    return process_meas_ex(raw, init_params, out_f16, reduce_across_ranks, chunk_frames)[0]


def ingest_raw(file_path, init_params: dict, device="cuda", file_shape=None, offset=0, gap=1024, out_f16=False,
               rank=0, world=1):
    """load_raw + _process_meas for this rank's share of the scan; returns (meas, info) where info
    holds the updated (pos_N_scan_slow, pos_N_scan_fast, meas_Npix, rows) like the reference's
    init_params after meas_crop / meas_pad / meas_resample, plus process_meas_ex's extras (the
    on-the-fly init_variables)."""
    N_slow, N_fast = int(init_params["pos_N_scan_slow"]), int(init_params["pos_N_scan_fast"])
    N, H, W = file_shape if file_shape is not None else (N_slow * N_fast, init_params["meas_Npix"],
                                                         init_params["meas_Npix"])
    if N != N_slow * N_fast:
        raise ValueError(f"file has {N} frames, scan is {N_slow} x {N_fast}")
    crop = init_params.get("meas_crop") or [None, None, None, None]
    s0, s1 = _bounds(crop[0], N_slow) if crop[0] is not None else (0, N_slow)
    f0, f1 = _bounds(crop[1], N_fast) if crop[1] is not None else (0, N_fast)
    rows = list(range(s0, s1))
    mine = rows[rank * len(rows) // world:(rank + 1) * len(rows) // world]
    dev = torch.device(device)
    raw = torch.empty((len(mine) * (f1 - f0), H, W), dtype=torch.float32, device=dev)
    lib = _lib.load()
    for i, r in enumerate(mine):           # one contiguous frame run per scan row
        dst = raw[i * (f1 - f0):(i + 1) * (f1 - f0)]
        _lib.check(lib.ptyx_raw_read(_stream(dev), str(file_path).encode(), int(offset), H, W, int(gap), N,
                                     r * N_fast + f0, f1 - f0, _p(dst)))
    meas, extras = process_meas_ex(raw, init_params, out_f16=out_f16, reduce_across_ranks=world > 1)
    del raw
    info = {"pos_N_scan_slow": s1 - s0, "pos_N_scan_fast": f1 - f0, "pos_N_scans": (s1 - s0) * (f1 - f0),
            "meas_shape": tuple(meas.shape[-2:]), "rows": (mine[0], mine[-1] + 1) if mine else (s0, s0)}
    info.update(extras)
    return meas, info
