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

Not supported here (NotImplementedError, run the reference's host path for them): meas_permute,
meas_reshape, meas_pad, meas_resample and the simulation options meas_add_source_size /
meas_add_detector_blur / meas_add_poisson_noise.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib

_NEG = {"clip_neg": 0, "subtract_min": 1, "clip_value": 2, "subtract_value": 3}
_NORM = {"max_at_one": 0, "mean_at_one": 1, "sum_to_one": 2, "divide_const": 3}
_UNSUPPORTED = ("meas_permute", "meas_reshape", "meas_pad", "meas_resample", "meas_add_source_size",
                "meas_add_detector_blur", "meas_add_poisson_noise")


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def proc_from_params(init_params: dict, H: int, W: int) -> _lib.MeasProc:
    """The ptyx_meas_proc of init_params (flipT, ky/kx crop, negative values, normalisation)."""
    for k in _UNSUPPORTED:
        if init_params.get(k) is not None:
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


def process_meas(raw: torch.Tensor, init_params: dict, out_f16=False, reduce_across_ranks=False, chunk_frames=None):
    """_process_meas (initialization.py:709-752) on a device-resident (n, H, W) f32 stack: flipT,
    ky/kx crop, negative values, normalisation, final clip.  With reduce_across_ranks the
    statistics are all-reduced so every rank uses the global constants."""
    p = proc_from_params(init_params, raw.shape[1], raw.shape[2])
    stats = meas_stats(raw, p, chunk_frames)
    if reduce_across_ranks:
        allreduce_stats(stats)
    return meas_finish(raw, p, stats, out_f16)


def ingest_raw(file_path, init_params: dict, device="cuda", file_shape=None, offset=0, gap=1024, out_f16=False,
               rank=0, world=1):
    """load_raw + _process_meas for this rank's share of the scan; returns (meas, info) where info
    holds the updated (pos_N_scan_slow, pos_N_scan_fast, meas_Npix, rows) like the reference's
    init_params after meas_crop."""
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
    meas = process_meas(raw, init_params, out_f16=out_f16, reduce_across_ranks=world > 1)
    del raw
    p = proc_from_params(init_params, H, W)
    Ho, Wo = _out_shape(p, H, W)
    info = {"pos_N_scan_slow": s1 - s0, "pos_N_scan_fast": f1 - f0, "pos_N_scans": (s1 - s0) * (f1 - f0),
            "meas_Npix": Wo, "meas_shape": (Ho, Wo), "rows": (mine[0], mine[-1] + 1) if mine else (s0, s0)}
    return meas, info
