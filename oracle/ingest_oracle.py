"""CPU oracle for measurement ingest.

TEST INFRASTRUCTURE ONLY: imported by tests/, never by ptyrad_amd (the product path is the
ptyx_raw_read / ptyx_meas_* C ABI of libptyx.so).

NumPy restatement of
  load_raw                  src/ptyrad/load.py:19-49       (EMPAD: offset + N × (H·W·4 + gap) bytes)
  Initializer._process_meas src/ptyrad/initialization.py:709-752, with
    _meas_flipT             :766-792   flipud (axis 1), fliplr (axis 2), transpose, in that order
    _meas_crop              :794-835   [[slow], [fast], [ky], [kx]] ranges, None = whole axis
    _meas_remove_neg_values :837-890   skipped when there is no negative value and not force
    _meas_normalization     :892-935   max_at_one (default), mean_at_one, sum_to_one, divide_const
    _meas_pad               :956-1048  constant / edge / linear_ramp (numpy.pad semantics, f32 amp)
                                       and exp / power (image_proc.py:458-492 background fit)
    _meas_resample          :1050-1102 precompute = scipy.ndimage.zoom(order=1), on-the-fly = factors
  and the final clip_neg guard (:750).
Pinned by tests/golden/ingest_*.npz, which make_golden_ingest.py produced by running the
reference functions themselves; the pad / zoom restatements are also checked against numpy.pad
and scipy.ndimage.zoom directly (tests/test_ingest.py).  The background fit calls
scipy.optimize.curve_fit, the reference's own third-party solver (scipy 1.15.3 here).
"""
from __future__ import annotations

import os

import numpy as np


def load_raw(path, shape, offset=0, gap=1024):
    """load.py:19-49."""
    N, H, W = shape
    expected = offset + N * (H * W * 4 + gap)
    if os.path.getsize(path) != expected:
        raise ValueError(f"file size {os.path.getsize(path)} != expected {expected}")
    b = np.fromfile(path, dtype=np.uint8, count=expected - offset, offset=offset)
    return b.reshape(N, H * W * 4 + gap)[:, :H * W * 4].copy().view(np.float32).reshape(N, H, W)


def process_meas(meas, params, n_slow, n_fast):
    """initialization.py:709-752 for the supported keys; returns (meas, n_slow, n_fast)."""
    m = np.asarray(meas, np.float32)
    f = params.get("meas_flipT")
    if f is not None:
        if int(f[0]):
            m = np.flip(m, axis=1)
        if int(f[1]):
            m = np.flip(m, axis=2)
        if int(f[2]):
            m = np.transpose(m, (0, 2, 1))
    c = params.get("meas_crop")
    if c is not None:
        m = m.reshape(n_slow, n_fast, *m.shape[-2:])
        sl = [slice(None) if b is None else slice(b[0], b[1]) for b in c]
        m = m[sl[0], sl[1], sl[2], sl[3]]
        n_slow, n_fast = m.shape[0], m.shape[1]
        m = m.reshape(-1, m.shape[-2], m.shape[-1])
    m = np.array(m, np.float32)
    neg = params.get("meas_remove_neg_values") or {}
    mode, value, force = neg.get("mode", "clip_neg"), neg.get("value"), neg.get("force", False)
    if (m < 0).any() or force:
        if mode == "subtract_min":
            m -= m.min()
        elif mode == "clip_value":
            m[m < value] = 0
        elif mode == "subtract_value":
            m -= np.float32(value)
        else:
            m[m < 0] = 0
        m[m < 0] = 0
    norm = params.get("meas_normalization") or {}
    nm = norm.get("mode", "max_at_one")
    avg = m.mean(0)          # f32, sequential over the frames (numpy's axis-0 reduction)
    const = {"max_at_one": avg.max(), "mean_at_one": avg.mean(), "sum_to_one": avg.sum()}.get(nm)
    if nm == "divide_const":
        const = norm["value"]
    m = (m / np.float32(const)).astype(np.float32)
    m[m < 0] = 0
    return m, n_slow, n_fast


def linear_ramp_pad(a, pads, end):
    """numpy.pad(a, pads, 'linear_ramp', end_values=end) for 2-D a, restated: axis 0 over the
    original columns first, then axis 1 over every row; ramp k of a side of width w is
    k·(edge − end)/w + end (linspace without endpoint), reversed on the trailing side."""
    (t, b), (l, r) = pads
    H, W = a.shape
    out = np.zeros((H + t + b, W + l + r), a.dtype)
    out[t:t + H, l:l + W] = a

    def ramp(edge, w):
        k = np.arange(w, dtype=np.float64)[:, None]
        return (k * ((edge.astype(np.float64) - end) / w) + end).astype(a.dtype)
    if t:
        out[:t, l:l + W] = ramp(a[0][None], t).reshape(t, W)
    if b:
        out[t + H:, l:l + W] = ramp(a[-1][None], b)[::-1].reshape(b, W)
    if l:
        out[:, :l] = ramp(out[:, l][None], l).T
    if r:
        out[:, l + W:] = ramp(out[:, l + W - 1][None], r)[::-1].T
    return out


def zoom_order1(m, sy, sx):
    """scipy.ndimage.zoom(m, (1, sy, sx), order=1) for (n, H, W) m: output shape round(H·s),
    output pixel o reads input coordinate o·(H−1)/(Ho−1) (grid_mode False), bilinear in f64."""
    n, H, W = m.shape
    Ho, Wo = int(round(H * sy)), int(round(W * sx))

    def axis(nin, nout):
        c = np.arange(nout) * ((nin - 1) / (nout - 1) if nout > 1 else 1.0)
        i0 = np.minimum(np.floor(c).astype(np.int64), nin - 1)
        t = np.maximum(c - i0, 0.0)
        return i0, np.minimum(i0 + 1, nin - 1), t, c > nin - 1
    y0, y1, ty, oy = axis(H, Ho)
    x0, x1, tx, ox = axis(W, Wo)
    f = m.astype(np.float64)
    wy, wx = (1 - ty)[:, None], (1 - tx)[None]
    ty, tx = ty[:, None], tx[None]
    v = f[:, y0][:, :, x0] * wy * wx
    v = v + f[:, y0][:, :, x1] * wy * tx
    v = v + f[:, y1][:, :, x0] * ty * wx
    v = v + f[:, y1][:, :, x1] * ty * tx
    # mode 'constant': a coordinate past the last pixel, even by the rounding of o·(H−1)/(Ho−1)
    # (e.g. 15·(31/15) = 31.000000000000004 when 32 px zoom by 0.5), is cval = 0 for the pixel
    v[:, oy[:, None] | ox[None]] = 0.0
    return v.astype(m.dtype)


def fit_background(amp, percentile, fit_type):
    """image_proc.py:458-492: the percentile mask and scipy.optimize.curve_fit of a·exp(-b r) or
    a·r^-b (bounds a, b ≥ 0, maxfev 10000)."""
    from scipy.optimize import curve_fit
    mask = amp <= np.percentile(amp, percentile)
    y, x = np.indices(amp.shape)
    c = np.array(amp.shape) // 2
    r = np.sqrt((x - c[1]) ** 2 + (y - c[0]) ** 2) + 1e-10
    f = (lambda r, a, b: a * np.exp(-b * r)) if fit_type == "exp" else (lambda r, a, b: a * r ** -b)
    p0 = [np.max(amp[mask]), 0.1 if fit_type == "exp" else 1]
    popt, _ = curve_fit(f, r[mask], amp[mask], p0=p0, bounds=([0, 0], [np.inf, np.inf]), maxfev=10000)
    return popt


def pad_meas(m, cfg):
    """_meas_pad :956-1048 → (meas, padded (1,Hp,Wp) or None, idx or None, Npix)."""
    mode, ptype, T = cfg["mode"], cfg["padding_type"], cfg["target_Npix"]
    value, thr = cfg.get("value", 10), cfg.get("threshold", 70)
    amp = np.sqrt(m.mean(axis=0))
    H, W = amp.shape
    py, px = max(0, T - H), max(0, T - W)
    t, l = py // 2, px // 2
    pads = ((t, py - t), (l, px - l))
    if ptype == "constant":
        ap = np.pad(amp, pads, mode="constant", constant_values=value)
    elif ptype == "edge":
        ap = np.pad(amp, pads, mode="edge")
    elif ptype == "linear_ramp":
        ap = linear_ramp_pad(amp, pads, value)
    else:
        yy, xx = np.ogrid[:T, :T]
        r = np.sqrt((yy - (H // 2 + t)) ** 2 + (xx - (W // 2 + l)) ** 2) + 1e-10
        a, b = fit_background(amp, thr, ptype)
        ap = a * np.exp(-b * r) if ptype == "exp" else a * r ** -b
    bg = np.square(ap)[None]
    bg[..., t:t + H, l:l + W] = 0
    if mode == "precompute":
        canvas = np.zeros((m.shape[0], *bg.shape[1:]))
        canvas += bg
        canvas[..., t:t + H, l:l + W] = m
        return canvas, None, None, bg.shape[-1]
    return m, bg, [t, t + H, l, l + W], bg.shape[-1]


def process_meas_full(meas, params, n_slow, n_fast):
    """process_meas + meas_pad + meas_resample: (meas, n_slow, n_fast, extras) with extras the
    on-the-fly init_variables and the final meas_Npix."""
    m, n_slow, n_fast = process_meas(meas, params, n_slow, n_fast)
    ex = {"on_the_fly_meas_padded": None, "on_the_fly_meas_padded_idx": None,
          "on_the_fly_meas_scale_factors": None, "meas_Npix": m.shape[-1]}
    pad = params.get("meas_pad")
    if pad is not None and pad.get("mode") is not None:
        m, bg, idx, ex["meas_Npix"] = pad_meas(m, pad)
        ex["on_the_fly_meas_padded"], ex["on_the_fly_meas_padded_idx"] = bg, idx
    rs = params.get("meas_resample")
    if rs is not None and rs.get("mode") is not None:
        sf = rs["scale_factors"]
        s = min(sf) if sf[0] != sf[1] else sf[0]
        mode = "on_the_fly" if ex["on_the_fly_meas_padded"] is not None else rs["mode"]
        if mode == "precompute":
            m = zoom_order1(m, s, s)
            ex["meas_Npix"] = m.shape[-1]
        else:
            ex["meas_Npix"] = int(np.floor(ex["meas_Npix"] * s))
            ex["on_the_fly_meas_scale_factors"] = [s, s]
    m = np.where(m < 0, 0, m)
    return m, n_slow, n_fast, ex
