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
  and the final clip_neg guard (:750).
Pinned by tests/golden/ingest_*.npz, which make_golden_ingest.py produced by running the
reference functions themselves.
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
    avg = m.astype(np.float64).mean(0)
    const = {"max_at_one": avg.max(), "mean_at_one": avg.mean(), "sum_to_one": avg.sum()}.get(nm)
    if nm == "divide_const":
        const = norm["value"]
    m = (m / np.float32(const)).astype(np.float32)
    m[m < 0] = 0
    return m, n_slow, n_fast
