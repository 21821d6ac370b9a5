"""CPU: the ingest oracle (oracle/ingest_oracle.py) against the reference's own load_raw +
_process_meas outputs (tests/golden/ingest_*.npz, meas_pad / meas_resample included), its pad and
zoom restatements against numpy.pad / scipy.ndimage.zoom, the host-side parameter mapping (the
demos' own init_params included), and the C-ABI argument checks that run before any HIP call."""
import ctypes
import glob
import json
import os

import numpy as np
import pytest

from oracle import ingest_oracle as io

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLD, "ingest_*.npz")))


def write_raw(path, frames, offset, gap):
    rng = np.random.default_rng(0)
    with open(path, "wb") as f:
        f.write(rng.integers(0, 255, offset, dtype=np.uint8).tobytes())
        for fr in frames:
            f.write(np.ascontiguousarray(fr, np.float32).tobytes())
            f.write(rng.integers(0, 255, gap, dtype=np.uint8).tobytes())


PAD_CASES = [c for c in CASES if "otf_padded" in np.load(os.path.join(GOLD, f"ingest_{c}.npz")).files]


def load_case(name):
    z = np.load(os.path.join(GOLD, f"ingest_{name}.npz"))
    return z, json.loads(str(z["params"]))


def demo_params():
    with open(os.path.join(GOLD, "demo_init_params.json")) as f:
        return json.load(f)


def test_cases_present():
    assert {"default", "flip_crop_submin", "fliplr_clipvalue", "nonneg_skip", "nonneg_force"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name, tmp_path):
    z, proc = load_case(name)
    fr = z["frames"]
    path = str(tmp_path / "scan.raw")
    write_raw(path, fr, int(z["offset"]), int(z["gap"]))
    raw = io.load_raw(path, fr.shape, int(z["offset"]), int(z["gap"]))
    assert np.array_equal(raw, fr)
    m, ns, nf, ex = io.process_meas_full(raw, proc, int(z["n_slow"]), int(z["n_fast"]))
    assert (ns, nf) == (int(z["out_n_slow"]), int(z["out_n_fast"]))
    assert m.shape == z["meas"].shape
    # bit for bit: the oracle restates numpy's f32 arithmetic (sequential axis-0 mean, f32 const)
    np.testing.assert_array_equal(m.astype(np.float32), z["meas"])
    if name in PAD_CASES:
        assert ex["meas_Npix"] == int(z["out_npix"])
        if z["otf_padded"].size:
            np.testing.assert_allclose(ex["on_the_fly_meas_padded"], z["otf_padded"], rtol=1e-6, atol=0)
            assert list(ex["on_the_fly_meas_padded_idx"]) == list(z["otf_padded_idx"])
        else:
            assert ex["on_the_fly_meas_padded"] is None
        sf = ex["on_the_fly_meas_scale_factors"]
        assert (sf is None and not z["otf_scale_factors"].size) or list(sf) == list(z["otf_scale_factors"])


def test_pad_cases_cover_every_option():
    """Fixtures for all five padding types, both pad modes, both resample modes and the demos."""
    seen = set()
    for c in PAD_CASES:
        _, proc = load_case(c)
        pad, rs = proc.get("meas_pad") or {}, proc.get("meas_resample") or {}
        if pad.get("mode"):
            seen |= {pad["padding_type"], "pad_" + pad["mode"]}
        if rs.get("mode"):
            seen.add("resample_" + rs["mode"])
    assert {"constant", "edge", "linear_ramp", "exp", "power", "pad_precompute", "pad_on_the_fly",
            "resample_precompute", "resample_on_the_fly"} <= seen
    assert {"pso_demo", "tbl_demo"} <= set(PAD_CASES)


def test_linear_ramp_restatement_matches_numpy_pad():
    rng = np.random.default_rng(7)
    for dt in (np.float32, np.float64):
        a = rng.random((9, 6)).astype(dt)
        for pads in (((3, 4), (2, 5)), ((0, 1), (7, 0)), ((5, 5), (0, 0))):
            want = np.pad(a, pads, mode="linear_ramp", end_values=0.3)
            got = io.linear_ramp_pad(a, pads, 0.3)
            assert got.dtype == want.dtype
            np.testing.assert_allclose(got, want, rtol=2e-7 if dt == np.float32 else 1e-15, atol=0)


def test_zoom_restatement_matches_scipy():
    """oracle zoom_order1 against scipy.ndimage.zoom(order=1) itself: same shapes, ≤ 1 f32 ulp
    (f64 arithmetic in a different association order rounds differently about 1 in 2000)."""
    import scipy.ndimage as nd
    rng = np.random.default_rng(8)
    for H, W in ((9, 11), (32, 32), (17, 40)):
        m = (rng.random((2, H, W)) * 5).astype(np.float32)
        for s in (2.0, 1.3334, 0.5, 0.75, 3.0, 1.1):
            want = nd.zoom(m, (1, s, s), order=1)
            got = io.zoom_order1(m, s, s)
            assert got.shape == want.shape
            np.testing.assert_allclose(got, want, rtol=1.2e-7, atol=1e-30)


@pytest.mark.parametrize("demo", ["PSO", "tBL_WSe2"])
def test_demo_init_params_are_accepted(demo):
    """The demos' own measurement settings (demo/params/*.yml, captured as data in
    tests/golden/demo_init_params.json) go through the host mapping: the tBL demo's {'mode': null}
    pad / resample dicts are off, the PSO demo's power pad is on the fly to 256 after a 68:188 crop."""
    from ptyrad_amd import ingest
    ip = demo_params()[demo]
    H = W = ip["meas_Npix"]
    p = ingest.proc_from_params(ip, H, W)
    Ho, Wo = ingest._out_shape(p, H, W)
    pad = ingest.pad_config(ip)
    rs = ingest.resample_config(ip, otf_pad=pad is not None and pad["mode"] == "on_the_fly")
    assert rs is None
    if demo == "tBL_WSe2":
        assert pad is None and (p.flipud, p.fliplr, p.transpose) == (1, 0, 0) and (Ho, Wo) == (128, 128)
    else:
        assert (Ho, Wo) == (120, 120)
        assert pad == {"mode": "on_the_fly", "type": "power", "target": 256, "value": 0, "threshold": 70}
        assert ingest.pad_geometry(Ho, Wo, pad) == (256, 256, 68, 68)


def test_pad_resample_config_rules():
    from ptyrad_amd import ingest
    assert ingest.pad_config({"meas_pad": None}) is None
    assert ingest.pad_config({"meas_pad": {"mode": None, "padding_type": "bogus"}}) is None
    with pytest.raises(ValueError):
        ingest.pad_config({"meas_pad": {"mode": "later", "padding_type": "edge", "target_Npix": 64}})
    with pytest.raises(ValueError):
        ingest.pad_config({"meas_pad": {"mode": "precompute", "padding_type": "reflect", "target_Npix": 64}})
    assert ingest.pad_config({"meas_pad": {"mode": "precompute", "padding_type": "edge", "target_Npix": 64}})[
        "value"] == 10       # initialization.py:981 default
    rs = {"meas_resample": {"mode": "precompute", "scale_factors": [0.75, 0.8]}}
    assert ingest.resample_config(rs, otf_pad=False) == {"mode": "precompute", "scale": 0.75}
    assert ingest.resample_config(rs, otf_pad=True) == {"mode": "on_the_fly", "scale": 0.75}
    with pytest.raises(ValueError):
        ingest.resample_config({"meas_resample": {"mode": "precompute", "scale_factors": [2]}}, False)
    with pytest.raises(ValueError):
        ingest.pad_geometry(130, 130, {"type": "power", "target": 128})
    assert ingest.pad_geometry(130, 100, {"type": "edge", "target": 128}) == (130, 128, 0, 14)


def test_proc_mapping_and_shapes():
    from ptyrad_amd import ingest
    p = ingest.proc_from_params({"meas_flipT": [1, 0, 1], "meas_crop": [[1, 5], [2, 7], [3, 29], [2, 30]],
                                 "meas_remove_neg_values": {"mode": "subtract_min"},
                                 "meas_normalization": {"mode": "mean_at_one"}}, 32, 40)
    assert (p.flipud, p.fliplr, p.transpose) == (1, 0, 1)
    assert (p.crop_ky0, p.crop_ky1, p.crop_kx0, p.crop_kx1) == (3, 29, 2, 30)
    assert (p.neg_mode, p.norm_mode) == (1, 1)
    assert ingest._out_shape(p, 32, 40) == (26, 28)
    q = ingest.proc_from_params({}, 16, 16)
    assert (q.neg_mode, q.norm_mode, q.crop_ky1) == (0, 0, -1) and ingest._out_shape(q, 16, 16) == (16, 16)
    with pytest.raises(NotImplementedError):
        ingest.proc_from_params({"meas_reshape": [4, 16, 16]}, 16, 16)
    ingest.proc_from_params({"meas_pad": {"mode": "on_the_fly"}, "meas_add_detector_blur": 0}, 16, 16)
    with pytest.raises(KeyError):
        ingest.proc_from_params({"meas_remove_neg_values": {"mode": "clip_value"}}, 16, 16)


def test_raw_read_checks_file_without_gpu(tmp_path):
    from ptyrad_amd import _lib
    lib = _lib.load()
    path = str(tmp_path / "x.raw")
    write_raw(path, np.zeros((3, 4, 4), np.float32), 0, 1024)
    # wrong frame count → the reference's size check (load.py:27-31) fails before any HIP call
    rc = lib.ptyx_raw_read(None, path.encode(), 0, 4, 4, 1024, 4, 0, 4, ctypes.c_void_p(8))
    assert rc == _lib.PTYX_EINVAL and b"file size" in lib.ptyx_last_error()
    assert lib.ptyx_raw_read(None, b"/nonexistent.raw", 0, 4, 4, 1024, 3, 0, 3, ctypes.c_void_p(8)) == _lib.PTYX_EINVAL
    assert lib.ptyx_raw_read(None, path.encode(), 0, 4, 4, 1024, 3, 2, 5, ctypes.c_void_p(8)) == _lib.PTYX_EINVAL
    assert lib.ptyx_meas_stats_len(4, 5) == 2 + 40
    # pad / resample argument checks fail before any launch
    assert lib.ptyx_meas_pad_background(None, None, 8, 8, 5, 0.0, 0.0, 0.0, 16, 16, 4, 4, ctypes.c_void_p(8)) == \
        _lib.PTYX_EINVAL
    assert lib.ptyx_meas_pad_background(None, None, 8, 8, 1, 0.0, 0.0, 0.0, 16, 16, 9, 4, ctypes.c_void_p(8)) == \
        _lib.PTYX_EINVAL
    assert lib.ptyx_meas_pad_resample(None, ctypes.c_void_p(8), 0, 2, 8, 8, None, 16, 16, 4, 4, 16, 16,
                                      ctypes.c_void_p(8), 0) == _lib.PTYX_EINVAL
    assert lib.ptyx_meas_pad_resample(None, None, 0, 0, 8, 8, None, 8, 8, 0, 0, 12, 12, None, 0) == _lib.PTYX_OK
