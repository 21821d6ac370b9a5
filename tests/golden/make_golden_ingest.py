"""Golden fixtures for measurement ingest, made by running the reference:
src/ptyrad/load.py:load_raw (:19-49, EMPAD layout: offset + N × (H·W·4 + gap) bytes) on a raw
file written here, then Initializer._process_meas (src/ptyrad/initialization.py:709-752:
flipT :766-792, crop :794-835, remove_neg_values :837-890, normalization :892-935) on it.

Run here (build container) only:  python tests/golden/make_golden_ingest.py [--pad-only]
Writes tests/golden/ingest_<case>.npz: frames (N,H,W) f32 = the data part of the raw file, the
file layout (offset, gap, N_slow, N_fast), the processing params (JSON) and the reference output
meas (after _process_meas).  The meas_pad / meas_resample cases (initialization.py:956-1102,
--pad-only) also hold the model-side on-the-fly variables (on_the_fly_meas_padded, its idx,
on_the_fly_meas_scale_factors) and the updated meas_Npix; two of them run the PSO and tBL_WSe2
demos' own measurement settings, whose values (not the YAML text) go to demo_init_params.json.
Data only; no reference source is copied.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from refimport import REF_SRC, import_reference  # noqa: E402

import_reference()
from ptyrad.initialization import Initializer  # noqa: E402
from ptyrad.load import load_raw  # noqa: E402

BASE = {"meas_permute": None, "meas_reshape": None, "meas_flipT": None, "meas_crop": None,
        "meas_remove_neg_values": None, "meas_normalization": None, "meas_pad": None,
        "meas_resample": None, "meas_add_source_size": None, "meas_add_detector_blur": None,
        "meas_add_poisson_noise": None}


def write_raw(path, frames, offset, gap, rng):
    with open(path, "wb") as f:
        f.write(rng.integers(0, 255, offset, dtype=np.uint8).tobytes())
        for fr in frames:
            f.write(np.ascontiguousarray(fr, dtype=np.float32).tobytes())
            f.write(rng.integers(0, 255, gap, dtype=np.uint8).tobytes())


def run_case(name, n_slow, n_fast, H, seed, proc, offset=0, gap=1024, nonneg=False):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[:H, :H] - H / 2
    disk = (np.hypot(yy, xx) < H / 4).astype(np.float32)
    N = n_slow * n_fast
    frames = (disk[None] * rng.uniform(50, 100, (N, 1, 1)) + rng.normal(0, 2.0, (N, H, H))).astype(np.float32)
    if nonneg:
        frames = np.abs(frames) + 0.2
    params = dict(BASE, **proc)
    params.update(pos_N_scans=N, meas_Npix=H, pos_N_scan_slow=n_slow, pos_N_scan_fast=n_fast)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scan.raw")
        write_raw(path, frames, offset, gap, rng)
        raw = load_raw(path, (N, H, H), offset=offset, gap=gap)
        assert np.array_equal(raw, frames)
    ini = Initializer.__new__(Initializer)
    ini.init_params = dict(params)
    ini.init_params_original = dict(params)
    ini.init_variables = {}
    ini.verbose = False
    meas = ini._process_meas(np.array(raw))
    out = os.path.join(HERE, f"ingest_{name}.npz")
    np.savez_compressed(out, frames=frames, offset=np.int64(offset), gap=np.int64(gap), n_slow=np.int64(n_slow),
                        n_fast=np.int64(n_fast), params=json.dumps(proc), meas=np.asarray(meas, np.float32),
                        meas_raw_avg=np.asarray(ini.init_variables["meas_raw_avg"], np.float32),
                        out_n_slow=np.int64(ini.init_params["pos_N_scan_slow"]),
                        out_n_fast=np.int64(ini.init_params["pos_N_scan_fast"]))
    print("wrote", out, os.path.getsize(out), "bytes", meas.shape)


def detector_frames(N, H, seed, radius, offset_neg=True):
    """Poisson-count CBED-like frames: a bright-field disk on a power-law tail (the background the
    'exp' / 'power' meas_pad fits), integer counts so the fixture compresses; with offset_neg a
    dark-reference subtraction leaves some negative pixels (the clip_neg path)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[:H, :H] - H // 2
    r = np.hypot(yy, xx)
    amp = 6.0 * (r < radius) + 3.0 * (r + 2.0) ** -0.9
    lam = 400.0 * (amp ** 2)[None] * rng.uniform(0.8, 1.2, (N, 1, 1))
    frames = rng.poisson(lam).astype(np.float32)
    if offset_neg:
        frames -= rng.integers(0, 2, frames.shape).astype(np.float32)
    return frames


def run_pad_case(name, n_slow, n_fast, H, seed, proc, radius=None):
    """_process_meas with meas_pad / meas_resample (initialization.py:956-1102) on in-memory frames;
    records the model-side on-the-fly variables and the updated meas_Npix as well."""
    N = n_slow * n_fast
    frames = detector_frames(N, H, seed, radius or H // 6)
    params = dict(BASE, **proc)
    params.update(pos_N_scans=N, meas_Npix=H, pos_N_scan_slow=n_slow, pos_N_scan_fast=n_fast)
    ini = Initializer.__new__(Initializer)
    ini.init_params = dict(params)
    ini.init_params_original = dict(params)
    ini.init_variables = {}
    ini.verbose = False
    meas = ini._process_meas(np.array(frames))
    iv = ini.init_variables
    pad = iv.get("on_the_fly_meas_padded")
    pidx = iv.get("on_the_fly_meas_padded_idx")
    sf = iv.get("on_the_fly_meas_scale_factors")
    out = os.path.join(HERE, f"ingest_{name}.npz")
    np.savez_compressed(out, frames=frames, offset=np.int64(0), gap=np.int64(0), n_slow=np.int64(n_slow),
                        n_fast=np.int64(n_fast), params=json.dumps(proc), meas=np.asarray(meas, np.float32),
                        meas_dtype=str(np.asarray(meas).dtype),
                        otf_padded=np.zeros((0,)) if pad is None else np.asarray(pad, np.float64),
                        otf_padded_idx=np.zeros((0,), np.int64) if pidx is None else np.asarray(pidx, np.int64),
                        otf_scale_factors=np.zeros((0,)) if sf is None else np.asarray(sf, np.float64),
                        out_npix=np.int64(ini.init_params["meas_Npix"]),
                        out_n_slow=np.int64(ini.init_params["pos_N_scan_slow"]),
                        out_n_fast=np.int64(ini.init_params["pos_N_scan_fast"]))
    print("wrote", out, os.path.getsize(out), "bytes", np.asarray(meas).shape, "Npix", ini.init_params["meas_Npix"])


DEMOS = {"PSO": "PSO_reconstruct.yml", "tBL_WSe2": "tBL_WSe2_reconstruct.yml"}
MEAS_KEYS = ("meas_Npix", "pos_N_scans", "pos_N_scan_slow", "pos_N_scan_fast", "meas_permute", "meas_reshape",
             "meas_flipT", "meas_crop", "meas_pad", "meas_resample", "meas_remove_neg_values", "meas_normalization",
             "meas_add_source_size", "meas_add_detector_blur", "meas_add_poisson_noise")


def write_demo_params():
    """The demo YAMLs' measurement-processing init_params (values only) as a JSON fixture, so the
    CPU tests can feed the demos' own settings through the ingest without reading the reference."""
    import yaml
    out = {}
    for name, fn in DEMOS.items():
        with open(os.path.join(os.path.dirname(REF_SRC), "demo", "params", fn)) as f:
            ip = yaml.safe_load(f)["init_params"]
        out[name] = {k: ip.get(k) for k in MEAS_KEYS}
    path = os.path.join(HERE, "demo_init_params.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)
    return out


def pad_cases():
    demos = write_demo_params()
    pso = {k: v for k, v in demos["PSO"].items() if k.startswith("meas_") and k != "meas_Npix"}
    tbl = {k: v for k, v in demos["tBL_WSe2"].items() if k.startswith("meas_") and k != "meas_Npix"}
    # the demos' own ingest settings at their detector sizes, on a small scan
    run_pad_case("pso_demo", 2, 3, 256, seed=11, proc=pso, radius=30)
    run_pad_case("tbl_demo", 2, 3, 128, seed=12, proc=tbl, radius=20)
    # every padding type, both modes, resample precompute (bilinear zoom) and on-the-fly scale factors
    run_pad_case("pad_exp_pre", 2, 2, 40, seed=13, proc={
        "meas_pad": {"mode": "precompute", "padding_type": "exp", "target_Npix": 64, "value": 0, "threshold": 60}})
    run_pad_case("pad_const_pre_rs", 2, 2, 32, seed=14, proc={
        "meas_crop": [None, None, [1, 31], [2, 30]],
        "meas_pad": {"mode": "precompute", "padding_type": "constant", "target_Npix": 48, "value": 0.05},
        "meas_resample": {"mode": "precompute", "scale_factors": [1.5, 1.5]}})
    run_pad_case("pad_edge_pre", 2, 2, 30, seed=15, proc={
        "meas_pad": {"mode": "precompute", "padding_type": "edge", "target_Npix": 45}})
    run_pad_case("pad_ramp_otf", 2, 2, 32, seed=16, proc={
        "meas_flipT": [0, 1, 1],
        "meas_pad": {"mode": "on_the_fly", "padding_type": "linear_ramp", "target_Npix": 50, "value": 0.02},
        "meas_resample": {"mode": "precompute", "scale_factors": [1.25, 1.25]}})
    run_pad_case("pad_power_otf_rs", 2, 2, 40, seed=17, proc={
        "meas_pad": {"mode": "on_the_fly", "padding_type": "power", "target_Npix": 64},
        "meas_resample": {"mode": "on_the_fly", "scale_factors": [1.3334, 1.3334]}})
    run_pad_case("resample_up_pre", 2, 3, 32, seed=18, proc={
        "meas_resample": {"mode": "precompute", "scale_factors": [2, 2]},
        "meas_normalization": {"mode": "sum_to_one"}})
    run_pad_case("resample_down_pre", 2, 3, 36, seed=19, proc={
        "meas_resample": {"mode": "precompute", "scale_factors": [0.75, 0.8]}})
    run_pad_case("resample_otf_only", 2, 2, 32, seed=20, proc={
        "meas_resample": {"mode": "on_the_fly", "scale_factors": [1.5, 1.5]}})
    run_pad_case("pad_power_pre_f64", 3, 2, 48, seed=21, proc={
        "meas_pad": {"mode": "precompute", "padding_type": "power", "target_Npix": 96, "threshold": 75},
        "meas_resample": {"mode": "precompute", "scale_factors": [0.5, 0.5]}})


def main():
    if "--pad-only" in sys.argv:
        pad_cases()
        return
    run_case("default", 6, 8, 32, seed=1, proc={})
    run_case("flip_crop_submin", 6, 8, 32, seed=2, offset=512,
             proc={"meas_flipT": [1, 0, 1], "meas_crop": [[1, 5], [2, 7], [3, 29], [2, 30]],
                   "meas_remove_neg_values": {"mode": "subtract_min"},
                   "meas_normalization": {"mode": "mean_at_one"}})
    run_case("fliplr_clipvalue", 4, 5, 32, seed=3, gap=0,
             proc={"meas_flipT": [0, 1, 0], "meas_remove_neg_values": {"mode": "clip_value", "value": -1.5},
                   "meas_normalization": {"mode": "sum_to_one"}})
    run_case("nonneg_skip", 3, 4, 32, seed=4, nonneg=True,
             proc={"meas_remove_neg_values": {"mode": "subtract_value", "value": 0.1},
                   "meas_normalization": {"mode": "divide_const", "value": 3.0}})
    run_case("nonneg_force", 3, 4, 32, seed=5, nonneg=True,
             proc={"meas_flipT": [1, 1, 0], "meas_crop": [None, [1, 3], None, [0, 31]],
                   "meas_remove_neg_values": {"mode": "subtract_value", "value": 0.5, "force": True}})
    pad_cases()


if __name__ == "__main__":
    assert os.path.isdir(REF_SRC), "the reference is needed to (re)generate fixtures"
    main()
