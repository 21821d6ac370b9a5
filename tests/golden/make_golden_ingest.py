"""Golden fixtures for measurement ingest, made by running the reference:
src/ptyrad/load.py:load_raw (:19-49, EMPAD layout: offset + N × (H·W·4 + gap) bytes) on a raw
file written here, then Initializer._process_meas (src/ptyrad/initialization.py:709-752:
flipT :766-792, crop :794-835, remove_neg_values :837-890, normalization :892-935) on it.

Run here (build container) only:  python tests/golden/make_golden_ingest.py
Writes tests/golden/ingest_<case>.npz: frames (N,H,W) f32 = the data part of the raw file, the
file layout (offset, gap, N_slow, N_fast), the processing params (JSON) and the reference output
meas (after _process_meas).  Data only; no reference source is copied.
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


def main():
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


if __name__ == "__main__":
    assert os.path.isdir(REF_SRC), "the reference is needed to (re)generate fixtures"
    main()
