"""CPU: the ingest oracle (oracle/ingest_oracle.py) against the reference's own load_raw +
_process_meas outputs (tests/golden/ingest_*.npz), the host-side parameter mapping, and the
C-ABI argument checks of ptyx_raw_read that run before any HIP call."""
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


def load_case(name):
    z = np.load(os.path.join(GOLD, f"ingest_{name}.npz"))
    return z, json.loads(str(z["params"]))


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
    m, ns, nf = io.process_meas(raw, proc, int(z["n_slow"]), int(z["n_fast"]))
    assert (ns, nf) == (int(z["out_n_slow"]), int(z["out_n_fast"]))
    assert m.shape == z["meas"].shape
    np.testing.assert_allclose(m, z["meas"], rtol=2e-6, atol=1e-7)


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
        ingest.proc_from_params({"meas_pad": {"mode": "on_the_fly"}}, 16, 16)
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
