"""GPU: raw EMPAD stack → HBM → processed measurements (ptyrad_amd/ingest.py → libptyx
ptyx_raw_read / ptyx_meas_stats / ptyx_meas_finish) against the reference's load_raw +
_process_meas outputs (tests/golden/ingest_*.npz)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from tests.test_ingest import CASES, GOLD, load_case, write_raw

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def init_params(z, proc):
    d = dict(proc)
    d.update(pos_N_scan_slow=int(z["n_slow"]), pos_N_scan_fast=int(z["n_fast"]), meas_Npix=z["frames"].shape[-1])
    return d


@pytest.mark.parametrize("name", CASES)
def test_ingest_matches_reference(name, dev, tmp_path):
    from ptyrad_amd.ingest import ingest_raw
    z, proc = load_case(name)
    path = str(tmp_path / "scan.raw")
    write_raw(path, z["frames"], int(z["offset"]), int(z["gap"]))
    meas, info = ingest_raw(path, init_params(z, proc), device=dev, file_shape=z["frames"].shape,
                            offset=int(z["offset"]), gap=int(z["gap"]))
    got = meas.cpu().numpy()
    assert got.shape == z["meas"].shape
    assert (info["pos_N_scan_slow"], info["pos_N_scan_fast"]) == (int(z["out_n_slow"]), int(z["out_n_fast"]))
    np.testing.assert_allclose(got, z["meas"], rtol=2e-6, atol=1e-7)
    m16, _ = ingest_raw(path, init_params(z, proc), device=dev, file_shape=z["frames"].shape,
                        offset=int(z["offset"]), gap=int(z["gap"]), out_f16=True)
    ref16 = z["meas"].astype(np.float16).astype(np.float32)
    np.testing.assert_allclose(m16.float().cpu().numpy(), ref16, rtol=1e-3, atol=1e-6)


def test_chunked_stats_and_rank_split(dev):
    """Stats accumulated over frame chunks are bitwise the single-pass ones; two 'ranks' that sum
    their stats reproduce the single-rank stack (the sharded ingest's reduction)."""
    from ptyrad_amd import ingest
    rng = np.random.default_rng(3)
    frames = torch.tensor(rng.normal(1.0, 2.0, (300, 64, 64)).astype(np.float32), device=dev)
    prm = {"meas_flipT": [0, 1, 1], "meas_crop": [None, None, [4, 60], [0, 50]],
           "meas_remove_neg_values": {"mode": "subtract_min"}}
    p = ingest.proc_from_params(prm, 64, 64)
    s1 = ingest.meas_stats(frames, p)
    s2 = ingest.meas_stats(frames, p, chunk_frames=64)
    assert torch.equal(s1[:2], s2[:2])
    torch.testing.assert_close(s1, s2, rtol=1e-14, atol=0)
    full = ingest.meas_finish(frames, p, s1)
    a, b = frames[:170], frames[170:]
    sa, sb = ingest.meas_stats(a, p), ingest.meas_stats(b, p)
    s = sa.clone()
    s[0] = torch.minimum(sa[0], sb[0])
    s[1:] = sa[1:] + sb[1:]
    two = torch.cat([ingest.meas_finish(a, p, s), ingest.meas_finish(b, p, s)])
    torch.testing.assert_close(two, full, rtol=1e-6, atol=0)
    from oracle import ingest_oracle as io
    want, _, _ = io.process_meas(frames.cpu().numpy(), prm, 1, 300)
    np.testing.assert_allclose(full.cpu().numpy(), want, rtol=2e-6, atol=1e-7)


def test_large_stack_streaming_read(dev, tmp_path):
    """A 2,048-frame 128² stack (134 MB with gaps: several 64 MiB pinned chunks) read back exactly."""
    from ptyrad_amd.ingest import load_raw
    rng = np.random.default_rng(4)
    fr = rng.standard_normal((2048, 128, 128)).astype(np.float32)
    path = str(tmp_path / "big.raw")
    write_raw(path, fr, 0, 1024)
    got = load_raw(path, fr.shape, 0, 1024, device=dev)
    assert torch.equal(got.cpu(), torch.from_numpy(fr))
    part = load_raw(path, fr.shape, 0, 1024, device=dev, first=1000, count=777)
    assert torch.equal(part.cpu(), torch.from_numpy(fr[1000:1777]))
