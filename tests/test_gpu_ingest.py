"""GPU: raw EMPAD stack → HBM → processed measurements (ptyrad_amd/ingest.py → libptyx
ptyx_raw_read / ptyx_meas_stats / ptyx_meas_finish, and for meas_pad / meas_resample
ptyx_meas_mean / ptyx_meas_pad_background / ptyx_meas_pad_resample) against the reference's
load_raw + _process_meas outputs (tests/golden/ingest_*.npz).

Tolerances.  A single-rank ingest takes the normalisation constant and meas_pad's fit input from
the reference's own f32 mean pattern (ptyx_meas_mean_seq: numpy's sequential f32 meas.mean(0),
bit for bit), so the stored stack and the fitted background match the reference to rounding of
the f64 background evaluation (rtol 1e-6).  The exactness matters: with integer detector counts
the fit's percentile mask has ties, and a one-ulp change of the mean pattern flips tied pixels
and moves the fitted (a, b) by up to 1e-2 (the pso_demo case).  The sharded path (f64 statistics
summed over ranks) is checked for rank-split invariance and against the reference at 1e-3."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from tests.test_ingest import CASES, GOLD, PAD_CASES, load_case, write_raw

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def init_params(z, proc):
    d = dict(proc)
    d.update(pos_N_scan_slow=int(z["n_slow"]), pos_N_scan_fast=int(z["n_fast"]), meas_Npix=z["frames"].shape[-1])
    return d


@pytest.mark.parametrize("name", [c for c in CASES if c not in PAD_CASES])
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
    # the reference's own f32 normalisation constant (ptyx_meas_mean_seq): within 1 ulp
    np.testing.assert_allclose(got, z["meas"], rtol=1.2e-7, atol=1e-30)
    m16, _ = ingest_raw(path, init_params(z, proc), device=dev, file_shape=z["frames"].shape,
                        offset=int(z["offset"]), gap=int(z["gap"]), out_f16=True)
    ref16 = z["meas"].astype(np.float16).astype(np.float32)
    np.testing.assert_allclose(m16.float().cpu().numpy(), ref16, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("name", PAD_CASES)
def test_ingest_pad_resample_matches_reference(name, dev, tmp_path):
    """meas_pad (five background types, precompute / on_the_fly) and meas_resample (precompute
    zoom, on-the-fly factors) through ingest_raw, against the reference's _process_meas."""
    from ptyrad_amd.ingest import ingest_raw
    z, proc = load_case(name)
    path = str(tmp_path / "scan.raw")
    write_raw(path, z["frames"], 0, 0)
    meas, info = ingest_raw(path, init_params(z, proc), device=dev, file_shape=z["frames"].shape, offset=0, gap=0)
    got = meas.cpu().numpy()
    assert got.shape == z["meas"].shape and meas.dtype == torch.float32
    assert info["meas_Npix"] == int(z["out_npix"])
    np.testing.assert_allclose(got, z["meas"], rtol=1e-6, atol=1e-30)
    pad = info["on_the_fly_meas_padded"]
    if z["otf_padded"].size:
        assert pad.shape == z["otf_padded"].shape
        np.testing.assert_allclose(pad.cpu().numpy(), z["otf_padded"], rtol=1e-9, atol=1e-30)
        assert list(info["on_the_fly_meas_padded_idx"]) == list(z["otf_padded_idx"])
        np.testing.assert_allclose(info["pad_int_sum"], z["otf_padded"].sum(), rtol=1e-9)
    else:
        assert pad is None
    sf = info["on_the_fly_meas_scale_factors"]
    assert (sf is None and not z["otf_scale_factors"].size) or list(sf) == list(z["otf_scale_factors"])
    m16, info16 = ingest_raw(path, init_params(z, proc), device=dev, file_shape=z["frames"].shape, offset=0, gap=0,
                             out_f16=True)
    assert m16.dtype == torch.float16
    np.testing.assert_allclose(m16.float().cpu().numpy(), z["meas"].astype(np.float16).astype(np.float32),
                               rtol=1e-3, atol=1e-6)


def test_pad_resample_kernel_vs_oracle_edges(dev):
    """ptyx_meas_pad_resample against the oracle's zoom restatement on shapes whose last output
    coordinate rounds past the edge (32 px × 0.5 → scipy's cval row/column), odd canvases and a
    one-pixel output axis; f16 input too."""
    from oracle import ingest_oracle as io
    from ptyrad_amd import ingest
    rng = np.random.default_rng(9)
    for (H, W), s in (((32, 32), 0.5), ((17, 40), 1.3334), ((9, 11), 3.0), ((45, 45), 0.75), ((2, 7), 0.5)):
        m = (rng.random((3, H, W)) * 4).astype(np.float32)
        want = io.zoom_order1(m, s, s)
        got = ingest.pad_resample(torch.tensor(m, device=dev), None, None, want.shape[1:]).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1.2e-7, atol=1e-30)
        got16 = ingest.pad_resample(torch.tensor(m, device=dev).half(), None, None, want.shape[1:]).cpu().numpy()
        want16 = io.zoom_order1(m.astype(np.float16).astype(np.float32), s, s)
        np.testing.assert_allclose(got16, want16, rtol=1.2e-7, atol=1e-30)


def test_pad_two_ranks_fit_the_global_mean(dev):
    """Sharded ingest with meas_pad: two 'ranks' summing their statistics fit the same background
    as one rank over the whole stack, and their padded halves concatenate to the single-rank stack."""
    from ptyrad_amd import ingest
    z, proc = load_case("pad_power_pre_f64")
    fr = torch.tensor(z["frames"], device=dev)
    ip = init_params(z, proc)
    p = ingest.proc_from_params(ip, *fr.shape[1:])
    pad = ingest.pad_config(ip)
    out_hw = z["meas"].shape[1:]
    # one rank, f64-statistics path (what each rank of a sharded ingest runs)
    s1 = ingest.meas_stats(fr, p)
    bg1, geom1, fit1 = ingest.pad_background(ingest.meas_mean(p, s1, *fr.shape[1:]), pad)
    full = ingest.pad_resample(ingest.meas_finish(fr, p, s1), bg1, geom1, out_hw)
    a, b = fr[:2], fr[2:]
    sa, sb = ingest.meas_stats(a, p), ingest.meas_stats(b, p)
    s = sa.clone()
    s[0] = torch.minimum(sa[0], sb[0])
    s[1:] = sa[1:] + sb[1:]
    bg, geom, fit = ingest.pad_background(ingest.meas_mean(p, s, *fr.shape[1:]), pad)
    assert fit == fit1 and geom == geom1      # (integer counts: the f64 sums are exact in any order)
    parts = [ingest.pad_resample(ingest.meas_finish(x, p, s), bg, geom, out_hw) for x in (a, b)]
    torch.testing.assert_close(torch.cat(parts), full, rtol=1e-6, atol=0)
    # and it agrees with the reference to the f64-statistics tolerance
    np.testing.assert_allclose(full.cpu().numpy(), z["meas"], rtol=1e-3, atol=1e-7)


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
