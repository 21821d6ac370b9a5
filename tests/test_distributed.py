"""Data-parallel driver (replacement of PtyRAD's DDP wrapper) on CPU with gloo, world_size 2.

The mini-batches of every optimizer step are dealt round-robin to the ranks, gradients are summed
by ONE all-reduce, and every rank takes the same Adam step.  Expected: identical replicas, and
the same trajectory as one rank (up to fp32 summation order) — which itself matches the reference
(tests/test_oracle_golden.py trajectory test).
"""
import glob
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.dist_helpers import dist_worker, run_recon

TRAJ = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "traj_*.npz")))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("path", TRAJ, ids=[os.path.basename(p)[:-4] for p in TRAJ])
def test_two_rank_gloo_matches_single_rank_and_reference(path, tmp_path):
    z = np.load(path, allow_pickle=False)
    single, _ = run_recon(z)
    out = str(tmp_path / "r.npz")
    mp.start_processes(dist_worker, args=(2, free_port(), path, out), nprocs=2, start_method="spawn")
    r0 = np.load(out)
    r1 = np.load(out.replace(".npz", "_r1.npz"))
    for k in ("obja", "objp", "probe", "shifts"):
        assert np.array_equal(r0[k], r1[k]), f"replicas diverged in {k}"          # bitwise replicas
        np.testing.assert_allclose(r0[k], single[k], rtol=0, atol=2e-6)
    # and the reference's own final object (north_star: object RMS error < 1e-5)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r0[k].astype(np.float64) - ref) ** 2))) < 1e-5


def test_two_rank_staggered_start_iter_and_sharded_measurements(tmp_path):
    """probe_pos_shifts frozen for iterations 1-2 (start_iter 3): its .grad must stay None on every
    rank (Adam's step count must not advance), so the 2-rank run equals the 1-rank run; and each rank
    holds only the DPs of its own mini-batches (the rest are NaN: touching one would poison it)."""
    path = [p for p in TRAJ if "traj_n32_p2_ga2" in p][0]
    z = np.load(path, allow_pickle=False)
    kw = {"niter": 5, "start_iter": {"probe_pos_shifts": 3, "probe": 2}}
    single, _ = run_recon(z, **kw)
    out = str(tmp_path / "r.npz")
    mp.start_processes(dist_worker, args=(2, free_port(), path, out, {**kw, "shard": True}), nprocs=2,
                       start_method="spawn")
    r0 = np.load(out)
    r1 = np.load(out.replace(".npz", "_r1.npz"))
    for k in ("obja", "objp", "probe", "shifts"):
        assert np.all(np.isfinite(r0[k])), k
        assert np.array_equal(r0[k], r1[k]), f"replicas diverged in {k}"
        np.testing.assert_allclose(r0[k], single[k], rtol=0, atol=2e-6)
    # the frozen iterations really were frozen: shifts moved only in iterations 3-5
    assert not np.array_equal(single["shifts"], z["init_shifts"])


def test_local_indices_cover_each_rank_exactly():
    from ptyrad_amd.reconstruction import DistContext
    batches = [np.arange(i * 4, i * 4 + 4) for i in range(7)]
    got = []
    for r in range(3):
        ctx = DistContext()
        ctx.rank, ctx.world = r, 3
        got.append(ctx.local_indices(batches, grad_accumulation=3))
    allidx = np.sort(np.concatenate(got))
    assert np.array_equal(allidx, np.arange(28))
    # group 0 = batches 0,1,2 -> ranks 0,1,2; group 1 = 3,4,5; group 2 = batch 6 -> rank 0
    assert np.array_equal(got[0], np.concatenate([batches[0], batches[3], batches[6]]))
