"""Data-parallel driver (replacement of PtyRAD's DDP wrapper) on CPU with gloo, world_size 2 to 8.

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
import torch
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
    # group 0 = batches 0,1,2 -> ranks 0,1,2; group 1 = 3,4,5; group 2 = batch 6 alone (fewer
    # mini-batches than ranks): split, rank 0 takes its first two positions, ranks 1, 2 one each
    assert np.array_equal(got[0], np.concatenate([batches[0], batches[3], batches[6][:2]]))
    assert np.array_equal(got[2], np.concatenate([batches[2], batches[5], batches[6][3:]]))
    # a loss that cannot be split (loss_pacbed): whole batches, group 2 on rank 0
    ctx = DistContext()
    ctx.rank, ctx.world = 0, 3
    assert np.array_equal(ctx.local_indices(batches, 3, split=False),
                          np.concatenate([batches[0], batches[3], batches[6]]))


def test_measurement_block_and_recon_step_share_the_split_decision():
    """the rank's DP block (local_indices) and recon_step decide the split of a group
    with fewer mini-batches than ranks the same way.  A loss that cannot be split (loss_pacbed) or
    a model stage that forces autograd (detector blur, on-the-fly measurements) gives whole
    mini-batches; a block built for the other decision is refused before any collective."""
    import os
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.reconstruction import DistContext, recon_step
    from tests.dist_helpers import OracleLoss, OracleModel
    batches = [np.arange(i * 4, i * 4 + 4) for i in range(4)]
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False}, "loss_pacbed": {"state": True, "weight": 0.5, "dp_pow": 0.2},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1}, "loss_simlar": {"state": False}}
    ctx = DistContext()
    ctx.rank, ctx.world = 1, 2
    whole = ctx.local_indices(batches, 1, loss_fn=CombinedLoss(lp, device="cpu"))
    assert ctx.block_split is False
    assert whole.size == 0                       # one mini-batch per step, unsplittable: rank 0 takes it
    assert ctx.local_indices(batches, 2, loss_fn=CombinedLoss(lp, device="cpu")).size == 8   # ga 2: one each
    lp_nopac = {**lp, "loss_pacbed": {"state": False}}
    assert ctx.local_indices(batches, 1, loss_fn=CombinedLoss(lp_nopac, device="cpu")).size == 8   # parts of all 4
    assert ctx.block_split is True
    assert not CombinedLoss(lp_nopac, device="cpu").supports_batch_split(model_params={"detector_blur_std": 1.0})
    assert not CombinedLoss(lp_nopac, device="cpu").supports_batch_split(
        init_variables={"on_the_fly_meas_scale_factors": [2.0, 2.0]})
    assert CombinedLoss(lp_nopac, device="cpu").supports_batch_split(
        model_params={"detector_blur_std": None}, init_variables={"on_the_fly_meas_scale_factors": [1.0, 1.0]})
    # a block built for split mini-batches, then a loss that cannot split: refused up front
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "traj_n64_b4_ga1.npz"), allow_pickle=False)
    zb = np.split(z["batches"], np.cumsum(z["batch_sizes"])[:-1])
    ctx = DistContext()
    ctx.rank, ctx.world = 0, 2
    mi = ctx.local_indices(zb, 1)
    model = OracleModel(z, meas_index=mi)
    opt = torch.optim.Adam(model.optimizable_params)
    with pytest.raises(ValueError, match="split_batches=True"):
        recon_step(zb, 1, model, opt, OracleLoss(lp), None, 1, verbose=False, dist_ctx=ctx)


def test_split_ranges_cut_groups_alike_on_every_rank():
    """a split group too large for one engine call is cut into mini-batch ranges from
    the whole mini-batches' sizes (rank 0's parts are the largest), identically on every rank."""
    from ptyrad_amd.reconstruction import DistContext
    group = [np.arange(10), np.arange(7), np.arange(4), np.arange(9)]
    got = []
    for r in range(3):
        ctx = DistContext()
        ctx.rank, ctx.world = r, 3
        got.append(ctx.split_ranges(group, 6))
        for a, b in got[-1]:   # every rank's share of a range fits the call
            assert sum(len(ctx.my_part(x)) for x in group[a:b]) <= 6
    assert got[0] == got[1] == got[2] == [(0, 1), (1, 3), (3, 4)]
    assert DistContext().split_ranges(group, None) == [(0, 4)]
    ctx = DistContext()
    ctx.rank, ctx.world = 2, 3
    with pytest.raises(ValueError, match="exceeds"):
        ctx.split_ranges(group, 3)


def _simulate_ranks(z, parts_of, lp):
    """forward_loss_grad_parts for every rank of an in-process 'job': pass 1 collects each rank's
    batch sums, pass 2 runs every rank with their sum (the all-reduce)."""
    from oracle import ptyx_oracle as orc
    args = (z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], z["H"], z["occu"], z["meas"])
    local = []
    for parts in parts_of:
        def grab(s):
            local.append(s.copy())
        orc.forward_loss_grad_parts(*args, parts, lp, grab)
    total = np.sum(local, axis=0)

    def put(s):
        s[...] = total
    return [orc.forward_loss_grad_parts(*args, parts, lp, put) for parts in parts_of]


@pytest.mark.parametrize("world", [2, 3, 5])
def test_oracle_split_mini_batches_equal_whole_batches(world):
    """Every mini-batch split over `world` ranks (ragged and, at world 5 > batch size 4, empty
    parts), per-batch sums all-reduced between forward and adjoint (ptyx_forward_loss_grad_begin /
    _end): the loss terms are the whole mini-batches' and the ranks' gradients sum to the
    single-device gradients (losses.py:45-47 normalisation per WHOLE mini-batch)."""
    import json
    from oracle import ptyx_oracle as orc
    from tests.test_oracle_golden import load_case
    d = load_case(os.path.join(os.path.dirname(__file__), "golden", "n32_p2o2z3_shift.npz"))   # P 2, O 2, Nz 3
    z = {"obja": d["obja"], "objp": d["objp"], "probe": d["probe"], "shifts": d["shifts"], "crop_pos": d["crop_pos"],
         "H": d["H"], "occu": d["occu"], "meas": d["meas"]}
    lp = json.loads(json.dumps(d["loss_params"]))
    for term in ("loss_single", "loss_poissn"):      # each data term (and both) with loss_sparse
        lp[term]["state"] = True
    rng = np.random.default_rng(0)
    S = z["shifts"].shape[0]
    batches = np.array_split(rng.permutation(S), max(1, S // 4))
    whole_terms, _, whole = orc.forward_loss_grad(*z.values(), batches, lp)
    parts_of = [[np.array_split(b, world)[r] for b in batches] for r in range(world)]
    res = _simulate_ranks(z, parts_of, lp)
    for terms, _ in res:
        np.testing.assert_allclose(terms, whole_terms, rtol=1e-12, atol=1e-15)
    for k in ("obja", "objp", "probe", "shifts"):
        got = sum(g[k] for _, g in res)
        np.testing.assert_allclose(got, whole[k], rtol=1e-10, atol=1e-13 * np.abs(whole[k]).max(), err_msg=k)


@pytest.mark.parametrize("world,slots", [(2, True), (3, False), (4, True), (8, True), (8, False)])
def test_ga1_split_batches_reproduce_single_rank(tmp_path, world, slots):
    """grad_accumulation = 1 (the reference default) on 3 and 8 gloo ranks: every mini-batch of 4
    is split over the ranks (2/1/1 at three; at eight, four ranks hold one position and four hold
    none but still join every collective), each rank holds only its parts' DPs (the rest NaN), and
    the trajectory equals the single-rank one (fp32 summation order) and the reference's.  slots:
    the split steps' object and position gradients by SlotExchange (all-gathered per-rank
    contributions summed in rank order on every rank; only the probe gradient and the loss terms
    all-reduced), else the flat all-reduce."""
    path = [p for p in TRAJ if "traj_n64_b4_ga1" in p][0]
    z = np.load(path, allow_pickle=False)
    single, _ = run_recon(z)
    out = str(tmp_path / "r.npz")
    mp.start_processes(dist_worker, args=(world, free_port(), path, out, {"shard": True, "slots": slots}),
                       nprocs=world, start_method="spawn")
    r = [np.load(out)] + [np.load(out.replace(".npz", f"_r{i}.npz")) for i in range(1, world)]
    for k in ("obja", "objp", "probe", "shifts"):
        assert np.all(np.isfinite(r[0][k])), k
        for i in range(1, world):
            assert np.array_equal(r[0][k], r[i][k]), f"replicas diverged in {k} (rank {i})"
        np.testing.assert_allclose(r[0][k], single[k], rtol=0, atol=2e-6)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r[0][k].astype(np.float64) - ref) ** 2))) < 1e-5


@pytest.mark.parametrize("name,start", [("traj_n32_p2_ga2", None), ("traj_n64_b4_ga1", None),
                                         ("traj_n32_p2_ga2", {"objp": 2, "probe": 2})],
                         ids=["ga2", "ga1_split", "ga2_objp_frozen_first"])
def test_band_exchange_equals_flat_allreduce(tmp_path, name, start):
    """Object gradients by row band (each rank sends only its touched rows to their owners,
    owners run Adam on their band, bands all-gathered) vs the flat all-reduce, 2 gloo ranks with
    rank-local DPs: bitwise-identical final parameters (every pixel has at most two contributors,
    and a + b = b + a), for whole-batch (ga 2) and split (ga 1) groups, and with the object phase
    frozen in the first iteration (its band optimizer state must start in iteration 2)."""
    path = [p for p in TRAJ if name in p][0]
    outs = {}
    for band in (False, True):
        out = str(tmp_path / f"b{int(band)}.npz")
        kw = {"shard": True, "band": band, **({"start_iter": start} if start else {})}
        mp.start_processes(dist_worker, args=(2, free_port(), path, out, kw), nprocs=2, start_method="spawn")
        outs[band] = (np.load(out), np.load(out.replace(".npz", "_r1.npz")))
    for k in ("obja", "objp", "probe", "shifts"):
        assert np.array_equal(outs[True][0][k], outs[True][1][k]), f"band replicas diverged in {k}"
        assert np.array_equal(outs[True][0][k], outs[False][0][k]), f"band != all-reduce in {k}"


@pytest.mark.parametrize("world", [2, 8])
def test_mismatched_ranks_refuse_instead_of_hanging(tmp_path, world):
    """A rank iterating another batching would pair mismatched collectives: recon_step's
    fingerprint all-reduce makes EVERY rank raise before the first step collective."""
    from tests.dist_helpers import mismatch_worker
    path = [p for p in TRAJ if "traj_n32_p2_ga2" in p][0]
    out = str(tmp_path / "m.npz")
    mp.start_processes(mismatch_worker, args=(world, free_port(), path, out, "batches"), nprocs=world,
                       start_method="spawn")
    for r in range(world):
        z = np.load(out.replace(".npz", f"_r{r}.npz"))
        assert int(z["ok"]) == 0 and "disagree" in str(z["msg"])


def test_graph_decision_disagreement_falls_back_to_eager(tmp_path):
    """Only rank 0 thinks its steps are graph-eligible: both ranks run eager steps (logged) and
    finish the ordinary two-rank trajectory."""
    from tests.dist_helpers import mismatch_worker
    path = [p for p in TRAJ if "traj_n32_p2_ga2" in p][0]
    z = np.load(path, allow_pickle=False)
    single, _ = run_recon(z, niter=2)
    out = str(tmp_path / "g.npz")
    mp.start_processes(mismatch_worker, args=(2, free_port(), path, out, "graphs"), nprocs=2, start_method="spawn")
    r0, r1 = (np.load(out.replace(".npz", f"_r{r}.npz")) for r in range(2))
    assert int(r0["ok"]) == 1 and int(r1["ok"]) == 1
    for k in ("obja", "objp", "probe", "shifts"):
        assert np.array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], single[k], rtol=0, atol=2e-6)


def test_agree_and_step_plan_single_process():
    """Without collectives agree() is trivially true; step_plan changes with the batching."""
    from ptyrad_amd.reconstruction import DistContext
    ctx = DistContext()
    assert ctx.agree((1, 2), ("x",)) == [True, True]
    b = [np.arange(4), np.arange(4, 8)]
    p1 = ctx.step_plan(b, 1, True, False, 100, None)
    assert p1 == ctx.step_plan([x.copy() for x in b], 1, True, False, 100, None)
    assert p1 != ctx.step_plan(b[::-1], 1, True, False, 100, None)
    assert p1 != ctx.step_plan(b, 2, True, False, 100, None)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_band_exchange_row_sharded_auto_equals_flat(tmp_path, world):
    """A row-sharded scan (each rank's mini-batches from its own scan rows, every pixel reached by
    at most two ranks): DistContext(band_exchange="auto") picks the band exchange by itself (halo rows to
    the owners, Adam on the owned band, updated rows back to their readers, no per-step
    all-gather; the whole object is synced only before the Fourier-filter constraint of the last
    iteration and at the end).  3 iterations with object constraints: every rank holds the same
    parameters; at two ranks they equal the flat all-reduce bit for bit; at three and four the
    probe / position gradients (which every rank contributes to) are all-reduced in a buffer of
    another size than the flat one, so gloo sums their three or four terms in another order: equal
    to fp32 summation order (2e-6), as is the one-rank run."""
    from tests.dist_helpers import band_worker, row_sharded_problem
    outs = {}
    for band in ("auto", False):
        out = str(tmp_path / f"b{band}.npz")
        mp.start_processes(band_worker, args=(world, free_port(), out, band), nprocs=world, start_method="spawn")
        outs[band] = [np.load(out.replace(".npz", f"_r{r}.npz")) for r in range(world)]
    single, _ = run_recon(row_sharded_problem(world))
    for r in range(world):
        assert bool(outs["auto"][r]["banded"]) and not bool(outs[False][r]["banded"])
        # halo traffic: a few window heights, far below the object's rows
        assert 0 < int(outs["auto"][r]["sent_rows"]) + int(outs["auto"][r]["halo_rows"]) <= 4 * 32
        for k in ("obja", "objp", "probe", "shifts"):
            assert np.array_equal(outs["auto"][r][k], outs["auto"][0][k]), f"band replicas diverged in {k}"
            if world == 2:
                assert np.array_equal(outs["auto"][r][k], outs[False][0][k]), f"band != all-reduce in {k}"
            else:
                np.testing.assert_allclose(outs["auto"][r][k], outs[False][0][k], rtol=0, atol=2e-6)
    for k in ("obja", "objp", "probe", "shifts"):
        np.testing.assert_allclose(outs["auto"][0][k], single[k], rtol=0, atol=2e-6)


def test_band_edges_and_auto_rule():
    """Owner edges sit in the middle of neighbouring ranks' overlaps; the auto rule takes the band
    exchange only for ranges ordered by rank that stay within a window of their bands."""
    from ptyrad_amd.reconstruction import ObjectBands
    rows = [(0, 300), (256, 556), (512, 812), (768, 1068)]          # 256-row shards, 44-row overlaps
    assert ObjectBands.band_edges(rows, 1068, 4) == [0, 278, 534, 790, 1068]
    assert ObjectBands.disjoint(rows, 1068, 4, 128)
    assert not ObjectBands.disjoint([(0, 1068)] * 4, 1068, 4, 128)          # random batches: all rows
    assert not ObjectBands.disjoint(rows[::-1], 1068, 4, 128)               # not ordered by rank
    assert ObjectBands.band_edges([(0, 10)] * 3, 30, 3) == [0, 10, 20, 30]  # (uniform fallback)
