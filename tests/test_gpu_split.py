"""Mini-batches split over data-parallel ranks (ptyx_forward_loss_grad_begin / _end), the prep
record that guards PTYX_PREP_REUSE, and RCCL (torch.distributed 'nccl') on the MI355X.

Reference: the multi-GPU path splits every mini-batch over the ranks (accelerate split_batches,
src/ptyrad/utils/common.py:63; reconstruction.py:125-132) and normalises each loss by its mini-batch
(losses.py:45-47).  Here a split call's per-batch loss sums are all-reduced between the engine's
forward and its adjoint, so the ranks' gradients sum exactly to the single-device ones.
"""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from tests.test_gpu_parity import TOL_G, TOL_G_BOTH, TOL_SH, TOL_TERMS, orc_default_loss, tensors
from tests.test_oracle_golden import rel

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def problem(N, P, O, Nz, seed, ns=3, nf=4):
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(N, ns, nf, P=P, O=O, Nz=Nz, seed=seed)
    return dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(60.0 if N == 128 else 30.0 if N == 256 else 40.0),
                shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True,
                loss_params=orc_default_loss())


def plan_for(d, device, max_patterns=64):
    """max_patterns 64: the register engines' segment slab then holds any of these calls."""
    from ptyrad_amd.engine import Plan
    O, Nz, Ny, Nx = d["obja"].shape
    P, N = d["probe"].shape[:2]
    return Plan(N, P, O, Nz, Ny, Nx, d["shifts"].shape[0], max_patterns, shift_probes=True, device=device)


def zero_grads(t):
    return {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}


def to_np(g):
    out = {k: v.cpu().numpy().astype(np.float64) for k, v in g.items()}
    out["probe"] = out["probe"][..., 0] + 1j * out["probe"][..., 1]
    return out


# geometry -> engine that serves it: k_fused3, k_fused3ms, the mixed-state register engine, the N = 256
# stripe engine, the two-pass engine
# (*_both: loss_single + loss_poissn, whose coefficients the stripe engine applies in a second k_s3,
# the mixed-state engine in k_fmm_adj and k_fused3 in its MODE 2 pass, all after k_finalize — i.e.
# in _end of a split call)
GEOMS = {"fused3": (128, 1, 1, 1), "fused3ms": (128, 1, 1, 3), "fmm": (128, 3, 1, 2), "stripe": (256, 2, 1, 1),
         "stripe_o2": (256, 2, 2, 1), "two_pass": (64, 2, 2, 2), "stripe_both": (256, 2, 1, 1),
         "stripe_o2_both": (256, 2, 2, 1), "fmm_both": (128, 3, 1, 2), "fused3_both": (128, 1, 1, 1),
         "fused3ms_both": (128, 1, 1, 3)}
ENGINE_KERNEL = {"fused3": "k_fused", "fused3ms": "k_fused", "fmm": "k_fmm_fwd", "stripe": "k_s3",
                 "stripe_o2": "k_obj_gather", "two_pass": "k_forward", "stripe_both": "k_s3",
                 "stripe_o2_both": "k_obj_gather", "fmm_both": "k_fmm_fwd", "fused3_both": "k_fused",
                 "fused3ms_both": "k_fused"}


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("geom", sorted(GEOMS))
def test_split_batches_sum_to_whole_call(geom, world):
    """Every mini-batch split over `world` simulated ranks (one plan each): the loss terms are the
    whole mini-batches' and the ranks' gradients sum to the whole call's (and the oracle's)."""
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    d = problem(*GEOMS[geom], seed=21 + world)
    if geom.endswith("_both"):
        d["loss_params"]["loss_poissn"]["state"] = True
    t = tensors(d, device)
    cfg = LossConfig.from_loss_params(d["loss_params"])
    batches = [np.array([3, 0, 9, 7, 11]), np.array([5, 1, 10, 2]), np.array([4, 8, 6])]
    whole = zero_grads(t)
    plan = plan_for(d, device)
    plan.profile_begin()
    wterms = plan.forward_loss_grad(t, np.concatenate(batches), batch_offsets(batches), cfg, whole)
    ks = plan.profile_end()
    assert ENGINE_KERNEL[geom] in ks, ks                          # the intended engine ran
    parts_of = [[np.array_split(b, world)[r] for b in batches] for r in range(world)]
    plans = [plan_for(d, device) for _ in range(world)]

    def run(r, reduce):
        parts = [p for p in parts_of[r] if p.size]
        g = zero_grads(t)
        terms = plans[r].forward_loss_grad(t, np.concatenate(parts), batch_offsets(parts), cfg, g,
                                           batch_sums_reduce=reduce)
        return terms, g

    local = []
    for r in range(world):                         # pass 1: each rank's sums (what the all-reduce sums)
        run(r, lambda s: local.append(s.clone()))
    total = torch.stack(local).sum(0)
    res = [run(r, lambda s: s.copy_(total)) for r in range(world)]   # pass 2: with the summed sums
    torch.cuda.synchronize()
    for terms, _ in res:
        np.testing.assert_allclose(terms.cpu().numpy(), wterms.cpu().numpy(), rtol=2e-6, atol=1e-9)
    got = {k: sum(to_np(g)[k] for _, g in res) for k in whole}
    ref = to_np(whole)
    for k in ("obja", "objp", "probe"):
        assert rel(got[k], ref[k]) < 2e-6, k
    assert rel(got["shifts"], ref["shifts"]) < 2e-5
    oterms, _, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                          d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(res[0][0].cpu().numpy(), oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        tol = TOL_G_BOTH if (k == "probe" and geom.endswith("_both")) else TOL_G
        assert rel(got[k], og[k]) < tol, k
    assert rel(got["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("geom", ["fused3", "fused3ms", "fmm", "stripe", "stripe_o2", "two_pass"])
def test_grad_store_overwrites_the_object_gradient(geom):
    """PTYX_PREP_GRAD_STORE (ABI 208): the call overwrites d_obja / d_objp with its own gradient —
    whatever they held before — and accumulates the probe / position gradients as usual.  Every
    engine (the register engines' gathers store, including the tiles no window reaches; the others
    clear the arrays first): bitwise the accumulate-into-zeros call; and, split over two calls at
    mini-batch boundaries (the Plan's pieces), only the first piece stores."""
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    d = problem(*GEOMS[geom], seed=31)
    t = tensors(d, device)
    cfg = LossConfig.from_loss_params(d["loss_params"])
    batches = [np.array([3, 0, 9, 7, 11]), np.array([5, 1, 10, 2]), np.array([4, 8, 6])]
    idx, off = np.concatenate(batches), batch_offsets(batches)
    plan = plan_for(d, device)
    ref = zero_grads(t)
    plan.forward_loss_grad(t, idx, off, cfg, ref)
    got = zero_grads(t)
    for k in ("obja", "objp"):
        got[k].fill_(123.0)                    # stale values: must not survive
    got["probe"].copy_(ref["probe"])           # these accumulate: start from a known value
    got["shifts"].copy_(ref["shifts"])
    plan.forward_loss_grad(t, idx, off, cfg, got, prep=_lib.PTYX_PREP_GRAD_STORE)
    torch.cuda.synchronize()
    atomics = geom in ("stripe", "two_pass")     # f32 object atomics: last bits follow arrival order
    for k in ("obja", "objp"):
        if atomics:
            assert rel(got[k].cpu().numpy(), ref[k].cpu().numpy()) < 1e-6, k
        else:
            assert torch.equal(got[k], ref[k]), k
    for k in ("probe", "shifts"):
        assert torch.equal(got[k], 2 * ref[k]) or rel(got[k].cpu().numpy(), 2 * ref[k].cpu().numpy()) < 1e-6, k
    # pieces: a plan whose capacity splits the call; the first piece stores, the second accumulates
    small = plan_for(d, device, max_patterns=9)
    pc = zero_grads(t)
    small.forward_loss_grad(t, idx, off, cfg, pc)
    ps = zero_grads(t)
    for k in ("obja", "objp"):
        ps[k].fill_(-7.0)
    small.forward_loss_grad(t, idx, off, cfg, ps, prep=_lib.PTYX_PREP_GRAD_STORE)
    torch.cuda.synchronize()
    for k in ("obja", "objp"):
        assert rel(ps[k].cpu().numpy(), pc[k].cpu().numpy()) < 1e-6, k


def test_plan_refuses_work_between_begin_and_end():
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    d = problem(64, 1, 1, 1, seed=3)
    t = tensors(d, device)
    plan = plan_for(d, device)
    cfg = LossConfig.from_loss_params(d["loss_params"])
    b = [np.array([0, 1, 2])]

    def reduce(_s):   # while the call is open, the plan takes no other compute call
        with pytest.raises(_lib.PtyxError, match="waiting for its _end"):
            plan.forward_loss_grad(t, np.array([4, 5]), batch_offsets([np.array([4, 5])]), cfg, zero_grads(t))
    plan.forward_loss_grad(t, b[0], batch_offsets(b), cfg, zero_grads(t), batch_sums_reduce=reduce)
    plan.forward_loss_grad(t, b[0], batch_offsets(b), cfg, zero_grads(t))     # closed again
    torch.cuda.synchronize()


def test_prep_reuse_after_engine_change_prepares_in_full():
    """a call split into pieces at the plan capacity whose first piece runs the
    two-pass engine (64 one-pattern mini-batches: more segments than k_fused3's slab holds) and
    whose second piece runs k_fused3 (two mini-batches of 32).  The second piece asks for
    PTYX_PREP_REUSE, but k_fused3's object / probe preparation was never made: the plan's prep
    record makes it prepare in full.  Loss terms and gradients match the oracle."""
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    pr = syn.random_problem(128, 8, 16, seed=17)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(60.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=orc_default_loss())
    t = tensors(d, device)
    plan = plan_for(d, device, max_patterns=64)
    batches = [np.array([i]) for i in range(64)] + [np.arange(64, 96), np.arange(96, 128)]
    g = zero_grads(t)
    plan.profile_begin()
    terms = plan.forward_loss_grad(t, np.concatenate(batches), batch_offsets(batches),
                                   LossConfig.from_loss_params(d["loss_params"]), g)
    ks = plan.profile_end()
    assert "k_forward" in ks and "k_fused" in ks, ks           # both engines ran, one piece each
    oterms, _, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                          d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(terms.cpu().numpy(), oterms, rtol=TOL_TERMS, atol=1e-7)
    gn = to_np(g)
    for k in ("obja", "objp", "probe"):
        assert rel(gn[k], og[k]) < TOL_G, k
    assert rel(gn["shifts"], og["shifts"]) < TOL_SH


def test_meas_rows_outside_the_block_is_refused():
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    d = problem(64, 1, 1, 1, seed=4)
    t = tensors(d, device)
    rows = torch.full((d["shifts"].shape[0],), -1, dtype=torch.int32, device=device)
    rows[:4] = torch.arange(4, dtype=torch.int32, device=device)
    t["meas"] = t["meas"][:4].contiguous()
    t["meas_rows"] = rows
    plan = plan_for(d, device)
    cfg = LossConfig.from_loss_params(d["loss_params"])
    plan.forward_loss_grad(t, np.array([0, 3]), batch_offsets([np.array([0, 3])]), cfg, zero_grads(t))
    plan.check()
    # the device flags the bad row (no host sync in the call); the plan reports it afterwards
    plan.forward_loss_grad(t, np.array([1, 6]), batch_offsets([np.array([1, 6])]), cfg, zero_grads(t))
    with pytest.raises(IndexError, match="meas_rows"):
        plan.check()
    plan.check()   # reported once, then clear


# ------------------------------------------------------------------ RCCL on the MI355X
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _nccl_worker(rank, port, path, out, split, band=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from ptyrad_amd.reconstruction import DistContext
        from tests.dist_helpers import gpu_recon
        assert torch.distributed.get_backend() == "nccl"
        z = np.load(path, allow_pickle=False)
        ctx = DistContext(split_batches=split, always_reduce=True, band_exchange=band)
        model = gpu_recon(z, ctx, shard=True)
        np.savez(out, obja=model.opt_obja.detach().cpu().numpy(), objp=model.opt_objp.detach().cpu().numpy(),
                 backend=np.array(torch.distributed.get_backend()))
    finally:
        torch.distributed.destroy_process_group()


def _nccl_graph_worker(rank, port, path, out, split):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from ptyrad_amd.reconstruction import DistContext
        from tests.dist_helpers import gpu_recon
        z = np.load(path, allow_pickle=False)
        res = {}
        for graphs in (False, True):
            ctx = DistContext(split_batches=split, always_reduce=True)
            model, _, _, _, last = gpu_recon(z, ctx, shard=True, graphs=graphs, ret_all=True)
            sg = getattr(model, "_step_graphs", None)
            tag = "g" if graphs else "e"
            res.update({f"{tag}_obja": model.opt_obja.detach().cpu().numpy(),
                        f"{tag}_objp": model.opt_objp.detach().cpu().numpy(),
                        f"{tag}_probe": model.opt_probe.detach().cpu().numpy(),
                        f"{tag}_terms": np.array([np.asarray(v) for v in last.values()]),
                        f"{tag}_replays": np.array(sg.replays if sg else 0)})
        np.savez(out, **res)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("split", [True, False], ids=["split_batches", "whole_batches"])
def test_recon_step_graphs_with_rccl_collectives_match_eager_and_reference(tmp_path, split):
    """recon_step's optimizer steps replayed from hipGraphs WITH their RCCL
    collectives captured (init_process_group('nccl'), always_reduce at world size 1: the split
    step's loss-sum all-reduce between the engine halves, and the gradient all-reduce that now also
    carries the loss terms).  On the deterministic register engine (traj_c1_n128, k_fused3) the
    trajectory and loss terms are BITWISE the eager ones, and the final object matches the
    reference's (RMS < 1e-5)."""
    dev()
    import torch.multiprocessing as mp
    path = os.path.join(GOLDEN, "traj_c1_n128.npz")
    out = str(tmp_path / "nccl_graph.npz")
    mp.start_processes(_nccl_graph_worker, args=(_free_port(), path, out, split), nprocs=1, start_method="spawn")
    r = np.load(out)
    assert int(r["g_replays"]) >= 1, int(r["g_replays"])
    for k in ("obja", "objp", "probe", "terms"):
        assert np.array_equal(r["e_" + k], r["g_" + k]), k
    z = np.load(path, allow_pickle=False)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r["g_" + k].astype(np.float64) - ref) ** 2))) < 1e-5, k


@pytest.mark.parametrize("split,band", [(True, False), (False, False), (False, True)],
                         ids=["split_batches", "whole_batches", "band_exchange"])
def test_recon_step_under_rccl_matches_reference(tmp_path, split, band):
    """recon_step under init_process_group('nccl') (RCCL) on the MI355X, with every collective of the
    data-parallel path executed (always_reduce at world size 1): the loss-sum all-reduce of split
    mini-batches, the flat gradient all-reduce and the loss-term gather.  The reference
    trajectory (grad_accumulation = 1) is reproduced: final object RMS < 1e-5.  band_exchange: the
    object optimizer steps run on band views (ObjectBands) and the bands are all-gathered."""
    dev()
    import torch.multiprocessing as mp
    path = os.path.join(GOLDEN, "traj_n64_b4_ga1.npz")
    out = str(tmp_path / "nccl.npz")
    mp.start_processes(_nccl_worker, args=(_free_port(), path, out, split, band), nprocs=1, start_method="spawn")
    r = np.load(out)
    assert str(r["backend"]) == "nccl"
    z = np.load(path, allow_pickle=False)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r[k].astype(np.float64) - ref) ** 2))) < 1e-5, k


def _nccl_slot_worker(rank, port, path, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from ptyrad_amd.reconstruction import DistContext
        from tests.dist_helpers import gpu_recon
        z = np.load(path, allow_pickle=False)
        from ptyrad_amd.stepgraph import StepGraphs
        res = {}
        # (slots, graphs, the slot gather taking the optimizer step: ptyx_obj_gather_slots_adam)
        for slots, graphs, fuse in ((False, False, True), (False, True, True), (True, False, True),
                                    (True, True, True), (True, True, False)):
            StepGraphs.FUSE_ADAM = fuse
            try:
                ctx = DistContext(split_batches=True, always_reduce=True, slot_exchange=slots)
                model, _, _, _, last = gpu_recon(z, ctx, shard=True, graphs=graphs, ret_all=True)
            finally:
                StepGraphs.FUSE_ADAM = True
            tag = f"{'s' if slots else 'f'}{'g' if graphs else 'e'}{'' if fuse else 'n'}"
            res.update({f"{tag}_obja": model.opt_obja.detach().cpu().numpy(),
                        f"{tag}_objp": model.opt_objp.detach().cpu().numpy(),
                        f"{tag}_probe": model.opt_probe.detach().cpu().numpy(),
                        f"{tag}_shifts": model.opt_probe_pos_shifts.detach().cpu().numpy(),
                        f"{tag}_terms": np.array([np.asarray(v) for v in last.values()]),
                        f"{tag}_bufs": np.array(len(ctx._slot_bufs))})
        np.savez(out, **res)
    finally:
        torch.distributed.destroy_process_group()


def test_slot_exchange_under_rccl_equals_flat_allreduce(tmp_path):
    """a split step's object gradient from all-gathered per-pattern slots
    (ptyx_forward_loss_grad_begin / _end with PTYX_PREP_DEFER_GATHER, ptyx_slots_export, RCCL
    all-gather, ptyx_obj_gather_slots) and its position-gradient rows exchanged the same way; only
    the probe gradient and the loss terms all-reduced.  At world size 1 under RCCL (always_reduce)
    the slot gather runs over the very patterns, in the very order, the engine's own gather takes:
    the trajectory is BITWISE the flat all-reduce's, eager and graph-replayed (the all-gathers
    captured; the graph steps' slot gather taking the optimizer step, ptyx_obj_gather_slots_adam,
    or not), and matches the reference's (RMS < 1e-5)."""
    dev()
    import torch.multiprocessing as mp
    path = os.path.join(GOLDEN, "traj_c1_n128.npz")
    out = str(tmp_path / "slots.npz")
    mp.start_processes(_nccl_slot_worker, args=(_free_port(), path, out), nprocs=1, start_method="spawn")
    r = np.load(out)
    assert int(r["sg_bufs"]) >= 1 and int(r["fe_bufs"]) == 0          # the exchange really ran (and only there)
    for tag in ("se", "sg", "sgn", "fg"):
        for k in ("obja", "objp", "probe", "shifts", "terms"):
            assert np.array_equal(r["fe_" + k], r[f"{tag}_" + k]), (tag, k)
    z = np.load(path, allow_pickle=False)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r["sg_" + k].astype(np.float64) - ref) ** 2))) < 1e-5, k


@pytest.mark.parametrize("slots", [True, False], ids=["slot_exchange", "flat_allreduce"])
def test_two_gloo_ranks_split_steps_on_one_gpu(tmp_path, slots):
    """Two gloo ranks sharing cuda:0, the reference's default cadence (grad_accumulation = 1) with
    every 32-pattern mini-batch split 16 / 16 (k_fused3), each rank holding only its parts' DPs:
    with the slot exchange (all-gathered slots, each rank gathers the whole object gradient) and
    with the flat all-reduce, the two replicas are bitwise equal and the final object is the
    reference's (RMS < 1e-5)."""
    dev()
    import torch.multiprocessing as mp
    from tests.dist_helpers import gpu_dist_worker
    path = os.path.join(GOLDEN, "traj_c1_n128.npz")
    z = np.load(path, allow_pickle=False)
    out = str(tmp_path / "r.npz")
    mp.start_processes(gpu_dist_worker, args=(2, _free_port(), path, out,
                                              {"split_batches": True, "slot_exchange": slots}),
                       nprocs=2, start_method="spawn")
    r0, r1 = np.load(out.replace(".npz", "_r0.npz")), np.load(out.replace(".npz", "_r1.npz"))
    assert int(r0["held"]) + int(r1["held"]) == z["batches"].size
    for k in ("obja", "objp", "probe"):
        assert np.array_equal(r0[k], r1[k]), k
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r0[k].astype(np.float64) - ref) ** 2))) < 1e-5, k


# (engine geometry, bad input): every engine flags out-of-range indices, windows and meas rows on the
# device and the C ABI reports PTYX_EINVAL at the next call instead of reading out of bounds
BAD = [("fused3", "idx"), ("fused3", "crop"), ("fused3ms", "crop"), ("fmm", "idx"), ("stripe", "crop"),
       ("stripe", "rows"), ("two_pass", "crop"), ("two_pass", "rows"), ("fused3", "rows")]


@pytest.mark.parametrize("geom,bad", BAD, ids=[f"{g}-{b}" for g, b in BAD])
def test_invalid_inputs_are_reported_through_the_c_abi(geom, bad):
    """VERDICT r03 item 5 (models.py:261-264 raises IndexError): a scan index outside [0, n_scans),
    a window crop_pos + N outside the object or a meas_rows entry outside the block, passed straight
    through the C ABI, is clamped by the kernels (no fault), flagged on the device, and returned as
    PTYX_EINVAL by the plan's next call / ptyx_plan_check; a valid call afterwards runs normally."""
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import LossConfig, batch_offsets
    device = dev()
    d = problem(*GEOMS[geom], seed=33)
    t = tensors(d, device)
    S = d["shifts"].shape[0]
    plan = plan_for(d, device)
    cfg = LossConfig.from_loss_params(d["loss_params"])
    good = [np.array([0, 1, 2, 3])]
    idx = np.array([0, 1, 2, 3], np.int32)
    if bad == "idx":
        idx = np.array([0, 1, S + 5, 3], np.int32)
    elif bad == "crop":
        cp = t["crop_pos"].clone()
        cp[2, 1] = int(d["obja"].shape[-1]) - 3          # window runs past the right edge
        cp[1, 0] = -7
        t["crop_pos"] = cp
    else:
        rows = torch.arange(S, dtype=torch.int32, device=device)
        rows[2] = S + 100                                 # outside the block
        t["meas_rows"] = rows
    g = zero_grads(t)
    plan.forward_loss_grad(t, idx, batch_offsets([idx]), cfg, g)   # returns: the check is on the device
    torch.cuda.synchronize()
    lib = _lib.load()
    assert lib.ptyx_plan_check(plan._h) == _lib.PTYX_EINVAL
    msg = lib.ptyx_last_error().decode()
    assert {"idx": "scan index", "crop": "window", "rows": "meas_rows"}[bad] in msg, msg
    assert lib.ptyx_plan_check(plan._h) == 0                       # reported once
    for v in g.values():                                          # clamped, not out of bounds
        assert bool(torch.isfinite(v).all())
    if bad == "crop":
        t["crop_pos"] = tensors(d, device)["crop_pos"]
    t.pop("meas_rows", None)
    plan.forward_loss_grad(t, good[0], batch_offsets(good), cfg, zero_grads(t))
    plan.check()
    # an error of one call surfaces as IndexError at the next call through the Python mirror
    plan.forward_loss_grad(t, np.array([0, S + 1], np.int32), batch_offsets([np.array([0, 1])]), cfg, zero_grads(t))
    torch.cuda.synchronize()
    with pytest.raises(IndexError, match="scan index"):
        plan.forward_loss_grad(t, good[0], batch_offsets(good), cfg, zero_grads(t))


def _nccl_chunk_worker(rank, port, path, out, split):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from ptyrad_amd.reconstruction import DistContext
        from ptyrad_amd.stepgraph import StepGraphs
        from tests.dist_helpers import gpu_recon
        z = dict(np.load(path, allow_pickle=False))
        z["batch_sizes"] = np.full(8, z["batches"].size // 8)     # 8 steps of one shape an iteration
        res = {}
        for tag, graphs, chunk in (("e", False, 1), ("g1", True, 1), ("g3", True, 3)):
            StepGraphs.CHUNK = chunk
            try:
                ctx = DistContext(split_batches=split, always_reduce=True, slot_exchange=split)
                model, _, _, _, last = gpu_recon(z, ctx, shard=True, graphs=graphs, ret_all=True, niter=3)
            finally:
                StepGraphs.CHUNK = 16
            sg = getattr(model, "_step_graphs", None)
            res.update({f"{tag}_obja": model.opt_obja.detach().cpu().numpy(),
                        f"{tag}_objp": model.opt_objp.detach().cpu().numpy(),
                        f"{tag}_probe": model.opt_probe.detach().cpu().numpy(),
                        f"{tag}_shifts": model.opt_probe_pos_shifts.detach().cpu().numpy(),
                        f"{tag}_terms": np.array([np.asarray(v) for v in last.values()]),
                        f"{tag}_chunks": np.array(sum(1 for k in (sg.graphs if sg else {}) if k[0] == "chunk"))})
        np.savez(out, **res)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("split", [True, False], ids=["split_slots", "whole_batches"])
def test_chunked_step_graphs_with_rccl_collectives_bitwise_eager(tmp_path, split):
    """StepGraphs.CHUNK with the collectives captured (RCCL at world size 1, every collective
    forced): 8 same-shape steps an iteration replayed as graphs of 3 step bodies (plus one-step
    graphs for the remainder) — with split mini-batches, each body holds its loss-sum all-reduce,
    the slot all-gather and the fused slot gather; with whole ones, the gradient all-reduce.
    Bitwise the eager trajectory and the one-step graphs' after three iterations."""
    dev()
    import torch.multiprocessing as mp
    path = os.path.join(GOLDEN, "traj_c1_n128.npz")
    out = str(tmp_path / "nccl_chunk.npz")
    mp.start_processes(_nccl_chunk_worker, args=(_free_port(), path, out, split), nprocs=1, start_method="spawn")
    r = np.load(out)
    assert int(r["g3_chunks"]) >= 1, int(r["g3_chunks"])
    for tag in ("g1", "g3"):
        for k in ("obja", "objp", "probe", "shifts", "terms"):
            assert np.array_equal(r["e_" + k], r[f"{tag}_" + k]), (tag, k)
