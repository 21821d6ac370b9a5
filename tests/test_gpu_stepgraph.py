"""recon_step with its optimizer steps replayed from hipGraphs (ptyrad_amd/stepgraph.py) on MI355X.

The graph replays the eager step's kernels with the same arguments, so on the deterministic
register engine (k_fused3: slots + gather, fixed-order reductions) the trajectory is BITWISE the
eager one; on the general engine (f32 object atomics) it agrees to fp32 summation order.  Both
match the reference's own trajectories (tests/golden/traj_*.npz, made by running PtyRAD).
"""
import os

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN
from tests.test_oracle_golden import rel

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _params(model):
    return {k: getattr(model, k).detach().cpu().numpy() for k in
            ("opt_obja", "opt_objp", "opt_probe", "opt_probe_pos_shifts")}


@pytest.mark.parametrize("name,bitwise", [("traj_c1_n128", True), ("traj_n64_b4_ga1", False),
                                          ("traj_n32_p2_ga2", False)])
def test_graph_replayed_trajectory_equals_eager_and_reference(name, bitwise):
    need_gpu()
    from tests.dist_helpers import gpu_recon
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    eager, _, _, _, last_e = gpu_recon(z, graphs=False, ret_all=True)
    graph, _, _, _, last_g = gpu_recon(z, graphs=True, ret_all=True)
    sg = graph._step_graphs
    assert sg.captures >= 1 and sg.replays >= 1, (sg.captures, sg.replays, sg.eager)
    pe, pg = _params(eager), _params(graph)
    for k in pe:
        if bitwise:
            assert np.array_equal(pe[k], pg[k]), k
        else:
            assert rel(pg[k], pe[k]) < 1e-5, k
    for k in last_e:
        np.testing.assert_allclose(last_g[k], last_e[k], rtol=1e-5, atol=1e-7)
    for k, ref in (("opt_obja", z["final_obja"]), ("opt_objp", z["final_objp"])):
        got = pg[k].astype(np.float64)
        assert float(np.sqrt(np.mean((got - ref) ** 2))) < 1e-5, k


def test_graphs_c2_like_ragged_batches_frozen_probe_then_live():
    """32×32 raster at N = 128 (k_fused3), 31 mini-batches of 33 / 34 (two step shapes), the probe
    frozen in iteration 1 (start_iter 2) and trainable from iteration 2 (a new live set: fresh Adam
    state, a new capture).  Three iterations, graphs vs eager: bitwise equal."""
    need_gpu()
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from ptyrad_amd.reconstruction import create_optimizer, recon_step
    dev = torch.device("cuda", 0)
    N, S = 128, 32
    scan = syn.raster_scan(S, S, N, seed=0)
    n = S * S
    Ny, Nx = scan.obj_shape
    rng = np.random.default_rng(11)
    meas = rng.random((n, N, N)).astype(np.float32)
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
          "loss_pacbed": {"state": False}, "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
          "loss_simlar": {"state": False}}
    batches = np.array_split(np.random.default_rng(3).permutation(n), 31)
    starts = {"obja": 1, "objp": 1, "probe": 2, "probe_pos_shifts": 1, "obj_tilts": None, "slice_thickness": None}
    lrs = {"obja": 5e-4, "objp": 5e-4, "probe": 1e-4, "probe_pos_shifts": 1e-4, "obj_tilts": 0.0,
           "slice_thickness": 0.0}

    def run(graphs):
        iv = {"obja": np.ones((1, 1, Ny, Nx), np.float32),
              "objp": (1e-3 * np.random.default_rng(5).random((1, 1, Ny, Nx))).astype(np.float32), "obj": None,
              "probe": (syn.stem_probe(N) * np.float32(60.0))[None], "probe_pos_shifts": scan.shifts,
              "omode_occu": np.ones(1, np.float32), "H": syn.fresnel_propagator(N, syn.DX_ANG, 2.0),
              "measurements": meas, "crop_pos": scan.crop_pos, "N_scan_slow": S, "N_scan_fast": S,
              "slice_thickness": 2.0, "dx": syn.DX_ANG, "dk": 1.0 / (N * syn.DX_ANG),
              "lambd": syn.electron_wavelength(syn.KV), "obj_tilts": np.zeros((1, 2), np.float32)}
        mp = {"detector_blur_std": None, "obj_preblur_std": None,
              "update_params": {k: {"start_iter": starts[k], "lr": v} for k, v in lrs.items()},
              "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}
        model = PtychoHIP(iv, mp, device=dev, verbose=False)
        opt = create_optimizer(model.optimizer_params, model.optimizable_params)
        loss_fn = CombinedLoss(lp, device=dev)
        hist = [recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
                for it in (1, 2, 3)]
        return model, opt, hist

    me, oe, he = run(False)
    mg, og, hg = run(True)
    sg = mg._step_graphs
    assert sg.captures >= 2 and sg.replays > 80, (sg.captures, sg.replays, sg.eager)   # one capture per live set
    pe, pg = _params(me), _params(mg)
    for k in pe:
        assert np.array_equal(pe[k], pg[k]), k
    assert not np.array_equal(pe["opt_probe"], (syn.stem_probe(N) * np.float32(60.0))[None].view(np.float32)
                              .reshape(pe["opt_probe"].shape))
    for a, b in zip(he, hg):
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    # optimizer state (step counts, moments) identical too: a checkpoint taken after either is the same
    for p_e, p_g in zip([p for g in oe.param_groups for p in g["params"]],
                        [p for g in og.param_groups for p in g["params"]]):
        se, sgs = oe.state.get(p_e, {}), og.state.get(p_g, {})
        assert se.keys() == sgs.keys()
        for k in se:
            assert torch.equal(se[k].cpu(), sgs[k].cpu()), k
    assert all(not g["capturable"] for g in og.param_groups)


def test_graphs_refused_with_reason_when_ineligible():
    need_gpu()
    from tests.dist_helpers import gpu_recon
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    from ptyrad_amd.reconstruction import recon_step
    model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
    sgd = torch.optim.SGD(model.optimizable_params, lr=1e-4)
    with pytest.raises(RuntimeError, match="optimizer is not"):
        recon_step(batches, 1, model, sgd, loss_fn, None, 1, verbose=False, graphs=True)


def test_graphs_follow_an_optimizer_state_reload():
    """A checkpoint resume replaces the optimizer's state tensors (load_state_dict): the captured
    steps bake in their addresses, so the graphs must be re-captured, not replayed onto the old
    state.  Reload between iterations 1 and 2, graphs vs eager: bitwise equal."""
    need_gpu()
    import copy
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.reconstruction import recon_step
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    out = []
    for graphs in (False, True):
        model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
        for it in (1, 2, 3):
            recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
            opt.load_state_dict(copy.deepcopy(opt.state_dict()))   # fresh state tensors, same values
        out.append(_params(model))
    for k in out[0]:
        assert np.array_equal(out[0][k], out[1][k]), k


def test_graphs_follow_hyperparameters_and_reuse_reshuffled_tables():
    """a captured step bakes in Adam's betas / eps / weight_decay and the loss
    configuration besides the learning rate; changing any of them between iterations makes a new
    capture (the trajectory stays bitwise the eager one), while reshuffled mini-batches of the same
    shapes (hypertune, reconstruction.py:1059) are copied into the persistent index tables and
    replay the existing graphs without a new capture."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.reconstruction import recon_step
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    out, caps = [], []
    for graphs in (False, True):
        model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
        recon_step(batches, 1, model, opt, loss_fn, None, 1, verbose=False, graphs=graphs)
        for g in opt.param_groups:
            g["betas"] = (0.8, 0.99)
            g["eps"] = 1e-7
        recon_step(batches, 1, model, opt, loss_fn, None, 2, verbose=False, graphs=graphs)
        loss_fn.loss_params["loss_sparse"]["weight"] = 0.2
        recon_step(batches, 1, model, opt, loss_fn, None, 3, verbose=False, graphs=graphs)
        out.append(_params(model))
        if graphs:
            sg = model._step_graphs
            caps.append(sg.captures)
            flat = np.concatenate(batches)
            perm = np.random.default_rng(7).permutation(flat.size)
            shuffled = np.split(flat[perm], np.cumsum([len(b) for b in batches])[:-1])
            recon_step(shuffled, 1, model, opt, loss_fn, None, 4, verbose=False, graphs=True)
            caps.append(sg.captures)
    for k in out[0]:
        assert np.array_equal(out[0][k], out[1][k]), k
    # iteration 1 (two steps) runs both eagerly: its first step creates the Adam state, so the
    # second has a new key; iterations 2 and 3 each capture once for their new betas / loss weight
    assert caps[0] >= 2, caps
    assert caps[1] == caps[0], caps      # reshuffled batches: same graphs


def test_graphs_two_beta_groups_and_a_failed_step_keep_adam_state():
    """ptyx_step_select advances the HIP Adam's step counts before the engine call and
    the update; an eager step that raises in between (here the optimizer itself) must take them
    back.  Param groups with different betas (several Adam launches a step), a step that raises
    at iteration 3, then the iterations rerun: graphs vs eager, parameters AND optimizer state
    (step counts, moments) bitwise equal."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.reconstruction import recon_step
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    out = []
    for graphs in (False, True):
        model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
        opt.param_groups[0]["betas"] = (0.85, 0.995)           # two Adam batches a step
        for it in (1, 2):
            recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
        plist = [p for g in opt.param_groups for p in g["params"]]
        before = [opt.state[p]["step"].clone() for p in plist if p in opt.state]
        opt.param_groups[-1]["eps"] = 1e-7                      # a new step key: the next step runs eagerly

        def boom(*a, **k):
            raise RuntimeError("injected optimizer failure")
        opt.step = boom
        with pytest.raises(RuntimeError, match="injected"):
            recon_step(batches, 1, model, opt, loss_fn, None, 3, verbose=False, graphs=graphs)
        del opt.step
        after = [opt.state[p]["step"].clone() for p in plist if p in opt.state]
        assert len(before) == len(after) > 0
        for b, a in zip(before, after):
            assert torch.equal(b, a), (b, a)                    # no step count moved without an update
        for it in (3, 4):
            recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
        st = [{k: v.detach().cpu().clone() for k, v in opt.state[p].items()} for p in plist if p in opt.state]
        out.append((_params(model), st))
        if graphs:
            assert model._step_graphs.replays > 0
    for k in out[0][0]:
        assert np.array_equal(out[0][0][k], out[1][0][k]), k
    for se, sg_ in zip(out[0][1], out[1][1]):
        assert se.keys() == sg_.keys()
        for k in se:
            assert torch.equal(se[k], sg_[k]), k


def _one_step(model, opt, loss_fn, idx, mode, store):
    """One optimizer step of the mini-batch idx through the engine call: 'off' = the call, then the
    HIP Adam; 'fast' / 'fallback' = the call with PTYX_PREP_FUSED_ADAM (fallback: tuning fuse_adam 0,
    the step as a k_adam launch after the epilogue).  Returns the kernels the plan launched."""
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import LossConfig
    t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
         "shifts": model.opt_probe_pos_shifts.detach(), "H": model._H_rv().detach(), "tilts": None}
    t.update(model._base())
    live = [p for g in opt.param_groups for p in g["params"] if p.requires_grad]
    for p in live:
        p.grad = torch.zeros_like(p) if p.grad is None else p.grad.zero_()
    grads = {k: p.grad for k, p in (("obja", model.opt_obja), ("objp", model.opt_objp), ("probe", model.opt_probe),
                                    ("shifts", model.opt_probe_pos_shifts)) if any(p is q for q in live)}
    if store:   # the call overwrites the object gradient: leave garbage there to prove it
        for k in ("obja", "objp"):
            if k in grads:
                grads[k].fill_(3.0)
    cfg = LossConfig.from_loss_params(loss_fn.loss_params)
    idx_t = torch.as_tensor(np.asarray(idx), dtype=torch.int32, device=model.opt_obja.device)
    off = np.array([0, len(idx)], np.int32)
    with torch.no_grad():
        for s in opt._step_tensors():
            s.add_(1)
    prep = _lib.PTYX_PREP_GRAD_STORE if store else 0
    opt._external_step_inc = True
    _lib.set_tuning("fuse_adam", 0 if mode == "fallback" else -1)
    _lib.set_tuning("tail_fin", 0 if mode == "nofold" else -1)
    _lib.set_tuning("rows_hu", 2 if mode == "hu2" else -1)
    _lib.set_tuning("gadam_lead", 0 if mode == "nolead" else -1)
    model.plan.profile_begin()
    try:
        if mode == "off":
            model.plan.forward_loss_grad(t, idx_t, off, cfg, grads, prep=prep)
            opt.step()
        else:
            model.plan.set_adam(opt.fused_step_args())
            model.plan.forward_loss_grad(t, idx_t, off, cfg, grads, prep=prep | _lib.PTYX_PREP_FUSED_ADAM)
    finally:
        prof = model.plan.profile_end()
        opt._external_step_inc = False
        _lib.set_tuning("fuse_adam", -1)
        _lib.set_tuning("tail_fin", -1)
        _lib.set_tuning("rows_hu", -1)
        _lib.set_tuning("gadam_lead", -1)
    torch.cuda.synchronize()
    return prof


@pytest.mark.parametrize("name,store,rows", [("traj_c1_n128", False, -1), ("traj_c1_n128", True, -1),
                                             ("traj_c1_n128", True, 1), ("traj_c1_n128", True, 2),
                                             ("traj_c1_n128", True, 3),
                                             ("traj_n128_p6z6_ga1", True, -1)])
def test_fused_adam_call_bitwise_the_call_then_adam(name, store, rows):
    """PTYX_PREP_FUSED_ADAM (ABI 209): the k_fused3 small call with the optimizer step folded into
    its last launch (k_gather_adam: object gather + Adam of obja / objp per tile, the probe
    gradient's rows + its Adam, k_adam's chunks for the positions) leaves parameters, gradients and
    optimizer state BITWISE what the call followed by the HIP Adam leaves; so does the fallback
    (fuse_adam 0: the registered step as a k_adam launch after the ordinary epilogue); so does the
    fused launch with its tile blocks first (gadam_lead 0, "nolead") instead of its probe-row and rest
    blocks.  The fused
    call also folds k_finalize into its tail launch (k_small_tail_fin: every workgroup recomputes
    the mini-batch coefficients); tail_fin 0 ("nofold") keeps the k_finalize launch: the same bits.
    traj_n128_p6z6_ga1 (the tBL demo's 6 probe modes, 6 slices): the mixed-state engine, whose fused
    launch runs the row-split gather over the slices and the probe rows of every mode.  rows 1
    (tuning gather_rows): the single-state call's gather row-split too, fused (k_gather_adam's
    one-plane row tiles; 2 / 3: k_gather_adam_r4 / _r5, the same held to 128 / 96 VGPRs; −1: the
    default, form 3 for these small single-state calls) and unfused (k_obj_gather_rows) alike."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd import _lib
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    res = {}
    _lib.set_tuning("gather_rows", rows)
    try:
        _fused_adam_modes(name, store, z, res)
    finally:
        _lib.set_tuning("gather_rows", -1)


def _fused_adam_modes(name, store, z, res):
    from tests.dist_helpers import gpu_recon
    modes = ("off", "fast", "fallback", "nofold", "nolead") + (("hu2",) if name == "traj_n128_p6z6_ga1" else ())
    for mode in modes:
        model, opt, loss_fn, batches, _ = gpu_recon(z, niter=1, ret_all=True)   # (Adam state exists)
        prof = _one_step(model, opt, loss_fn, batches[0], mode, store)
        plist = [p for g in opt.param_groups for p in g["params"] if p in opt.state]
        res[mode] = (_params(model), [p.grad.detach().cpu().clone() for p in plist],
                     [{k: v.detach().cpu().clone() for k, v in opt.state[p].items()} for p in plist], prof)
    assert "k_gather_adam" in res["fast"][3] and "k_obj_gather" not in res["fast"][3], res["fast"][3]
    assert "k_gather_adam" not in res["fallback"][3] and "k_obj_gather" in res["fallback"][3]
    if name == "traj_c1_n128":   # (the mixed-state engine needs k_finalize before its adjoint)
        assert "k_finalize" not in res["fast"][3] and "k_finalize" in res["nofold"][3], res["fast"][3]
    assert "k_gather_adam" in res["nofold"][3]
    for mode in modes[1:]:
        for k in res["off"][0]:
            assert np.array_equal(res["off"][0][k], res[mode][0][k]), (mode, k)
        for a, b in zip(res["off"][1], res[mode][1]):
            assert torch.equal(a, b), mode
        for se, sf in zip(res["off"][2], res[mode][2]):
            for k in se:
                assert torch.equal(se[k], sf[k]), (mode, k)
    # the step moved the parameters
    model0, *_ = gpu_recon(z, niter=1, ret_all=True)
    assert not np.array_equal(_params(model0)["opt_obja"], res["fast"][0]["opt_obja"])


@pytest.mark.parametrize("name", ["traj_c1_n128", "traj_n128_p6z6_ga1"])
def test_graphs_fused_adam_bitwise_unfused_and_reference(name):
    """Graph-replayed recon_step with the optimizer step folded into the engine call
    (StepGraphs.FUSE_ADAM, the default) and the step selection too (StepGraphs.SELECT,
    PTYX_PREP_SELECT: inside the small call's preparation launch, or its own launch first with
    tuning sel_fold 0) against the separate ptyx_step_select / HIP Adam launches: bitwise equal
    trajectories, at the reference's (RMS < 1e-5)."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.stepgraph import StepGraphs
    from ptyrad_amd import _lib
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {}
    # (fuse, select, sel_fold): the optimizer step in the call or not; the step selection in the
    # call (inside k_small_prep, or its k_step_select launch first with sel_fold 0) or not
    variants = [(False, False, -1), (True, False, -1), (True, True, -1), (True, True, 0), (False, True, -1)]
    try:
        for fuse, sel, fold in variants:
            StepGraphs.FUSE_ADAM, StepGraphs.SELECT = fuse, sel
            _lib.set_tuning("sel_fold", fold)
            m = gpu_recon(z, graphs=True)
            assert m._step_graphs.replays >= 1
            out[(fuse, sel, fold)] = _params(m)
    finally:
        StepGraphs.FUSE_ADAM, StepGraphs.SELECT = True, True
        _lib.set_tuning("sel_fold", -1)
    base = out[variants[0]]
    for v in variants[1:]:
        for k in base:
            assert np.array_equal(base[k], out[v][k]), (v, k)
    for k, ref in (("opt_obja", z["final_obja"]), ("opt_objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((out[(True, True, -1)][k].astype(np.float64) - ref) ** 2))) < 1e-5, k


def test_graphs_fused_step_with_grad_accumulation():
    """grad_accumulation = 2 on the k_fused3 geometry: a step's call holds two mini-batches, so the
    folded k_finalize (k_small_tail_fin) computes two coefficients a workgroup and the fused Adam
    follows a two-batch gradient.  Eager, graph-replayed with every fold, and graph-replayed with
    none: bitwise the same parameters and optimizer state after three iterations."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.reconstruction import recon_step
    from ptyrad_amd.stepgraph import StepGraphs
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    out = {}
    for tag, graphs, fold in (("eager", False, True), ("fused", True, True), ("plain", True, False)):
        StepGraphs.FUSE_ADAM = StepGraphs.SELECT = fold
        try:
            model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
            flat = np.concatenate(batches)
            quarters = np.array_split(flat, 4)           # 4 mini-batches, 2 optimizer steps an iteration
            for it in (1, 2, 3):
                recon_step(quarters, 2, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
            if graphs:
                assert model._step_graphs.replays >= 1
        finally:
            StepGraphs.FUSE_ADAM = StepGraphs.SELECT = True
        plist = [p for g in opt.param_groups for p in g["params"] if p in opt.state]
        out[tag] = (_params(model), [{k: v.detach().cpu().clone() for k, v in opt.state[p].items()} for p in plist])
    for tag in ("fused", "plain"):
        for k in out["eager"][0]:
            assert np.array_equal(out["eager"][0][k], out[tag][0][k]), (tag, k)
        for se, sf in zip(out["eager"][1], out[tag][1]):
            for k in se:
                assert torch.equal(se[k], sf[k]), (tag, k)


@pytest.mark.parametrize("ga", [1, 2])
def test_graphs_chunked_replay_bitwise_one_step_graphs(ga):
    """StepGraphs.CHUNK: a run of consecutive same-shape steps replays as ONE graph of CHUNK step
    bodies (the device counter picks each body's mini-batch), the run's remainder as one-step
    graphs.  64 patterns in 10·ga mini-batches (ga 1: runs of 4 and 6 steps of one shape; ga 2: runs of
    2 and 8), CHUNK 3, 16 (no run that long: one-step graphs only) and 1, against eager: bitwise the same
    parameters, optimizer state and loss history after three iterations."""
    need_gpu()
    from tests.dist_helpers import gpu_recon
    from ptyrad_amd.reconstruction import recon_step
    from ptyrad_amd.stepgraph import StepGraphs
    z = np.load(os.path.join(GOLDEN, "traj_c1_n128.npz"), allow_pickle=False)
    out = {}
    for tag, graphs, chunk in (("eager", False, 1), ("c1", True, 1), ("c3", True, 3), ("c16", True, 16)):
        StepGraphs.CHUNK = chunk
        try:
            model, opt, loss_fn, batches, _ = gpu_recon(z, niter=0, ret_all=True)
            flat = np.concatenate(batches)
            parts = np.array_split(flat, 10 * ga)      # ragged: two step shapes, each a run of 5
            hist = [recon_step(parts, ga, model, opt, loss_fn, None, it, verbose=False, graphs=graphs)
                    for it in (1, 2, 3)]
            sg = model._step_graphs if graphs else None
        finally:
            StepGraphs.CHUNK = 16
        if chunk == 3:
            assert any(k[0] == "chunk" for k in sg.graphs), list(sg.graphs)
        if graphs:
            assert sg.replays >= 1
        plist = [p for g in opt.param_groups for p in g["params"] if p in opt.state]
        out[tag] = (_params(model), [{k: v.detach().cpu().clone() for k, v in opt.state[p].items()} for p in plist],
                    hist)
    for tag in ("c1", "c3", "c16"):
        for k in out["eager"][0]:
            assert np.array_equal(out["eager"][0][k], out[tag][0][k]), (tag, k)
        for se, sf in zip(out["eager"][1], out[tag][1]):
            for k in se:
                assert torch.equal(se[k], sf[k]), (tag, k)
        for a, b in zip(out["eager"][2], out[tag][2]):
            for k in a:
                assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (tag, k)
