"""BASELINE configs c3 / c5 at their shapes through the HIP path vs the oracle, rank-local
measurement storage, GPU checkpoint resume, and the c1-shape trajectory.

c3: N = 256, P = 8 probe modes × O = 2 object modes, Nz = 1 (BASELINE configs[2]);
c5: N = 256, P = 4, fp16 DP storage / fp32 accumulate (configs[4]).  A 3×3 scan in the
config's geometry, two mini-batches per call, random DPs (SURVEY §8d allows them for c3-c5);
the oracle runs on the same fp16-rounded DPs.  Tolerances as tests/test_gpu_parity.py.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from tests.test_gpu_parity import TOL_DP, TOL_G, TOL_SH, TOL_TERMS, orc_default_loss, run_fused
from tests.test_oracle_golden import rel

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def config_problem(P, O, meas_f16, seed):
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(256, 3, 3, P=P, O=O, Nz=1, seed=seed)
    meas = pr.meas.astype(np.float16).astype(np.float32) if meas_f16 else pr.meas
    return dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts,
                crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=meas, shift_probes=True,
                loss_params=json.loads(json.dumps(orc_default_loss())))


def check_against_oracle(d, batches, meas_f16, gather=None):
    ks = {}
    terms, dp, g, _ = run_fused(d, dev(), batches, meas_f16=meas_f16, kernels=ks)
    assert {"k_s1", "k_s2", "k_s3", "k_s4", "k_s5"} <= set(ks), ks      # the N = 256 stripe engine ran
    if gather is not None:   # object gradient by slots + k_obj_gather (else k_s4's f32 atomics)
        assert ("k_obj_gather" in ks) == gather, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH
    return g


def test_c3_shape_p8_o2_vs_oracle():
    d = config_problem(8, 2, False, seed=11)
    batches = [np.array([0, 4, 8]), np.array([5, 1])]
    g1 = check_against_oracle(d, batches, meas_f16=False, gather=True)
    # two object modes: slots + k_obj_gather, so the object gradient is bitwise reproducible
    _, _, g2, _ = run_fused(d, dev(), batches, meas_f16=False)
    for k in ("obja", "objp"):
        assert np.array_equal(g1[k], g2[k]), k


def test_c5_shape_p4_fp16_dps_vs_oracle():
    d = config_problem(4, 1, True, seed=12)
    check_against_oracle(d, [np.array([2, 6, 7, 3]), np.array([8, 0])], meas_f16=True)


@pytest.fixture
def tuning():
    """ptyx_set_tuning for one test; every key back to its measured default afterwards."""
    from ptyrad_amd import _lib
    yield _lib.set_tuning
    for k in _lib.TUNING_KEYS:
        _lib.set_tuning(k, -1)


@pytest.mark.parametrize("hold,park", [(0, 1), (1, 1), (3, 0), (4, 1)])
def test_stripe_mode_hold_and_psi0_variants(tuning, hold, park):
    """k_s3 with the first `hold` of P·O = 6 modes held in registers (the rest recomputed), and
    k_s4 with ψ⁰ parked (1) or recomputed from T1 (0): all the same gradients."""
    tuning("s3_hold", hold)
    tuning("s_psi0", park)
    d = config_problem(3, 2, False, seed=13)
    check_against_oracle(d, [np.array([1, 3, 4]), np.array([7, 2, 0])], meas_f16=False)


@pytest.mark.parametrize("O,flag", [(1, 1), (2, 0)])
def test_stripe_object_gradient_atomics_and_slots(tuning, O, flag):
    """k_s4's object-gradient form the mode count does not pick by default (tuning "s_gather"):
    slots + k_obj_gather for one object mode, f32 atomics for two; the same gradients."""
    tuning("s_gather", flag)
    d = config_problem(2, O, False, seed=14)
    check_against_oracle(d, [np.array([6, 2, 3]), np.array([0, 8, 4, 1])], meas_f16=False, gather=flag == 1)


@pytest.mark.parametrize("rows,N,P,O,Nz,holdh", [(1, 128, 1, 1, 1, -1), (1, 128, 1, 1, 3, -1), (0, 128, 3, 1, 2, -1),
                                                 (-1, 128, 3, 1, 3, 0), (-1, 128, 2, 1, 4, -1),
                                                 (1, 256, 8, 2, 1, -1)])
def test_gather_rows_variant_vs_oracle(tuning, rows, N, P, O, Nz, holdh):
    """k_obj_gather_rows (tuning "gather_rows" 1: every unsplit gather lists a chunk's hits and
    gives each wave its rows) and the whole-hit k_obj_gather (0, also for mixed-state small calls
    that take the rows form by default): the same gradients on k_fused3, k_fused3ms, the
    mixed-state engine and the N = 256 stripe engine with slots.  Also the mixed-state engine's
    H/N² streamed per propagation (tuning "fmm_hold_h" 0) instead of held in registers (the
    default when the call has at most one workgroup a CU)."""
    tuning("gather_rows", rows)
    tuning("fmm_hold_h", holdh)
    if N == 256:
        tuning("s_gather", 1)
        d = config_problem(P, O, False, seed=15)
        check_against_oracle(d, [np.array([1, 3, 4]), np.array([7, 2, 0, 8])], meas_f16=False, gather=True)
        return
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(N, 4, 4, P=P, O=O, Nz=Nz, seed=16)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=json.loads(json.dumps(orc_default_loss())))
    batches = [np.array([0, 5, 9, 14]), np.array([3, 12, 6]), np.array([15, 1, 10, 7, 2])]
    ks = {}
    terms, dp, g, _ = run_fused(d, dev(), batches, meas_f16=False, kernels=ks)
    assert "k_obj_gather" in ks, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


# ------------------------------------------------------------------ rank-local measurements
def test_rank_local_measurement_block_equals_full_stack():
    """PtychoHIP holding only the DPs of the positions it uses (rows in a shuffled order, via
    measurements_index) gives bit-identical loss terms and gradients to the full stack, on the
    register engine (c1 shape, k_fused3) and on the general engine (mixed state)."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from tests.test_gpu_model import init_vars, model_params
    from tests.test_oracle_golden import CASES, load_case
    for name in ("n128_c1_b32", "n32_p2o2z3"):
        d = load_case([c for c in CASES if name in c][0])
        b = d["batch"]
        lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
               "probe_pos_shifts": 5e-4}
        out = []
        for shard in (False, True):
            iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"], d["meas"])
            if shard:
                mi = np.random.default_rng(0).permutation(np.unique(b))
                iv["measurements"] = np.ascontiguousarray(d["meas"][mi])
                iv["measurements_index"] = mi
            model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
            loss = CombinedLoss(d["loss_params"], device=device)
            terms = loss.fused_into(model, [b])
            out.append((terms.cpu().numpy(), [p.grad.cpu().numpy() for p in
                                              (model.opt_obja, model.opt_objp, model.opt_probe,
                                               model.opt_probe_pos_shifts)]))
            if shard:
                assert model.measurements.shape[0] == np.unique(b).size
                outside = np.setdiff1d(np.arange(d["shifts"].shape[0]), b)
                if outside.size:
                    with pytest.raises(IndexError):
                        loss.fused_into(model, [outside[:1]])
        np.testing.assert_array_equal(out[0][0], out[1][0])
        for a, c in zip(out[0][1], out[1][1]):
            assert rel(c, a) < 1e-6, name          # same arithmetic; atomics may reorder sums
        np.testing.assert_allclose(out[0][0][0], d["loss_terms"], rtol=TOL_TERMS, atol=1e-7)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_each_holding_half_the_dps_match_reference_trajectory(tmp_path):
    """Two gloo ranks (both on cuda:0), each PtychoHIP holding only its own mini-batches' DPs
    (DistContext.local_indices), one all-reduce per optimizer step: bitwise-identical replicas
    whose final object matches the reference's recon_step trajectory (RMS < 1e-5)."""
    dev()
    import torch.multiprocessing as mp
    from tests.dist_helpers import gpu_dist_worker
    path = os.path.join(GOLDEN, "traj_n32_p2_ga2.npz")
    z = np.load(path, allow_pickle=False)
    out = str(tmp_path / "r.npz")
    mp.start_processes(gpu_dist_worker, args=(2, _free_port(), path, out), nprocs=2, start_method="spawn")
    r0, r1 = np.load(out.replace(".npz", "_r0.npz")), np.load(out.replace(".npz", "_r1.npz"))
    assert int(r0["held"]) + int(r1["held"]) == z["batches"].size      # each rank: only its DPs
    assert int(r0["held"]) < z["batches"].size and int(r1["held"]) < z["batches"].size
    for k in ("obja", "objp", "probe"):
        assert np.array_equal(r0[k], r1[k]), k
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        assert float(np.sqrt(np.mean((r0[k].astype(np.float64) - ref) ** 2))) < 1e-5, k


# ------------------------------------------------------------------ checkpoint resume on the GPU
def test_ptychohip_checkpoint_resume_matches_reference_trajectory(tmp_path):
    """save after iteration 1 (save.py:85-140 layout, Adam state included), resume into a fresh
    PtychoHIP + Adam (reconstruction.py:356-366), run iterations 2-3: the reference trajectory's
    final object is reproduced (RMS < 1e-5) and equals the uninterrupted run."""
    dev()
    from ptyrad_amd.checkpoint import load_ptyrad, make_save_dict, resume, save_ptyrad
    from ptyrad_amd.reconstruction import recon_step
    from tests.dist_helpers import gpu_recon
    z = np.load(os.path.join(GOLDEN, "traj_n64_b4_ga1.npz"), allow_pickle=False)
    full = gpu_recon(z)
    model, opt, loss_fn, batches, bl = gpu_recon(z, niter=1, ret_all=True)
    params = {"recon_params": {"save_result": ["model", "optim_state"]}}
    p = save_ptyrad(str(tmp_path / "model_iter0001.pt"),
                    make_save_dict(str(tmp_path), model, params, opt, 1, None, bl))
    model2, opt2, _, _, _ = gpu_recon(z, niter=0, ret_all=True)
    assert resume(model2, opt2, load_ptyrad(p)) == 1
    for it in (2, 3):
        recon_step(batches, int(z["grad_accumulation"]), model2, opt2, loss_fn, None, it, verbose=False)
    for k, ref in (("opt_obja", z["final_obja"]), ("opt_objp", z["final_objp"])):
        got = getattr(model2, k).detach().cpu().numpy().astype(np.float64)
        assert float(np.sqrt(np.mean((got - ref) ** 2))) < 1e-5, k
        assert rel(got, getattr(full, k).detach().cpu().numpy()) < 1e-6, k
    assert len(model2.loss_iters) == 3


# ------------------------------------------------------------------ c1 shape trajectory
def test_c1_shape_trajectory_matches_reference():
    """c1 (tBL_WSe2 params: N = 128, 8×8 scan, probe / position lr 1e-4, 2 iterations of Adam)
    through PtychoHIP + recon_step: final object RMS < 1e-5 vs the reference run."""
    path = os.path.join(GOLDEN, "traj_c1_n128.npz")
    if not os.path.exists(path):
        pytest.skip("traj_c1_n128.npz not generated")
    from tests.dist_helpers import gpu_recon
    z = np.load(path, allow_pickle=False)
    model = gpu_recon(z)
    for k, ref in (("opt_obja", z["final_obja"]), ("opt_objp", z["final_objp"])):
        got = getattr(model, k).detach().cpu().numpy().astype(np.float64)
        assert float(np.sqrt(np.mean((got - ref) ** 2))) < 1e-5, k
    prb = torch.view_as_complex(model.opt_probe.detach()).cpu().numpy()
    assert rel(prb, z["final_probe"]) < 1e-5


def test_c5_shape_call_split_by_stripe_capacity(monkeypatch):
    """A call larger than the stripe engine's per-call capacity (PTYX_STRIPE_MB) is split at
    mini-batch boundaries; the pieces after the first reuse the first one's object / probe
    preparation (PTYX_PREP_FULL then PTYX_PREP_REUSE).  Same results as the oracle."""
    monkeypatch.setenv("PTYX_STRIPE_MB", "8")         # (P T1 + P·O T2) · 512 KiB = 4 MiB a pattern (O = 1:
                                                      # ψ⁰ recomputed, not parked)
    d = config_problem(4, 1, True, seed=13)
    batches = [np.array([0, 4]), np.array([8, 1]), np.array([5, 2]), np.array([6, 3]), np.array([7])]
    ks = {}
    terms, dp, g, plan = run_fused(d, dev(), batches, meas_f16=True, kernels=ks)
    assert plan.register_capacity == 2 and ks["k_s3"][0] == 5          # five calls (one mini-batch each)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("spec,P,Nz", [(-1, 1, 1), (0, 1, 1), (-1, 3, 2), (0, 3, 2)])
def test_small_call_probe_spectrum_variants_vs_oracle(tuning, spec, P, Nz):
    """Small calls (one mini-batch per optimizer step) take the shifted probe's spectrum F(P) in
    k_small_prep's leading workgroups, one register-resident 2-D FFT a mode (tuning "small_spec",
    the default), or as the row pass there plus a k_lines_cols launch (0): both against the oracle
    on k_fused3 / k_fused3ms and the mixed-state engine, and against each other to fp32 rounding."""
    tuning("small_spec", spec)
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 4, 4, P=P, O=1, Nz=Nz, seed=21)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=json.loads(json.dumps(orc_default_loss())))
    batches = [np.array([0, 5, 9, 14, 3, 12])]
    ks = {}
    terms, dp, g, _ = run_fused(d, dev(), batches, meas_f16=False, kernels=ks)
    assert ("k_probe_spectrum" in ks) == (spec == 0), ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("q1", [0.5, 1.0])
def test_small_call_psi_hold_bitwise(tuning, q1):
    """k_fused3 with ψ⁰ held in registers instead of parked (calls of at most one workgroup a CU,
    256 VGPRs + AGPRs; the default there, tuning "psi_hold" 0 parks): the park stores exactly the
    registers it reloads, so the results are bitwise the parking kernel's, and at the oracle's."""
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 5, 5, P=1, O=1, Nz=1, seed=23)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=json.loads(json.dumps(orc_default_loss())))
    d["loss_params"]["loss_single"]["dp_pow"] = q1
    batches = [np.array([0, 5, 9, 14, 3, 12, 22]), np.array([7, 18, 2, 24])]
    out = []
    for hold in (0, 1):
        tuning("psi_hold", hold)
        ks = {}
        out.append(run_fused(d, dev(), batches, meas_f16=False, kernels=ks))
        assert "k_fused" in ks, ks
    (t0, dp0, g0, _), (t1, dp1, g1, _) = out
    np.testing.assert_array_equal(t0, t1)
    np.testing.assert_array_equal(dp0, dp1)
    for k in g0:
        np.testing.assert_array_equal(g0[k], g1[k])
    oterms, _, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                          d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(t1, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g1[k], og[k]) < TOL_G, k


def test_large_call_psi_hold_forced_vs_parking_and_oracle(tuning):
    """tuning psi_hold 2 (an A/B switch for large calls): one k_fused3 workgroup a CU, each running
    several patterns with ψ⁰ held in registers, instead of two a CU parking it.  400 patterns in
    two mini-batches (more than the CUs): both forms at the oracle's; their probe-gradient segments
    differ (another workgroup count), so they agree to fp32 summation order, not bitwise."""
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 20, 20, P=1, O=1, Nz=1, seed=29)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=json.loads(json.dumps(orc_default_loss())))
    perm = np.random.default_rng(4).permutation(400)
    batches = [perm[:200], perm[200:]]
    out = []
    for hold in (0, 2):
        tuning("psi_hold", hold)
        ks = {}
        out.append(run_fused(d, dev(), batches, meas_f16=False, kernels=ks))
        assert "k_fused" in ks, ks
    (t0, dp0, g0, _), (t2, dp2, g2, _) = out
    np.testing.assert_array_equal(dp0, dp2)          # the forward model is per pattern: same bits
    np.testing.assert_allclose(t2, t0, rtol=1e-6, atol=1e-9)
    for k in g0:
        assert rel(g2[k], g0[k]) < 1e-6, k
    oterms, _, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                          d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(t2, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g2[k], og[k]) < TOL_G, k
