"""HIP path (libptyx.so through the C ABI) vs the reference's golden vectors and the oracle.

Tolerances (fp32 engine vs fp32 reference / fp64 oracle, relative L2 over the array):
  dp and loss terms          ≤ 1e-5
  object / probe gradients   ≤ 5e-5
  position gradients         ≤ 2e-4   (a sum of cancelling terms; the reference's own fp32
                                       rounding is ~6e-5 here, tests/test_oracle_golden.py)
"""
import json

import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from ptyrad_amd.csrc.build import GEN_SIZES
from tests.test_oracle_golden import CASES as ALL_CASES, load_case, rel

# raw C-ABI cases: the optional-stage (blur) and optimised-propagator fixtures run through
# PtychoHIP in test_gpu_stages.py / test_gpu_propagator.py
CASES = [c for c in ALL_CASES if not any(k in c for k in ("blur", "_opt", "each", "pacbed", "simlar"))]

pytestmark = pytest.mark.gpu

TOL_DP, TOL_TERMS, TOL_G, TOL_SH = 1e-5, 1e-5, 5e-5, 2e-4
# probe gradient with loss_single AND loss_poissn: the two terms' contributions cancel in the
# probe's sum over patterns, so fp32 lands at ≈ 5e-5 relative to the fp64 oracle on every engine
# (multislice N 128 Nz 3: general engine 4.9e-5, k_fused3ms 5.2e-5; one term 5e-6 —
# tools/diag_both_terms.py, profiles/r04/w/diag_both_terms.txt)
TOL_G_BOTH = 1e-4


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def tensors(d, device, meas_dtype=torch.float32):
    t = {
        "obja": torch.tensor(d["obja"], device=device),
        "objp": torch.tensor(d["objp"], device=device),
        "probe": torch.view_as_real(torch.tensor(d["probe"].astype(np.complex64), device=device)).contiguous(),
        "shifts": torch.tensor(d["shifts"], device=device),
        "H": torch.tensor(d["H"].astype(np.complex64), device=device),
        "occu": torch.tensor(d["occu"], device=device),
        "crop_pos": torch.tensor(d["crop_pos"].astype(np.int32), device=device),
        "meas": torch.tensor(d["meas"], device=device).to(meas_dtype),
    }
    return t


def make_plan(d, device, max_patterns=None, meas_f16=False):
    from ptyrad_amd.engine import Plan
    O, Nz, Ny, Nx = d["obja"].shape
    P, N = d["probe"].shape[:2]
    return Plan(N, P, O, Nz, Ny, Nx, d["shifts"].shape[0], max_patterns or d["shifts"].shape[0],
                shift_probes=bool(d["shift_probes"]), meas_f16=meas_f16, device=device)


def run_fused(d, device, batches, grad_scale=1.0, meas_f16=False, want=("obja", "objp", "probe", "shifts"),
              kernels=None):
    """kernels: a dict that receives the plan's per-kernel launch statistics (engine check)."""
    from ptyrad_amd.engine import LossConfig, batch_offsets
    plan = make_plan(d, device, meas_f16=meas_f16)
    if kernels is not None:
        plan.profile_begin()
    t = tensors(d, device, torch.float16 if meas_f16 else torch.float32)
    grads = {k: torch.zeros_like(t[k if k != "shifts" else "shifts"]) for k in want}
    if not d["shift_probes"]:
        grads.pop("shifts", None)
    flat = np.concatenate(batches).astype(np.int32)
    N = d["probe"].shape[-1]
    dp = torch.zeros((len(flat), N, N), device=device)
    terms = plan.forward_loss_grad(t, flat, batch_offsets(batches), LossConfig.from_loss_params(d["loss_params"]),
                                   grads, grad_scale=grad_scale, dp_out=dp)
    torch.cuda.synchronize()
    if kernels is not None:
        kernels.update(plan.profile_end())
    g = {k: v.cpu().numpy() for k, v in grads.items()}
    if "probe" in g:
        g["probe"] = g["probe"][..., 0] + 1j * g["probe"][..., 1]
    return terms.cpu().numpy(), dp.cpu().numpy(), g, plan


# the engine each BASELINE-config / demo-shaped fixture (make_golden.py --large) must run on
ENGINE_OF = {"n256_p8o2z1_c3": "k_s1", "n256_p4o1z1_c5f16": "k_s1", "n128_p1o1z16_c4": "k_fused",
             "n128_p6o1z6_tbl": "k_fmm_fwd", "n256_p4o1z5_pso": "k_adjoint",
             # loss_single + loss_poissn (make_golden.py --both-terms): the two-pass register / stripe paths
             "n128_p1o1z1_both": "k_fused", "n128_p1o1z3_both": "k_fused", "n128_p3o1z2_both": "k_fmm_fwd",
             "n256_p2o2z1_both": "k_s3",
             # radix 7 / 14 / 21 (make_golden.py --radix7): the general engine
             "n112_p2o1z2_r7": "k_adjoint", "n49_p1o2z1_r7": "k_adjoint", "n196_p1o1z2_r14": "k_adjoint",
             "n189_p2o1z1_r27x7": "k_adjoint",
             # N above 256 (make_golden.py --big-n): the general engine's line-block plans
             "n384_p1o1z1_big": "k_adjoint", "n343_p1o1z2_r49": "k_adjoint", "n512_p2o1z1_big": "k_adjoint"}


@pytest.mark.parametrize("path", CASES, ids=[p.split("/")[-1][:-4] for p in CASES])
def test_fused_matches_reference_golden(path):
    device = dev()
    d = load_case(path)
    ks = {}
    terms, dp, g, _ = run_fused(d, device, [d["batch"]], meas_f16=bool(d.get("meas_storage_f16", False)), kernels=ks)
    name = path.split("/")[-1][:-4]
    if name in ENGINE_OF:
        assert ENGINE_OF[name] in ks, (name, sorted(ks))
    if "dp" in d:
        assert rel(dp, d["dp"]) < TOL_DP
    else:
        assert rel(dp[:4], d["dp_head"]) < TOL_DP
        assert rel(dp.reshape(len(dp), -1).astype(np.float64).sum(1), d["dp_sums"]) < TOL_DP
    np.testing.assert_allclose(terms[0], d["loss_terms"], rtol=TOL_TERMS, atol=1e-7)
    assert rel(g["obja"], d["g_obja"]) < TOL_G
    assert rel(g["objp"], d["g_objp"]) < TOL_G
    lp = d["loss_params"]
    both = lp["loss_single"]["state"] and lp["loss_poissn"]["state"]
    assert rel(g["probe"], d["g_probe"][..., 0] + 1j * d["g_probe"][..., 1]) < (TOL_G_BOTH if both else TOL_G)
    if d["shift_probes"]:
        assert rel(g["shifts"], d["g_shifts"]) < TOL_SH


@pytest.mark.parametrize("path", CASES[:4], ids=[p.split("/")[-1][:-4] for p in CASES[:4]])
def test_forward_only_matches_oracle(path):
    device = dev()
    d = load_case(path)
    plan = make_plan(d, device)
    t = tensors(d, device)
    dp = plan.forward(t, d["batch"].astype(np.int32))
    ref = orc.forward_dp(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"],
                         d["batch"], shift_probes=bool(d["shift_probes"]))
    assert rel(dp.cpu().numpy(), ref) < TOL_DP


def test_multibatch_call_equals_sum_of_batches():
    """Several mini-batches in one call: per-batch NRMSE normalisation, gradients summed."""
    device = dev()
    d = load_case([c for c in CASES if "n32_p2o2z3" in c][0])
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(5).permutation(S)
    batches = np.array_split(perm, 3)
    terms, _, g, _ = run_fused(d, device, batches, grad_scale=0.5)
    oterms, _, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                          d["occu"], d["meas"], batches, d["loss_params"],
                                          shift_probes=True, grad_scale=0.5)
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_meas_fp16_storage():
    device = dev()
    d = load_case([c for c in CASES if "n32_p1o1z1" in c][0])
    d16 = dict(d)
    d16["meas"] = d["meas"].astype(np.float16).astype(np.float32)
    terms, _, g, _ = run_fused(d16, device, [d["batch"]], meas_f16=True)
    oterms, _, og = orc.forward_loss_grad(d16["obja"], d16["objp"], d16["probe"], d16["shifts"], d16["crop_pos"],
                                          d16["H"], d16["occu"], d16["meas"], [d["batch"]], d["loss_params"])
    np.testing.assert_allclose(terms[0], oterms[0], rtol=TOL_TERMS, atol=1e-7)
    assert rel(g["objp"], og["objp"]) < TOL_G


def test_null_gradients_skip_work_and_others_unchanged():
    device = dev()
    d = load_case([c for c in CASES if "n32_p1o1z1" in c][0])
    terms, _, g, _ = run_fused(d, device, [d["batch"]], want=("objp",))
    assert set(g) == {"objp"}
    assert rel(g["objp"], d["g_objp"]) < TOL_G
    np.testing.assert_allclose(terms[0], d["loss_terms"], rtol=TOL_TERMS, atol=1e-7)


def test_external_dldi_adjoint_matches_oracle():
    """ptyx_adjoint_dldi with dL/dI from the oracle loss == oracle adjoint (no sparse term)."""
    device = dev()
    d = load_case([c for c in CASES if "n32_p2o2z3" in c][0])
    b = d["batch"]
    n = d["probe"].shape[-1]
    amp, ph = orc.get_patches(d["obja"], d["objp"], d["crop_pos"], b, n)
    probes = orc.get_probes(d["probe"], d["shifts"][b], True)
    cache = orc.forward(amp, ph, probes, d["H"], d["occu"])
    _, dLdI, _ = orc.loss_terms(cache.dp, d["meas"][b], ph, d["occu"], d["loss_params"])
    dA, dP, dprobe, dshift = orc.adjoint(cache, dLdI, np.zeros_like(ph, np.float64), amp, ph, d["probe"],
                                         d["shifts"][b], d["H"], d["occu"], True)
    gA = np.zeros(d["obja"].shape)
    gP = np.zeros(d["objp"].shape)
    for i, s in enumerate(b):
        cy, cx = d["crop_pos"][s]
        gA[:, :, cy:cy + n, cx:cx + n] += dA[i]
        gP[:, :, cy:cy + n, cx:cx + n] += dP[i]
    plan = make_plan(d, device)
    t = tensors(d, device)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    plan.adjoint_dldi(t, b.astype(np.int32), torch.tensor(dLdI, dtype=torch.float32, device=device), grads)
    torch.cuda.synchronize()
    assert rel(grads["obja"].cpu().numpy(), gA) < TOL_G
    assert rel(grads["objp"].cpu().numpy(), gP) < TOL_G
    gp = grads["probe"].cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], dprobe) < TOL_G


def test_loss_terms_deterministic():
    device = dev()
    d = load_case([c for c in CASES if "n64_p3o1z1" in c][0])
    t1, _, g1, _ = run_fused(d, device, [d["batch"]])
    t2, _, g2, _ = run_fused(d, device, [d["batch"]])
    assert np.array_equal(t1, t2)
    assert np.array_equal(g1["probe"], g2["probe"])   # slab reduction in fixed order


def test_n256_mixed_state_vs_oracle():
    """c3-shaped (N=256, P=2, O=2) small problem through the global-scratch FFT path."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(256, 2, 2, P=2, O=2, Nz=1, seed=3)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True,
             loss_params=json.loads(json.dumps(orc_default_loss())))
    b = np.array([0, 3, 1])
    terms, dp, g, _ = run_fused(d, device, [b])
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], [b], d["loss_params"])
    assert rel(dp, odps[0]) < TOL_DP
    np.testing.assert_allclose(terms[0], oterms[0], rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("P,O,Nz,shift,both", [(2, 1, 3, True, False), (1, 1, 3, True, False),
                                               (1, 2, 2, False, False), (2, 2, 2, True, False),
                                               (1, 3, 1, True, False), (2, 2, 2, True, True)])
def test_n256_general_engine_vs_oracle(P, O, Nz, shift, both):
    """N = 256 through the general two-pass engine (multislice, more object modes than the
    stripe engine takes, or broadcast probes) — the fused g256_fstage chains, with
    and without the far-field cache (P·O > 1 vs P·O = 1), ψ⁰ parking (O > 1) and broadcast
    probes: ragged mini-batches vs the oracle, plus ptyx_forward's DPs and the external-dL/dI
    adjoint."""
    _general_engine_case(256, P, O, Nz, shift, both)


@pytest.mark.parametrize("P,O,q1", [(2, 1, 0.5), (2, 2, 0.5), (3, 2, 1.0), (1, 1, 0.7)])
def test_stripe_engine_both_terms_vs_oracle(P, O, q1):
    """N = 256 stripe engine with loss_single + loss_poissn (+ loss_sparse): k_s3 takes both terms'
    partial sums, k_finalize both coefficients, a second k_s3 the weighted ∂ℓ/∂I; ragged
    mini-batches vs the oracle (losses.py:36-75)."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(256, 3, 3, P=P, O=O, Nz=1, seed=60 + 3 * P + O)
    lp = orc_default_loss()
    lp["loss_poissn"]["state"] = True
    lp["loss_single"]["dp_pow"] = q1
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(30.0), shifts=pr.shifts, crop_pos=pr.crop_pos,
             H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True, loss_params=lp)
    batches = [np.array([4, 0, 7, 2]), np.array([8]), np.array([1, 5, 3, 6])]
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    assert "k_s3" in ks and ks["k_s3"][0] == 2 and "k_adjoint" not in ks, ks     # k_s3 around k_finalize
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, lp, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("P,O,Nz,shift,both", [(2, 2, 3, True, True), (1, 2, 2, False, False),
                                               (3, 2, 1, True, False), (1, 1, 1, True, True)])
def test_n128_general_engine_vs_oracle(P, O, Nz, shift, both):
    """N = 128 through the general engine's LDS FFT — mixed-state multislice with both data terms
    and two object modes (one object mode takes the mixed-state register engine), several object
    modes with the far-field cache and the probe-mode split, broadcast probes, and the single-mode
    two-term path (k_forward1 / k_adjoint1): vs the oracle as above."""
    _general_engine_case(128, P, O, Nz, shift, both)


@pytest.mark.parametrize("N,P,O,Nz,shift,both", [(96, 2, 1, 2, True, False), (96, 1, 1, 1, True, True),
                                                 (160, 1, 2, 1, True, False), (192, 2, 1, 2, False, False)])
def test_mixed_radix_general_engine_vs_oracle(N, P, O, Nz, shift, both):
    """N with factors 3 / 5 (the reference takes whatever meas_crop /
    meas_resample / meas_pad produce, init_params.py:53, 340, 361): the general engine's mixed-radix
    Stockham passes (16 × 6 in LDS at N = 96, 16 × 10 and 16 × 12 in global scratch at 160 / 192)
    vs the oracle, as above."""
    _general_engine_case(N, P, O, Nz, shift, both)


# every 2·3·5·7-smooth N in [32, 512] (the sizes ptyx_gen.hip registers), cycling through mode /
# slice / shift / loss-term configurations; 128 and 256 run the register / stripe engines for some
# of these and have their own cases
_SMOOTH_CFGS = [(1, 1, 1, True, False), (2, 1, 2, True, False), (1, 2, 1, True, True), (2, 1, 1, False, False),
                (1, 1, 3, True, False)]
_SMOOTH_N = [n for n in GEN_SIZES if n not in (128, 256)]


@pytest.mark.parametrize("N", _SMOOTH_N)
def test_every_smooth_n_vs_oracle(N):
    """Radix plans 2-27 (ptyx_fft.hpp plan_r1): odd N, radix 9 / 15 / 25 / 27 in-register DFTs, the
    LDS (N ≤ 128) and global-scratch layouts, 512-thread workgroups for radices above 16."""
    P, O, Nz, shift, both = _SMOOTH_CFGS[_SMOOTH_N.index(N) % len(_SMOOTH_CFGS)]
    _general_engine_case(N, P, O, Nz, shift, both)


@pytest.mark.parametrize("N,P,O,Nz,shift,both", [(64, 2, 8, 1, True, False), (32, 3, 8, 2, True, True),
                                                 (96, 8, 1, 2, False, False), (32, 1, 12, 1, True, False),
                                                 (48, 2, 20, 2, True, True), (32, 1, 32, 1, False, False)])
def test_general_engine_maximum_modes_vs_oracle(N, P, O, Nz, shift, both):
    """The plan's limits: up to 32 object modes (kMaxModesO, the loss_sparse sums per mode, the
    per-mode sparse coefficients) and 8 probe modes (the probe-mode split of small calls)."""
    _general_engine_case(N, P, O, Nz, shift, both)


def test_object_modes_beyond_limit_are_refused():
    dev()
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import Plan
    with pytest.raises(_lib.PtyxError, match="EUNSUPPORTED"):
        Plan(32, 1, 33, 1, 100, 100, 4, 4, device=torch.device("cuda", 0))


@pytest.mark.parametrize("seed", range(12))
def test_random_configuration_vs_oracle(seed, monkeypatch):
    """Seeded random (N, P, O, Nz, shifted probes, one or both data terms, far-field cache on /
    off, ragged mini-batches) through whichever engine the plan picks, vs the oracle — the
    combinations no hand-written case lists (tools/check_sweep.py runs the long form)."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    rng = np.random.default_rng(1000 + seed)
    N = int(rng.choice([32, 48, 64, 96, 128, 160, 256]))
    P, O = int(rng.integers(1, 4)), int(rng.integers(1, 3))
    Nz = int(rng.integers(1, 4)) if N <= 128 else int(rng.integers(1, 3))
    shift, both, cache = (bool(rng.integers(0, 2)) for _ in range(3))
    if not cache:
        monkeypatch.setenv("PTYX_FFC_MB", "0")
    pr = syn.random_problem(N, 3, 3, P=P, O=O, Nz=Nz, seed=int(rng.integers(0, 1 << 30)))
    lp = orc_default_loss()
    lp["loss_poissn"]["state"] = both
    d = dict(obja=pr.obja, objp=(pr.objp / Nz).astype(np.float32), probe=pr.probe * np.float32(30.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=lp)
    perm = rng.permutation(9)
    cut = sorted(set([0, 9] + [int(c) for c in rng.integers(1, 9, 2)]))
    batches = [perm[a:b] for a, b in zip(cut[:-1], cut[1:])]
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, lp, shift_probes=shift, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-6)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < (TOL_G_BOTH if both and k == "probe" else TOL_G), k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_unsupported_n_is_refused():
    """N with a prime factor above 7 (88 = 8·11, 143 = 11·13), or outside [32, 512], is refused
    with PTYX_EUNSUPPORTED at plan creation, not run."""
    dev()
    from ptyrad_amd import _lib
    from ptyrad_amd.engine import Plan
    for n in (88, 143, 16, 540, 1024):
        with pytest.raises(_lib.PtyxError, match="EUNSUPPORTED"):
            Plan(n, 1, 1, 1, 300, 300, 4, 4, device=torch.device("cuda", 0))
    Plan(100, 1, 1, 1, 200, 200, 4, 4, device=torch.device("cuda", 0)).close()


def _general_engine_case(N, P, O, Nz, shift, both):
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(N, 3, 3, P=P, O=O, Nz=Nz, seed=40 + 7 * P + O + Nz)
    lp = orc_default_loss()
    if both:
        lp["loss_poissn"]["state"] = True
    d = dict(obja=pr.obja, objp=(pr.objp / Nz).astype(np.float32), probe=pr.probe * np.float32(30.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=lp)
    perm = np.random.default_rng(P + O + Nz).permutation(9)
    batches = [perm[:4], perm[4:5], perm[5:]]
    ks = {}
    terms, dp, g, plan = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    assert ("k_adjoint" in ks or "k_adjoint1" in ks) and "k_s1" not in ks and "k_fused" not in ks, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH
    t = tensors(d, device)
    b = perm[:5].astype(np.int32)
    dpf = torch.zeros((len(b), N, N), device=device)
    plan.forward(t, b, dp_out=dpf)
    torch.cuda.synchronize()
    assert rel(dpf.cpu().numpy(), np.concatenate(odps)[:5]) < TOL_DP
    # external dL/dI through k_adjoint<EXT> (recomputed forward, no cache)
    amp, ph = orc.get_patches(d["obja"], d["objp"], d["crop_pos"], b, N)
    probes = orc.get_probes(d["probe"], d["shifts"][b], shift)
    cache = orc.forward(amp, ph, probes, d["H"], d["occu"])
    dLdI = np.random.default_rng(1).standard_normal(cache.dp.shape).astype(np.float32) * 1e-3
    dA, dP, dprobe, _ = orc.adjoint(cache, dLdI, np.zeros_like(ph, np.float64), amp, ph, d["probe"],
                                    d["shifts"][b], d["H"], d["occu"], shift)
    gA = np.zeros(d["obja"].shape)
    gP = np.zeros(d["objp"].shape)
    for i, s in enumerate(b):
        cy, cx = d["crop_pos"][s]
        gA[:, :, cy:cy + N, cx:cx + N] += dA[i]
        gP[:, :, cy:cy + N, cx:cx + N] += dP[i]
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe")}
    plan.adjoint_dldi(t, b, torch.tensor(dLdI, device=device), grads)
    torch.cuda.synchronize()
    assert rel(grads["obja"].cpu().numpy(), gA) < TOL_G
    assert rel(grads["objp"].cpu().numpy(), gP) < TOL_G
    gp = grads["probe"].cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], dprobe) < TOL_G


def orc_default_loss():
    return {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
            "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
            "loss_pacbed": {"state": False}, "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
            "loss_simlar": {"state": False}}


def test_bench_config_sample_vs_oracle():
    """The bench workload (c2: 256x256 scan, N=128, object 1033^2): one mini-batch of 32 vs oracle."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 256, 256, seed=0, meas="none")
    rng = np.random.default_rng(9)
    sel = rng.choice(256 * 256, 32, replace=False)      # 32 scan positions of the full scan
    meas = rng.random((32, 128, 128), dtype=np.float32)
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(60.0), shifts=pr.shifts[sel],
             crop_pos=pr.crop_pos[sel], H=pr.H, occu=pr.occu, meas=meas, shift_probes=True,
             loss_params=orc_default_loss())
    b = rng.permutation(32)
    terms, dp, g, _ = run_fused(d, device, [b])
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], [b], d["loss_params"])
    assert rel(dp, odps[0]) < TOL_DP
    np.testing.assert_allclose(terms[0], oterms[0], rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


def _c2_like(n_slow, n_fast, seed):
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, n_slow, n_fast, seed=seed)
    return dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(60.0), shifts=pr.shifts,
                crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True,
                loss_params=orc_default_loss())


@pytest.mark.parametrize("shift", [True, False])
def test_register_engine_ragged_batches_vs_oracle(shift):
    """N=128 single mode through k_fused3 (register-resident FFT): ragged mini-batches, more
    patterns than one per workgroup segment, gradients summed over batches vs the oracle."""
    device = dev()
    d = _c2_like(12, 12, seed=11)
    d["shift_probes"] = shift
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(4).permutation(S)
    cuts = [0, 5, 37, 38, 70, 101, 144]                   # ragged: 5, 32, 1, 32, 31, 43
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.25)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.25)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH


@pytest.mark.parametrize("shift,q1,n", [(True, 0.5, 144), (False, 0.5, 144), (True, 1.0, 144), (True, 0.5, 300)])
def test_register_engine_both_terms_vs_oracle(shift, q1, n):
    """loss_single + loss_poissn on k_fused3: a forward pass taking both terms' sums (MODE 1),
    k_finalize, then the full pass with c_single u_single + c_poissn u_poissn (MODE 2; the gather,
    probe and position sums then take coefficient 1).  Ragged mini-batches vs the oracle; n 300
    takes the binned (non-small-call) gather and tail."""
    device = dev()
    d = _c2_like(12 if n == 144 else 18, 12 if n == 144 else 17, seed=12)
    d["shift_probes"] = shift
    d["loss_params"]["loss_poissn"]["state"] = True
    d["loss_params"]["loss_single"]["dp_pow"] = q1
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(5).permutation(S)[:n]
    cuts = sorted({0, 5, 37, 38, 70, 101, n})
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.25, kernels=ks)
    assert ks["k_fused"][0] == 2 and "k_adjoint" not in ks, ks          # MODE 1 + MODE 2
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.25)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):   # (the probe: both terms' cancellation, TOL_G_BOTH as elsewhere)
        assert rel(g[k], og[k]) < (TOL_G_BOTH if k == "probe" else TOL_G), k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_register_engine_is_the_path_taken():
    """The c2-shaped call runs k_fused3 (its prep kernels show up in the per-kernel timing; a
    small call's table, object rows and bounding box are one k_small_prep launch, timed as
    k_pattern_table)."""
    device = dev()
    from ptyrad_amd.engine import LossConfig, batch_offsets
    d = _c2_like(8, 8, seed=2)
    plan = make_plan(d, device)
    t = tensors(d, device)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    batches = np.array_split(np.arange(64), 2)
    plan.profile_begin()
    plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                           LossConfig.from_loss_params(d["loss_params"]), grads)
    torch.cuda.synchronize()
    stats = plan.profile_end()
    assert "k_pattern_table" in stats and "k_fused" in stats and "k_obj_prep" not in stats, stats


@pytest.mark.parametrize("nz,shift", [(3, True), (2, False), (16, True)])
def test_multislice_register_engine_vs_oracle(nz, shift):
    """N=128, P=O=1, Nz slices through k_fused3ms (4·Nz FFTs per pattern, no recompute):
    ragged mini-batches vs the oracle, and the path is the multislice register engine."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, batch_offsets
    pr = syn.random_problem(128, 6, 7, Nz=nz, seed=20 + nz)
    d = dict(obja=pr.obja, objp=(pr.objp / nz).astype(np.float32), probe=pr.probe * np.float32(60.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=orc_default_loss())
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(5).permutation(S)
    cuts = [0, 9, 10, 30, S]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH
    plan = make_plan(d, device)
    t = tensors(d, device)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    plan.profile_begin()
    plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                           LossConfig.from_loss_params(d["loss_params"]), grads)
    torch.cuda.synchronize()
    stats = plan.profile_end()
    assert "k_pattern_table" in stats and "k_fused" in stats and "k_adjoint" not in stats, stats


@pytest.mark.parametrize("nz,shift,q1", [(3, True, 0.5), (2, False, 1.0), (4, True, 1.0)])
def test_multislice_register_engine_both_terms_vs_oracle(nz, shift, q1):
    """loss_single + loss_poissn on k_fused3ms: MODE 1 (forward through every slice, both terms'
    sums), k_finalize, MODE 2 (the full pass, coefficients applied) — vs the oracle."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 6, 7, Nz=nz, seed=40 + nz)
    lp = orc_default_loss()
    lp["loss_poissn"]["state"] = True
    lp["loss_single"]["dp_pow"] = q1
    d = dict(obja=pr.obja, objp=(pr.objp / nz).astype(np.float32), probe=pr.probe * np.float32(60.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=lp)
    perm = np.random.default_rng(7).permutation(42)
    cuts = [0, 9, 10, 30, 42]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    assert ks["k_fused"][0] == 2 and "k_adjoint" not in ks, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, lp, shift_probes=shift, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < (TOL_G_BOTH if k == "probe" else TOL_G), k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_multislice_call_split_at_batch_boundaries(monkeypatch):
    """A call larger than the register engine's slot capacity is split by engine.Plan at
    mini-batch boundaries: same loss terms and gradients as the oracle."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    monkeypatch.setenv("PTYX_OBJ_SCRATCH_MB", "8")      # 8 MiB / (3 x 128 KiB) = 21 patterns per call
    pr = syn.random_problem(128, 6, 7, Nz=3, seed=31)
    d = dict(obja=pr.obja, objp=(pr.objp / 3).astype(np.float32), probe=pr.probe * np.float32(60.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True,
             loss_params=orc_default_loss())
    perm = np.random.default_rng(6).permutation(42)
    cuts = [0, 9, 10, 30, 42]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    assert make_plan(d, device).register_capacity == 21
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"], grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_register_engine_band_of_tall_object_vs_oracle():
    """A rank's shard of a multi-GPU scan: patterns from a band of scan rows in a tall replicated
    object.  The bounding-box skip of k_obj_prep / k_obj_gather leaves every other row's
    gradient at exactly zero and matches the oracle inside the band."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, 24, 6, seed=41)
    band = np.arange(8 * 6, 12 * 6)                       # scan rows 8..11
    rng = np.random.default_rng(8)
    perm = rng.permutation(band)
    batches = [perm[:13], perm[13:]]
    d = dict(obja=pr.obja, objp=pr.objp, probe=pr.probe * np.float32(60.0), shifts=pr.shifts,
             crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=True,
             loss_params=orc_default_loss())
    terms, dp, g, _ = run_fused(d, device, batches)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    y0, y1 = pr.crop_pos[band, 0].min(), pr.crop_pos[band, 0].max() + 128
    assert not np.any(g["objp"][..., :y0, :]) and not np.any(g["objp"][..., y1:, :])


def test_calls_larger_than_max_patterns_are_split():
    """engine.Plan splits forward / adjoint calls into max_patterns pieces and fused calls at
    mini-batch boundaries: identical to one big plan's results (mixed state, general engine)."""
    device = dev()
    from ptyrad_amd.engine import LossConfig, batch_offsets
    d = load_case([c for c in CASES if "n32_p2o2z3" in c][0])
    S = d["shifts"].shape[0]
    idx = np.arange(S, dtype=np.int32)
    batches = np.array_split(np.random.default_rng(1).permutation(S), 4)
    out = []
    for mp in (S, 5):
        plan = make_plan(d, device, max_patterns=mp)
        t = tensors(d, device)
        dp = plan.forward(t, idx)
        grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
        terms = plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                                       LossConfig.from_loss_params(d["loss_params"]), grads)
        g2 = {k: torch.zeros_like(v) for k, v in grads.items()}
        plan.adjoint_dldi(t, idx, torch.ones_like(dp), g2)
        torch.cuda.synchronize()
        out.append((dp.cpu().numpy(), terms.cpu().numpy(), {k: v.cpu().numpy() for k, v in grads.items()},
                    {k: v.cpu().numpy() for k, v in g2.items()}))
    (dp0, t0, g0, a0), (dp1, t1, g1, a1) = out
    np.testing.assert_allclose(dp1, dp0, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(t1, t0, rtol=1e-6, atol=1e-9)
    for k in g0:
        assert rel(g1[k], g0[k]) < 1e-5, k
        assert rel(a1[k], a0[k]) < 1e-5, k


def _mixed_state(P, Nz, shift, seed, ns=6, nf=7):
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(128, ns, nf, P=P, Nz=Nz, seed=seed)
    return dict(obja=pr.obja, objp=(pr.objp / Nz).astype(np.float32), probe=pr.probe * np.float32(60.0),
                shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
                loss_params=orc_default_loss())


@pytest.mark.parametrize("P,Nz,shift,q", [(2, 1, True, 0.5), (3, 2, True, 0.5), (6, 6, True, 0.5), (2, 3, False, 0.5),
                                          (4, 1, False, 1.0), (2, 2, True, 0.7), (3, 2, True, "both"),
                                          (2, 1, False, "both"), (8, 2, True, 0.5)])
def test_mixed_state_register_engine_vs_oracle(P, Nz, shift, q):
    """N = 128, P probe modes, Nz slices through the mixed-state register engine (k_fmm_fwd →
    k_fmm_loss → k_fmm_adj, ptyx_fmm.hpp): ragged mini-batches vs the oracle — the tBL_WSe2 demo's
    6 × 6 geometry, single slice, broadcast probes, the general dp_pow form, and loss_single +
    loss_poissn together (both coefficients applied in k_fmm_adj)."""
    device = dev()
    d = _mixed_state(P, Nz, shift, seed=50 + 7 * P + Nz)
    if q == "both":
        d["loss_params"]["loss_poissn"]["state"] = True
    else:
        d["loss_params"]["loss_single"]["dp_pow"] = q
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(P + Nz).permutation(S)
    cuts = [0, 9, 10, 30, S]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    assert "k_fmm_fwd" in ks and "k_fmm_adj" in ks, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < (TOL_G_BOTH if q == "both" and k == "probe" else TOL_G), k
    if shift:
        assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_mixed_state_register_engine_poisson_and_binned_gather():
    """loss_poissn as the data term, and a call of 300 patterns (> the small-call limit: binned
    gather, summed-area-table window sums) with P = 2, Nz = 2: vs the oracle, bitwise repeatable."""
    device = dev()
    d = _mixed_state(2, 2, True, seed=77, ns=15, nf=20)
    d["loss_params"]["loss_single"]["state"] = False
    d["loss_params"]["loss_poissn"]["state"] = True
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(3).permutation(S)
    batches = np.array_split(perm, 10)
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, kernels=ks)
    assert "k_fmm_fwd" in ks and "k_obj_gather" in ks, ks
    terms2, _, g2, _ = run_fused(d, device, batches)
    assert np.array_equal(terms, terms2) and np.array_equal(g["obja"], g2["obja"]) and np.array_equal(g["probe"], g2["probe"])
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH


def test_mixed_state_call_split_at_batch_boundaries(monkeypatch):
    """A call larger than the far-field cache the mixed-state engine keeps its slots in is split
    by engine.Plan at mini-batch boundaries (prep reuse across the pieces): vs the oracle."""
    device = dev()
    monkeypatch.setenv("PTYX_FFC_MB", "20")   # 20 MiB / (3 · 3 planes · 128 KiB) = 17 patterns per call
    d = _mixed_state(3, 2, True, seed=81)
    perm = np.random.default_rng(6).permutation(42)
    cuts = [0, 9, 10, 25, 42]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    assert make_plan(d, device).register_capacity == 17
    ks = {}
    terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    assert ks["k_fmm_fwd"][0] >= 3, ks
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"], grad_scale=0.5)
    assert rel(dp, np.concatenate(odps)) < TOL_DP
    np.testing.assert_allclose(terms, oterms, rtol=TOL_TERMS, atol=1e-7)
    for k in ("obja", "objp", "probe"):
        assert rel(g[k], og[k]) < TOL_G, k
    assert rel(g["shifts"], og["shifts"]) < TOL_SH
