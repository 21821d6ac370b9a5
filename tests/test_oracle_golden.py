"""Pin the oracle (oracle/ptyx_oracle.py) to golden vectors produced by the PtyRAD reference.

Fixtures: tests/golden/*.npz, made by tests/golden/make_golden.py (reference autograd,
fp32, CPU).  Tolerance: the reference itself runs in fp32, so the fp64 oracle is compared
with relative-L2 error ≤ 2e-6 on dp, ≤ 1e-6 relative on loss terms, ≤ 5e-5 on the object /
probe gradients and ≤ 1e-4 on the position gradient (a sum of cancelling terms, where the
reference's own fp32 rounding is largest).
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle import ptyx_oracle as orc

CASES = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "n*.npz")))


def rel(a, b):
    a = np.asarray(a, np.complex128 if np.iscomplexobj(a) or np.iscomplexobj(b) else np.float64)
    b = np.asarray(b, a.dtype)
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def load_case(path):
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    if "meas_f16" in d:
        S, n = d["shifts"].shape[0], d["probe"].shape[-1]
        meas = np.zeros((S, n, n), np.float32)
        meas[d["batch"]] = d["meas_f16"].astype(np.float32)
        d["meas"] = meas
    d["loss_params"] = json.loads(str(d["loss_params"]))
    return d


def dp_tolerance(d):
    """The fp32 reference's own dp rounding grows with the slice count (2·Nz chained FFTs): 2e-6
    up to Nz = 6, proportionally above (n128_p1o1z16_c4: 2.5e-6 against the fp64 oracle)."""
    return 2e-6 * max(1.0, d["obja"].shape[1] / 6.0)


def tilt_kw(d):
    """Per-position tilt arguments of a tilt_type 'each' fixture (make_golden.py --each-only)."""
    if "tilt_each" not in d:
        return {}
    return {"tilts": d["obj_tilts"], "dx": float(d["dx"]), "dz": float(d["slice_thickness"])}


def blur_kw(d):
    """Optional-stage options a fixture was made with (make_golden.py --blur-only)."""
    return {k: float(d[k]) for k in ("detector_blur_std", "obj_preblur_std") if k in d}


def test_blur_adjoint_is_transpose():
    """gaussian_blur_adjoint = the transpose of gaussian_blur (explicit matrix, reflect edges)."""
    rng = np.random.default_rng(5)
    shape = (7, 9)
    n = shape[0] * shape[1]
    M = np.stack([orc.gaussian_blur(np.eye(n)[k].reshape(shape), 0.9).ravel() for k in range(n)], 1)
    y = rng.standard_normal(n)
    np.testing.assert_allclose(orc.gaussian_blur_adjoint(y.reshape(shape), 0.9).ravel(), M.T @ y, atol=1e-14)


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_oracle_matches_reference(path):
    d = load_case(path)
    terms, dps, g = orc.forward_loss_grad(
        d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"],
        d["meas"], [d["batch"]], d["loss_params"], shift_probes=bool(d["shift_probes"]), **blur_kw(d),
        **tilt_kw(d))
    dp = dps[0]
    tol_dp = dp_tolerance(d)
    if "dp" in d:
        assert rel(dp, d["dp"]) < tol_dp
    else:
        assert rel(dp[:4], d["dp_head"]) < tol_dp
        assert rel(dp.reshape(len(dp), -1).sum(1), d["dp_sums"]) < tol_dp
    np.testing.assert_allclose(terms[0], d["loss_terms"], rtol=1e-6, atol=1e-8)
    assert rel(g["obja"], d["g_obja"]) < 5e-5
    assert rel(g["objp"], d["g_objp"]) < 5e-5
    gp = d["g_probe"][..., 0] + 1j * d["g_probe"][..., 1]
    assert rel(g["probe"], gp) < 5e-5
    if d["shift_probes"]:
        assert rel(g["shifts"], d["g_shifts"]) < 1e-4
    if "tilt_each" in d and "g_obj_tilts" in d:
        assert rel(g["tilts"], d["g_obj_tilts"]) < 1e-4


TRAJ = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "traj_*.npz")))


def oracle_trajectory(z, grad_fn=None):
    """Replays reference recon_step (reconstruction.py:658-781, Adam branch) with oracle grads."""
    lp = json.loads(str(z["loss_params"]))
    lrs = json.loads(str(z["lrs"]))
    sizes = z["batch_sizes"]
    flat = z["batches"]
    batches = np.split(flat, np.cumsum(sizes)[:-1])
    ga = int(z["grad_accumulation"])
    params = {"obja": z["init_obja"].copy(), "objp": z["init_objp"].copy(),
              "probe": np.stack([z["init_probe"].real, z["init_probe"].imag], -1).astype(np.float32),
              "probe_pos_shifts": z["init_shifts"].copy()}
    state, t = {}, 0
    grad_fn = grad_fn or (lambda prm, b, scale: orc.forward_loss_grad(
        prm["obja"], prm["objp"], prm["probe"][..., 0] + 1j * prm["probe"][..., 1],
        prm["probe_pos_shifts"], z["crop_pos"], z["H"], z["occu"], z["meas"], [b], lp,
        shift_probes=True, grad_scale=scale)[2])
    cp = json.loads(str(z["constraint_params"])) if "constraint_params" in z.files else None
    for it in range(1, int(z["niter"]) + 1):
        acc = None
        for bi, b in enumerate(batches):
            g = grad_fn(params, b, 1.0 / ga)
            g = {"obja": g["obja"], "objp": g["objp"],
                 "probe": np.stack([g["probe"].real, g["probe"].imag], -1),
                 "probe_pos_shifts": g["shifts"]}
            acc = g if acc is None else {k: acc[k] + g[k] for k in acc}
            if (bi + 1) % ga == 0 or bi + 1 == len(batches):
                t += 1
                orc.adam_step(params, {k: v.astype(np.float32) for k, v in acc.items()}, state, lrs, t)
                acc = None
        if cp is not None:   # CombinedConstraint after the iteration (reconstruction.py:776-780)
            apply_constraint_oracle(params, cp, float(z["probe_int_sum"]), it)
    return params


def apply_constraint_oracle(params, cp, probe_int_sum, niter):
    from oracle import constraints_oracle as co
    st = {"obja": params["obja"], "objp": params["objp"], "probe_int_sum": probe_int_sum,
          "probe": params["probe"][..., 0] + 1j * params["probe"][..., 1]}
    out = co.combined(cp, st, niter)
    params["obja"] = out["obja"].astype(np.float32)
    params["objp"] = out["objp"].astype(np.float32)
    params["probe"] = np.stack([out["probe"].real, out["probe"].imag], -1).astype(np.float32)


@pytest.mark.parametrize("path", TRAJ, ids=[os.path.basename(p)[:-4] for p in TRAJ])
def test_oracle_trajectory_matches_reference(path):
    """3 reference iterations (Adam, fixed batches): object RMS error vs reference < 1e-5."""
    z = np.load(path, allow_pickle=False)
    p = oracle_trajectory(z)
    for k, ref in (("obja", z["final_obja"]), ("objp", z["final_objp"])):
        rms = float(np.sqrt(np.mean((p[k].astype(np.float64) - ref) ** 2)))
        assert rms < 1e-5, (k, rms)
    prb = p["probe"][..., 0] + 1j * p["probe"][..., 1]
    assert rel(prb, z["final_probe"]) < 1e-5


PROP = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "n*_opt*.npz"))
              if "each" not in p)


def prop_case(d):
    """get_propagators case of a --prop-only fixture: 1 (tilts + dz), 2 (2A: tilts), 3 (dz)."""
    lr = json.loads(str(d["prop_lr"]))
    return 1 if len(lr) == 2 else (2 if "obj_tilts" in lr else 3)


@pytest.mark.parametrize("path", PROP, ids=[os.path.basename(p)[:-4] for p in PROP])
def test_oracle_propagator_gradient_matches_reference(path):
    """dL/dH from the oracle's adjoint, chained to dz / tilts, equals the reference's autograd
    gradients of opt_slice_thickness / opt_obj_tilts (models.py:339-356)."""
    d = load_case(path)
    _, _, g = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                    d["occu"], d["meas"], [d["batch"]], d["loss_params"],
                                    shift_probes=bool(d["shift_probes"]))
    case = prop_case(d)
    gdz, gt = orc.propagator_param_grads(g["H"], d["H"], float(d["slice_thickness"]),
                                         d["obj_tilts"][0].astype(np.float64), float(d["dx"]), float(d["lambd"]), case)
    if case in (1, 3):   # the f32 reference's own floor: dz·k phase cancellation (k = 2π/λ ≈ 150 Å⁻¹)
        np.testing.assert_allclose(gdz, float(d["g_slice_thickness"]), rtol=5e-3)
    if case in (1, 2):
        np.testing.assert_allclose(gt, d["g_obj_tilts"][0], rtol=2e-3, atol=1e-3 * np.abs(d["g_obj_tilts"]).max())


OTF = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "otf_*.npz")))


def otf_args(z):
    return (z["on_the_fly_meas_padded"] if "on_the_fly_meas_padded" in z else None,
            z["on_the_fly_meas_padded_idx"] if "on_the_fly_meas_padded_idx" in z else None,
            z["on_the_fly_meas_scale_factors"] if "on_the_fly_meas_scale_factors" in z else None)


@pytest.mark.parametrize("path", OTF, ids=[os.path.basename(p)[:-4] for p in OTF])
def test_oracle_on_the_fly_measurements_match_reference(path):
    """get_measurements with on-the-fly padding / resampling (models.py:384-412), and the
    loss / gradients computed on those DPs, against the reference."""
    z = np.load(path, allow_pickle=False)
    got = orc.otf_measurements(z["meas_small"], z["batch"], *otf_args(z))
    assert rel(got, z["meas_otf"]) < 2e-6
    S = z["shifts"].shape[0]
    meas = orc.otf_measurements(z["meas_small"], np.arange(S), *otf_args(z))
    terms, dps, g = orc.forward_loss_grad(z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], z["H"],
                                          z["occu"], meas, [z["batch"]], json.loads(str(z["loss_params"])))
    assert rel(dps[0], z["dp"]) < 2e-6
    np.testing.assert_allclose(terms[0], z["loss_terms"], rtol=1e-6, atol=1e-8)
    assert rel(g["obja"], z["g_obja"]) < 5e-5
    assert rel(g["objp"], z["g_objp"]) < 5e-5
    gp = z["g_probe"][..., 0] + 1j * z["g_probe"][..., 1]
    assert rel(g["probe"], gp) < 5e-5


def test_oracle_dz_gradient_with_per_position_tilts():
    """Case 1 with tilt_type 'each' (models.py:339-344): dL/d(dz) = Re Σ conj(g_H) i Kz H (base H =
    exp(i dz Kz)) + the tilt ramps' part, against the reference's autograd (rtol 1e-2: the dz·k
    phase cancellation floor of the f32 reference, see test_oracle_propagator_gradient_*)."""
    d = load_case(os.path.join(os.path.dirname(__file__), "golden", "n32_p2o1z3_opttiltdzeach.npz"))
    _, _, g = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"],
                                    d["meas"], [d["batch"]], d["loss_params"], **tilt_kw(d))
    gdz_base, _ = orc.propagator_param_grads(g["H_base"], d["H"], float(d["slice_thickness"]), np.zeros(2),
                                             float(d["dx"]), float(d["lambd"]), 3)
    np.testing.assert_allclose(gdz_base + g["dz_ramp"], float(d["g_slice_thickness"]), rtol=1e-2)

