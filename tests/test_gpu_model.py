"""PtychoHIP / CombinedLoss / recon_step on the GPU vs the reference's golden trajectories.

north_star: reconstructed object RMS error vs the reference < 1e-5 (3 Adam iterations, fixed
batches, grad_accumulation 1 and 2).  Also the generic path: model(indices) -> torch loss ->
backward through ptyx_adjoint_dldi.
"""
import glob
import json
import os

import numpy as np
import pytest
import torch

from tests.test_oracle_golden import CASES, load_case, rel

pytestmark = pytest.mark.gpu
TRAJ = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "traj_*.npz")))


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def model_params(lrs):
    up = {k: {"start_iter": (1 if v else None), "lr": v} for k, v in lrs.items()}
    return {"detector_blur_std": None, "obj_preblur_std": None, "update_params": up,
            "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}


def init_vars(obja, objp, probe, shifts, crop_pos, H, occu, meas):
    return {"obja": obja, "objp": objp, "obj": obja * np.exp(1j * objp), "probe": probe,
            "probe_pos_shifts": shifts, "omode_occu": occu, "H": H, "measurements": meas,
            "crop_pos": crop_pos, "N_scan_slow": 4, "N_scan_fast": 4, "slice_thickness": 2.0,
            "dx": 0.1494, "dk": 0.05, "lambd": 0.04, "obj_tilts": np.zeros((1, 2), np.float32)}


@pytest.mark.parametrize("path", TRAJ, ids=[os.path.basename(p)[:-4] for p in TRAJ])
def test_recon_step_trajectory_matches_reference(path):
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from ptyrad_amd.reconstruction import create_optimizer, recon_step
    z = np.load(path, allow_pickle=False)
    lrs = json.loads(str(z["lrs"]))
    iv = init_vars(z["init_obja"], z["init_objp"], z["init_probe"], z["init_shifts"], z["crop_pos"], z["H"],
                   z["occu"], z["meas"])
    model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
    opt = create_optimizer(model.optimizer_params, model.optimizable_params)
    loss_fn = CombinedLoss(json.loads(str(z["loss_params"])), device=device)
    batches = np.split(z["batches"], np.cumsum(z["batch_sizes"])[:-1])
    cp = json.loads(str(z["constraint_params"])) if "constraint_params" in z.files else None
    cfn = None
    if cp is not None:   # the reference ran its CombinedConstraint: run the on-device one
        from ptyrad_amd.constraints import CombinedConstraint
        cfn = CombinedConstraint(cp, device=device, verbose=False)
    for it in range(1, int(z["niter"]) + 1):
        recon_step(batches, int(z["grad_accumulation"]), model, opt, loss_fn, cfn, it, verbose=False)
    for k, ref in (("opt_obja", z["final_obja"]), ("opt_objp", z["final_objp"])):
        got = getattr(model, k).detach().cpu().numpy().astype(np.float64)
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        assert rms < 1e-5, (k, rms)
    prb = torch.view_as_complex(model.opt_probe.detach()).cpu().numpy()
    assert rel(prb, z["final_probe"]) < 1e-5
    hist = np.array([v for _, v in model.loss_iters])
    np.testing.assert_allclose(hist, z["loss_hist"].sum(1), rtol=1e-5)


def test_generic_autograd_path_matches_reference():
    """model(batch) -> CombinedLoss.forward (torch) -> backward (HIP adjoint for dp, torch for patches)."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    d = load_case([c for c in CASES if "n32_p2o2z3" in c][0])
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 5e-4}
    iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"], d["meas"])
    model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    dp = model(d["batch"])
    total, terms = loss_fn(dp, model.get_measurements(d["batch"]), model._current_object_patches, model.omode_occu)
    total.backward()
    np.testing.assert_allclose([float(t.detach()) if torch.is_tensor(t) else float(t) for t in terms], d["loss_terms"], rtol=2e-5, atol=1e-7)
    assert rel(model.opt_obja.grad.cpu().numpy(), d["g_obja"]) < 5e-5
    assert rel(model.opt_objp.grad.cpu().numpy(), d["g_objp"]) < 5e-5
    gp = model.opt_probe.grad.cpu().numpy()
    assert rel(gp, d["g_probe"]) < 5e-5
    assert rel(model.opt_probe_pos_shifts.grad.cpu().numpy(), d["g_shifts"]) < 2e-4


def test_fused_loss_equals_generic_loss():
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    d = load_case([c for c in CASES if "n64_p3o1z1" in c][0])
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 5e-4}
    iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"], d["meas"])
    model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    total, terms = loss_fn.fused(model, [d["batch"]])
    total.backward()
    np.testing.assert_allclose(terms.cpu().numpy()[0], d["loss_terms"], rtol=1e-5, atol=1e-7)
    assert rel(model.opt_objp.grad.cpu().numpy(), d["g_objp"]) < 5e-5


def test_invalid_indices_raise():
    device = dev()
    from ptyrad_amd.models import PtychoHIP
    d = load_case([c for c in CASES if "n32_p1o1z1" in c][0])
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 5e-4}
    iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"], d["meas"])
    model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
    with pytest.raises(IndexError):
        model(np.array([0, 999]))
    with pytest.raises(ValueError):
        PtychoHIP(iv, {**model_params(lrs), "detector_blur_std": -1.0}, device=device, verbose=False)


def test_fixed_global_tilt_propagator():
    """Fixed non-zero global tilt (models.py:346-349, case 2B) on 3 slices: PtychoHIP builds the
    tilted propagator itself from (H, obj_tilts, slice_thickness, dx) and matches the reference's
    dp, loss terms and gradients."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    d = load_case([c for c in CASES if "tilt" in c][0])
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 5e-4}
    iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H_untilted"], d["occu"],
                   d["meas"])
    iv.update(obj_tilts=d["obj_tilts"], slice_thickness=float(d["slice_thickness"]), dx=float(d["dx"]))
    model = PtychoHIP(iv, model_params(lrs), device=device, verbose=False)
    assert rel(model.get_propagators([0])[0].cpu().numpy(), d["H"]) < 1e-6
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    dp = model(d["batch"])
    assert rel(dp.detach().cpu().numpy(), d["dp"]) < 1e-5
    total, terms = loss_fn.fused(model, [d["batch"]])
    total.backward()
    np.testing.assert_allclose(terms.cpu().numpy()[0], d["loss_terms"], rtol=1e-5, atol=1e-7)
    assert rel(model.opt_objp.grad.cpu().numpy(), d["g_objp"]) < 5e-5
    assert rel(model.opt_obja.grad.cpu().numpy(), d["g_obja"]) < 5e-5
    assert rel(model.opt_probe.grad.cpu().numpy(), d["g_probe"]) < 5e-5
    S = d["shifts"].shape[0]
    with pytest.raises(ValueError):   # per-position tilts must have one row per scan position
        PtychoHIP({**iv, "obj_tilts": np.tile(d["obj_tilts"], (S + 1, 1))},
                  model_params({**lrs, "slice_thickness": 1e-3}), device=device, verbose=False)
