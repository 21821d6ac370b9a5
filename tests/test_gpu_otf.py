"""On-the-fly measurement padding / resampling on MI355X (models.py:81-86, :384-412).

ptyx_meas_gather against the reference's get_measurements (tests/golden/otf_*.npz, made by
make_golden.py --otf-only): rel-L2 ≤ 2e-6.  PtychoHIP with the options on — generic path and
fused path (call-local positions / shifts / gathered DPs) — against the reference's loss terms
(rtol 2e-5) and gradients (≤ 5e-5; positions ≤ 2e-4), and a fused call split into several
call-local groups against the oracle.
"""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from tests.test_gpu_model import init_vars, model_params
from tests.test_oracle_golden import otf_args, rel

pytestmark = pytest.mark.gpu
OTF = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "otf_*.npz")))
LRS = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
       "probe_pos_shifts": 5e-4}


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _model(z, device, max_patterns=None):
    from ptyrad_amd.models import PtychoHIP
    iv = init_vars(z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], z["H"], z["occu"], z["meas_small"])
    for k in ("on_the_fly_meas_padded", "on_the_fly_meas_padded_idx", "on_the_fly_meas_scale_factors"):
        if k in z.files:
            iv[k] = z[k]
    return PtychoHIP(iv, model_params(LRS), device=device, verbose=False, max_patterns=max_patterns)


def _check(model, z, terms):
    np.testing.assert_allclose(terms, z["loss_terms"], rtol=2e-5, atol=1e-7)
    assert rel(model.opt_obja.grad.cpu().numpy(), z["g_obja"]) < 5e-5
    assert rel(model.opt_objp.grad.cpu().numpy(), z["g_objp"]) < 5e-5
    assert rel(model.opt_probe.grad.cpu().numpy(), z["g_probe"]) < 5e-5
    assert rel(model.opt_probe_pos_shifts.grad.cpu().numpy(), z["g_shifts"]) < 2e-4


@pytest.mark.parametrize("path", OTF, ids=[os.path.basename(p)[:-4] for p in OTF])
def test_meas_gather_matches_reference(path):
    device = dev()
    z = np.load(path, allow_pickle=False)
    model = _model(z, device)
    got = model.get_measurements(z["batch"]).cpu().numpy()
    assert rel(got, z["meas_otf"]) < 2e-6
    with torch.no_grad():
        model.measurements = model.measurements.half()     # fp16 storage reads through the same kernel
    got16 = model.get_measurements(z["batch"]).cpu().numpy()
    assert rel(got16, z["meas_otf"]) < 2e-3


@pytest.mark.parametrize("path", OTF, ids=[os.path.basename(p)[:-4] for p in OTF])
def test_generic_and_fused_paths_match_reference(path):
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    z = np.load(path, allow_pickle=False)
    lp = json.loads(str(z["loss_params"]))
    model = _model(z, device)
    dp = model(z["batch"])
    assert rel(dp.detach().cpu().numpy(), z["dp"]) < 1e-5
    total, terms = CombinedLoss(lp, device=device)(dp, model.get_measurements(z["batch"]),
                                                   model._current_object_patches, model.omode_occu)
    total.backward()
    _check(model, z, np.array([float(t.detach()) for t in terms]))
    model = _model(z, device)
    total, terms = CombinedLoss(lp, device=device).fused(model, [z["batch"]])
    total.backward()
    _check(model, z, terms.detach().cpu().numpy()[0])


def test_fused_call_local_groups_vs_oracle():
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    z = np.load([p for p in OTF if "pad_resample" in p][0], allow_pickle=False)
    lp = json.loads(str(z["loss_params"]))
    model = _model(z, device, max_patterns=5)
    S = z["shifts"].shape[0]
    perm = np.random.default_rng(4).permutation(S)
    batches = [perm[:3], perm[3:5], perm[5:9], perm[9:10], perm[10:15]]
    total, terms = CombinedLoss(lp, device=device).fused(model, batches)
    total.backward()
    meas = orc.otf_measurements(z["meas_small"], np.arange(S), *otf_args(z))
    oterms, _, g = orc.forward_loss_grad(z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], z["H"],
                                         z["occu"], meas, batches, lp)
    np.testing.assert_allclose(terms.detach().cpu().numpy(), oterms, rtol=2e-5, atol=1e-7)
    assert rel(model.opt_objp.grad.cpu().numpy(), g["objp"]) < 5e-5
    assert rel(model.opt_probe_pos_shifts.grad.cpu().numpy(), g["shifts"]) < 2e-4


def test_on_the_fly_measurements_with_optimised_thickness_vs_oracle():
    """Call-local (on-the-fly) engine calls compose with the propagator gradient: optimised slice
    thickness (case 3) on 2 slices with resampled measurements, two mini-batches, vs the oracle."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    z = np.load([p for p in OTF if p.endswith("otf_n32_resample.npz")][0], allow_pickle=False)
    lp = json.loads(str(z["loss_params"]))
    iv = init_vars(z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], z["H"], z["occu"], z["meas_small"])
    iv["on_the_fly_meas_scale_factors"] = z["on_the_fly_meas_scale_factors"]
    model = PtychoHIP(iv, model_params({**LRS, "slice_thickness": 1e-3}), device=device, verbose=False)
    S = z["shifts"].shape[0]
    perm = np.random.default_rng(5).permutation(S)
    batches = [perm[:6], perm[6:11]]
    total, terms = CombinedLoss(lp, device=device).fused(model, batches)
    total.backward()
    Heff = model.get_propagators([0])[0].detach().cpu().numpy()
    meas = orc.otf_measurements(z["meas_small"], np.arange(S), *otf_args(z))
    oterms, _, g = orc.forward_loss_grad(z["obja"], z["objp"], z["probe"], z["shifts"], z["crop_pos"], Heff,
                                         z["occu"], meas, batches, lp)
    np.testing.assert_allclose(terms.detach().cpu().numpy(), oterms, rtol=2e-5, atol=1e-7)
    assert rel(model.opt_objp.grad.cpu().numpy(), g["objp"]) < 5e-5
    gdz, _ = orc.propagator_param_grads(g["H"], Heff, 2.0, np.zeros(2), 0.1494, float(model.lambd), 3)
    np.testing.assert_allclose(model.opt_slice_thickness.grad.item(), gdz, rtol=1e-2)
