"""Optional forward stages on MI355X: detector blur (models.py:379-380) and
object pre-blur (models.py:275-284).

* kernels: ptyx_obj_rblur / ptyx_blur_adjoint / ptyx_patch_gather / ptyx_patch_scatter_add vs the
  oracle (float64) — rel-L2 ≤ 1e-6 (fp32 taps and sums); the adjoint is checked against the
  oracle's explicit transpose, and by the dot-product identity <Bx, g> = <x, Bᵀg>;
* model: PtychoHIP with the stages on, generic path (model(idx) → CombinedLoss.forward →
  backward) and fused path (CombinedLoss.fused), against the reference's own outputs
  (tests/golden/n*_*blur.npz, made by make_golden.py --blur-only with torchvision's gaussian_blur
  restated, since torchvision is absent) — dp ≤ 1e-5, loss terms rtol 2e-5, gradients ≤ 5e-5
  (≤ 2e-4 for the position gradient, a sum of cancelling terms);
* ragged multi-batch fused calls split into several patch-stack groups vs the oracle.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from tests.test_gpu_model import init_vars, model_params
from tests.test_oracle_golden import blur_kw, load_case, rel

pytestmark = pytest.mark.gpu
BLUR_CASES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "n*blur.npz")))
LRS = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
       "probe_pos_shifts": 5e-4}


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("shape,ks,sigma", [((3, 33, 47), 5, 1.0), ((32, 128, 128), 5, 0.7), ((2, 9, 8), 7, 2.0),
                                            ((4, 64, 64), 3, 0.5), ((2, 100, 130), 9, 1.5), ((1, 40, 70), 15, 3.0),
                                            ((1, 17, 16), 1, 1.0)])
def test_blur_and_adjoint_vs_oracle(shape, ks, sigma):
    device = dev()
    from ptyrad_amd.stages import blur_planes
    rng = np.random.default_rng(1)
    x = rng.standard_normal(shape).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    xt, gt = torch.tensor(x, device=device), torch.tensor(g, device=device)
    bx = blur_planes(xt, sigma, ks).cpu().numpy()
    btg = blur_planes(gt, sigma, ks, adjoint=True).cpu().numpy()
    assert rel(bx, orc.gaussian_blur(x, sigma, ks)) < 1e-6
    assert rel(btg, orc.gaussian_blur_adjoint(g, sigma, ks)) < 1e-6
    lhs = float(np.sum(bx.astype(np.float64) * g))
    rhs = float(np.sum(x.astype(np.float64) * btg))
    assert abs(lhs - rhs) <= 1e-5 * max(abs(lhs), 1.0)


def test_patch_gather_scatter_vs_numpy():
    device = dev()
    from ptyrad_amd.stages import patch_gather, patch_scatter_add
    rng = np.random.default_rng(2)
    O, Nz, Ny, Nx, N = 2, 3, 70, 90, 32
    obj = rng.standard_normal((O, Nz, Ny, Nx)).astype(np.float32)
    cp = np.stack([rng.integers(0, Ny - N + 1, 40), rng.integers(0, Nx - N + 1, 40)], 1).astype(np.int32)
    idx = rng.permutation(40)[:17].astype(np.int32)
    t = lambda a: torch.tensor(a, device=device)   # noqa: E731
    p = patch_gather(t(obj), t(cp), t(idx), N).cpu().numpy()
    ref = np.stack([obj[:, :, cp[s, 0]:cp[s, 0] + N, cp[s, 1]:cp[s, 1] + N] for s in idx], 2)
    np.testing.assert_array_equal(p, ref)
    gp = rng.standard_normal(p.shape).astype(np.float32)
    gobj = torch.zeros((O, Nz, Ny, Nx), device=device)
    patch_scatter_add(t(gp), t(cp), t(idx), gobj)
    want = np.zeros((O, Nz, Ny, Nx), np.float64)
    for b, s in enumerate(idx):
        want[:, :, cp[s, 0]:cp[s, 0] + N, cp[s, 1]:cp[s, 1] + N] += gp[:, :, b]
    assert rel(gobj.cpu().numpy(), want) < 1e-6


def _model(d, device):
    from ptyrad_amd.models import PtychoHIP
    iv = init_vars(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"], d["occu"], d["meas"])
    mp = {**model_params(LRS), **blur_kw(d)}
    return PtychoHIP(iv, mp, device=device, verbose=False)


def _check_grads(model, d):
    assert rel(model.opt_obja.grad.cpu().numpy(), d["g_obja"]) < 5e-5
    assert rel(model.opt_objp.grad.cpu().numpy(), d["g_objp"]) < 5e-5
    assert rel(model.opt_probe.grad.cpu().numpy(), d["g_probe"]) < 5e-5
    assert rel(model.opt_probe_pos_shifts.grad.cpu().numpy(), d["g_shifts"]) < 2e-4


@pytest.mark.parametrize("path", BLUR_CASES, ids=[os.path.basename(p)[:-4] for p in BLUR_CASES])
def test_generic_path_with_stages_matches_reference(path):
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = load_case(path)
    model = _model(d, device)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    dp = model(d["batch"])
    assert rel(dp.detach().cpu().numpy(), d["dp"]) < 1e-5
    total, terms = loss_fn(dp, model.get_measurements(d["batch"]), model._current_object_patches, model.omode_occu)
    total.backward()
    np.testing.assert_allclose([float(t.detach()) if torch.is_tensor(t) else float(t) for t in terms], d["loss_terms"], rtol=2e-5, atol=1e-7)
    _check_grads(model, d)


@pytest.mark.parametrize("path", BLUR_CASES, ids=[os.path.basename(p)[:-4] for p in BLUR_CASES])
def test_fused_path_with_stages_matches_reference(path):
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = load_case(path)
    model = _model(d, device)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    total, terms = loss_fn.fused(model, [d["batch"]])
    total.backward()
    np.testing.assert_allclose(terms.detach().cpu().numpy()[0], d["loss_terms"], rtol=2e-5, atol=1e-7)
    _check_grads(model, d)


def test_preblur_fused_groups_vs_oracle():
    """Ragged mini-batches (each its own NRMSE normalisation) split over several patch-stack
    groups; gradients accumulate across groups."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = load_case([c for c in BLUR_CASES if "n32_p1o2z1_preblur" in c][0])
    model = _model(d, device)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    loss_fn.PREBLUR_GROUP = 5
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(7).permutation(S)
    batches = [perm[:3], perm[3:7], perm[7:8], perm[8:14]]
    total, terms = loss_fn.fused(model, batches)
    total.backward()
    oterms, _, g = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                         d["occu"], d["meas"], batches, d["loss_params"], shift_probes=True,
                                         **blur_kw(d))
    np.testing.assert_allclose(terms.detach().cpu().numpy(), oterms, rtol=2e-5, atol=1e-7)
    assert rel(model.opt_obja.grad.cpu().numpy(), g["obja"]) < 5e-5
    assert rel(model.opt_objp.grad.cpu().numpy(), g["objp"]) < 5e-5
    gp = model.opt_probe.grad.cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], g["probe"]) < 5e-5


def test_recon_step_with_stages_runs_on_device():
    """recon_step (Adam) with both stages on: finite losses that decrease over 3 iterations."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.reconstruction import create_optimizer, recon_step
    d = load_case([c for c in BLUR_CASES if "bothblur" in c][0])
    model = _model(d, device)
    opt = create_optimizer(model.optimizer_params, model.optimizable_params)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    S = d["shifts"].shape[0]
    batches = np.array_split(np.arange(S), 3)
    for it in range(1, 4):
        recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False)
    hist = np.array([v for _, v in model.loss_iters])
    assert np.all(np.isfinite(hist)) and hist[-1] < hist[0]


PACBED = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "n*pacbed*.npz")) +
                glob.glob(os.path.join(os.path.dirname(__file__), "golden", "n*simlar*.npz")))


@pytest.mark.parametrize("path", PACBED, ids=[os.path.basename(p)[:-4] for p in PACBED])
@pytest.mark.parametrize("fused", [True, False], ids=["fused", "generic"])
def test_loss_pacbed_matches_reference(path, fused):
    """loss_pacbed (losses.py:77-89): fused path = engine call with dp_out → ptyx_loss_pacbed →
    ptyx_adjoint_dldi; generic path = torch loss on the engine's dp.  Reference fixtures from
    make_golden.py --pacbed-only (one with loss_single + loss_sparse, one with pacbed alone).
    Also loss_simlar (losses.py:106-141; patches blurred by the HIP gaussian_blur), whose
    fused call runs per mini-batch (make_golden.py --simlar-only)."""
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = load_case(path)
    model = _model(d, device)
    loss_fn = CombinedLoss(d["loss_params"], device=device)
    if fused:
        total, terms = loss_fn.fused(model, [d["batch"]])
        terms = terms.detach().cpu().numpy()[0]
    else:
        dp = model(d["batch"])
        total, terms = loss_fn(dp, model.get_measurements(d["batch"]), model._current_object_patches,
                               model.omode_occu)
        terms = np.array([float(t.detach()) for t in terms])
    total.backward()
    np.testing.assert_allclose(terms, d["loss_terms"], rtol=2e-5, atol=1e-7)
    _check_grads(model, d)


def test_loss_pacbed_multi_batch_vs_oracle():
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = load_case([c for c in PACBED if "n32_p2o1z2_pacbed" in c][0])
    model = _model(d, device)
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(11).permutation(S)
    batches = [perm[:5], perm[5:6], perm[6:13]]
    total, terms = CombinedLoss(d["loss_params"], device=device).fused(model, batches)
    total.backward()
    oterms, _, g = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                         d["occu"], d["meas"], batches, d["loss_params"])
    np.testing.assert_allclose(terms.detach().cpu().numpy(), oterms, rtol=2e-5, atol=1e-7)
    assert rel(model.opt_objp.grad.cpu().numpy(), g["objp"]) < 5e-5
    gp = model.opt_probe.grad.cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], g["probe"]) < 5e-5



SIMLAR = [c for c in PACBED if "simlar" in c]


@pytest.mark.parametrize("variant", ["fixture", "area_phase", "chunked_amp"])
def test_loss_simlar_beside_engine_matches_per_batch_path(variant):
    """loss_simlar with several mini-batches: the data terms in one engine call and loss_simlar
    vectorised over the call (CombinedLoss._simlar_terms: HIP patch gather + blur, per-batch
    normalisation) against the per-mini-batch generic path (torch loss_simlar on each mini-batch's
    patches, losses.py:106-141) — terms and gradients, through fused() and fused_into()."""
    import json
    import torch
    device = dev()
    from ptyrad_amd.losses import CombinedLoss
    d = dict(load_case(SIMLAR[0]))
    lp = json.loads(json.dumps(d["loss_params"]))
    if variant == "area_phase":
        lp["loss_simlar"].update(obj_type="phase", scale_factor=[1.0, 0.5, 0.5], blur_std=0)
    elif variant == "chunked_amp":
        lp["loss_simlar"].update(obj_type="amplitude", blur_std=1.5)
    S = d["shifts"].shape[0]
    perm = np.random.default_rng(5).permutation(S)
    batches = [perm[:5], perm[5:6], perm[6:13], perm[13:]]

    def grads(m):
        return {k: getattr(m, "opt_" + k).grad.detach().cpu().numpy().copy() for k in ("obja", "objp", "probe")}

    ref_model = _model(d, device)
    ref = CombinedLoss(lp, device=device)
    total, rterms = ref._per_batch(ref_model, batches)
    total.backward()
    g_ref = grads(ref_model)
    rterms = rterms.detach().cpu().numpy()
    assert np.all(np.isfinite(rterms)) and np.all(rterms[:, 4] > 0)

    loss = CombinedLoss(lp, device=device)
    if variant == "chunked_amp":
        loss.SIMLAR_PATCH_BYTES = 4 * 2 * 2 * 32 * 32 * 3   # 3 patterns a chunk: chunks cut mini-batches
    model = _model(d, device)
    total, terms = loss.fused(model, batches)
    total.backward()
    np.testing.assert_allclose(terms.detach().cpu().numpy(), rterms, rtol=2e-5, atol=1e-7)
    g = grads(model)
    for k in g:
        assert rel(g[k], g_ref[k]) < 2e-5, k

    model2 = _model(d, device)
    for k in ("obja", "objp", "probe"):
        p = getattr(model2, "opt_" + k)
        p.grad = torch.zeros_like(p)
    terms2 = loss.fused_into(model2, batches, grad_scale=0.5)
    np.testing.assert_allclose(terms2.detach().cpu().numpy(), rterms, rtol=2e-5, atol=1e-7)
    g2 = grads(model2)
    for k in g2:
        assert rel(g2[k], 0.5 * g_ref[k]) < 2e-5, k
