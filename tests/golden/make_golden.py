"""Generate golden fixtures for the ptyx hot path by running the PtyRAD reference itself.

Run here (build container) only:  python tests/golden/make_golden.py
It imports /root/reference/src (read-only) via refimport.py, builds the
reference ``PtychoAD`` (src/ptyrad/models.py:70) straight from an
``init_variables`` dict, evaluates ``CombinedLoss`` (src/ptyrad/losses.py:143)
and ``loss.backward()`` (autograd), and stores inputs + outputs as .npz:

  inputs : obja, objp (O,Nz,Ny,Nx) f32 [the model's own abs/angle of obj],
           probe (P,N,N) c64, shifts (S,2) f32, crop_pos (S,2) i32, H (N,N) c64,
           occu (O,) f32, meas (S,N,N) f32 (only batch rows are non-zero),
           batch (B,) i64, loss_params (json), shift_probes (bool)
  outputs: dp (B,N,N) f32 (or dp_head + dp_sums for the big case), loss_terms (5,),
           loss_total, g_obja, g_objp, g_probe (P,N,N,2), g_shifts (S,2)

and a 3-iteration recon_step trajectory (src/ptyrad/reconstruction.py:658)
with fixed batches, Adam, and a no-op constraint (plus one with the schema-default
CombinedConstraint, constraints.py:227-246).  The data written are
inputs and outputs only; no reference source is copied.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import refimport  # noqa: E402
from refimport import import_reference  # noqa: E402
from ptyrad_amd import synthetic as syn  # noqa: E402

models, losses, reconstruction = import_reference()

DEFAULT_LOSS = {
    "loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
    "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
    "loss_pacbed": {"state": False, "weight": 0.5, "dp_pow": 0.2},
    "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
    "loss_simlar": {"state": False, "weight": 0.1, "obj_type": "both",
                    "scale_factor": [1.0, 1.0, 1.0], "blur_std": 1.0},
}


BLUR = {"detector_blur_std": None, "obj_preblur_std": None}   # set by --blur-only cases
PROP_LR = {}   # optimised obj_tilts / slice_thickness lrs, set by --prop-only cases


def model_params(shift_lr=5e-4):
    up = {
        "obja": {"start_iter": 1, "lr": 5e-4},
        "objp": {"start_iter": 1, "lr": 5e-4},
        "obj_tilts": {"start_iter": None, "lr": 0.0},
        "slice_thickness": {"start_iter": None, "lr": 0.0},
        "probe": {"start_iter": 1, "lr": 1e-4},
        "probe_pos_shifts": {"start_iter": 1 if shift_lr else None, "lr": shift_lr},
    }
    for k, lr in PROP_LR.items():
        up[k] = {"start_iter": 1, "lr": lr}
    return {"detector_blur_std": BLUR["detector_blur_std"], "obj_preblur_std": BLUR["obj_preblur_std"],
            "update_params": up,
            "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}


def init_variables(obja, objp, probe, H, occu, crop_pos, shifts, meas, n_slow, n_fast, dz=2.0, tilts=None):
    lam = syn.electron_wavelength(syn.KV)
    n = probe.shape[-1]
    return {
        "obj": (obja * np.exp(1j * objp)).astype(np.complex64),
        "obj_tilts": np.zeros((1, 2), np.float32) if tilts is None else np.asarray(tilts, np.float32).reshape(-1, 2),
        "slice_thickness": np.float32(dz),
        "probe": probe.astype(np.complex64),
        "probe_pos_shifts": shifts.astype(np.float32),
        "omode_occu": occu.astype(np.float32),
        "H": H.astype(np.complex64),
        "measurements": meas.astype(np.float32),
        "N_scan_slow": n_slow, "N_scan_fast": n_fast,
        "crop_pos": crop_pos.astype(np.int32),
        "dx": np.float32(syn.DX_ANG), "dk": np.float32(1.0 / (syn.DX_ANG * n)),
        "lambd": np.float32(lam), "scan_affine": None,
    }


def build_model(iv, shift_lr):
    torch.manual_seed(0)
    return models.PtychoAD(iv, model_params(shift_lr), device="cpu", verbose=False)


def make_inputs(n, P, O, Nz, n_slow, n_fast, seed, defocus=40.0, pstd=0.2):
    rng = np.random.default_rng(seed)
    scan = syn.raster_scan(n_slow, n_fast, n, seed=seed)
    probe = syn.mixed_probe(syn.stem_probe(n, defocus=defocus), P)
    probe = probe * np.float32(np.sqrt(n * n * 0.5))   # intensity scale ~ DP sum
    H = syn.fresnel_propagator(n, syn.DX_ANG, 2.0)
    occu = syn.omode_occupancy(O)
    shape = (O, Nz) + scan.obj_shape
    obja = (1.0 + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    objp = (pstd * rng.standard_normal(shape)).astype(np.float32)
    gta = (1.0 + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    gtp = (pstd * rng.standard_normal(shape)).astype(np.float32)
    return scan, probe, H, occu, obja, objp, gta, gtp


def simulate_meas(scan, probe, H, occu, gta, gtp, shift_lr, tilts=None):
    """Measurements = the reference forward model on a different (ground-truth) object."""
    n = probe.shape[-1]
    S = scan.crop_pos.shape[0]
    iv = init_variables(gta, gtp, probe, H, occu, scan.crop_pos, scan.shifts,
                        np.zeros((S, n, n), np.float32), scan.n_slow, scan.n_fast, tilts=tilts)
    m = build_model(iv, shift_lr)
    with torch.no_grad():
        dp = m(np.arange(S)).numpy()
    return dp.astype(np.float32)


def run_case(name, n, P, O, Nz, n_slow, n_fast, B, seed, shift_lr=5e-4, loss_params=None,
             big=False, tilts=None, f16_storage=False):
    loss_params = loss_params or DEFAULT_LOSS
    scan, probe, H, occu, obja, objp, gta, gtp = make_inputs(n, P, O, Nz, n_slow, n_fast, seed)
    meas = simulate_meas(scan, probe, H, occu, gta, gtp, shift_lr, tilts=tilts)
    S = scan.crop_pos.shape[0]
    batch = np.random.default_rng(seed + 100).permutation(S)[:B].astype(np.int64)
    if big:  # keep the fixture small: only the batch rows of meas, stored as f16 and used as such
        keep = np.zeros_like(meas)
        keep[batch] = meas[batch]
        meas = keep.astype(np.float16).astype(np.float32)
    iv = init_variables(obja, objp, probe, H, occu, scan.crop_pos, scan.shifts, meas,
                        scan.n_slow, scan.n_fast, tilts=tilts)
    model = build_model(iv, shift_lr)
    loss_fn = losses.CombinedLoss(loss_params, device="cpu")
    dp = model(batch)
    mdp = model.get_measurements(batch)
    total, terms = loss_fn(dp, mdp, model._current_object_patches, model.omode_occu)
    total.backward()

    def g(t):
        return None if t.grad is None else t.grad.detach().numpy().copy()

    out = dict(
        obja=model.opt_obja.detach().numpy(), objp=model.opt_objp.detach().numpy(),
        probe=torch.view_as_complex(model.opt_probe.detach()).numpy(),
        shifts=model.opt_probe_pos_shifts.detach().numpy(), crop_pos=scan.crop_pos,
        H=(model.H.numpy() if tilts is None else model.H_fixed_tilts_full[0].detach().numpy()),
        occu=model.omode_occu.numpy(),
        batch=batch, loss_params=json.dumps(loss_params), shift_probes=bool(model.shift_probes),
        loss_terms=np.array([float(t) for t in terms], np.float64),
        loss_total=np.float64(float(total)),
        g_obja=g(model.opt_obja), g_objp=g(model.opt_objp), g_probe=g(model.opt_probe),
    )
    gs = g(model.opt_probe_pos_shifts)
    out["g_shifts"] = gs if gs is not None else np.zeros_like(out["shifts"])
    dpn = dp.detach().numpy()
    if big:
        out["meas_f16"] = meas[batch].astype(np.float16)
        out["dp_head"] = dpn[:4]
        out["dp_sums"] = dpn.reshape(B, -1).astype(np.float64).sum(1)
        if f16_storage:   # c5: the engine reads these DPs from f16 storage (same values)
            out["meas_storage_f16"] = True
    else:
        out["meas"] = meas
        out["dp"] = dpn
    if tilts is not None:   # fixed global tilt (models.py:346-349, case 2B): H above is the tilted one
        out.update(H_untilted=model.H.numpy(), obj_tilts=np.asarray(tilts, np.float32).reshape(-1, 2),
                   slice_thickness=np.float32(model.opt_slice_thickness.item()), dx=np.float32(model.dx.item()),
                   lambd=np.float32(model.lambd.item()))
    for k, v in BLUR.items():
        if v:
            out[k] = np.float32(v)
    if PROP_LR:   # optimised propagator (models.py:339-356 cases 1 / 2A / 3): H is the untilted one
        out.update(H=model.get_propagators(np.array([0]))[0].detach().numpy(), H_untilted=model.H.numpy(),
                   obj_tilts=model.opt_obj_tilts.detach().numpy().copy(),
                   slice_thickness=np.float32(model.opt_slice_thickness.item()), dx=np.float32(model.dx.item()),
                   lambd=np.float32(model.lambd.item()), prop_lr=json.dumps(PROP_LR),
                   g_obj_tilts=np.zeros((1, 2), np.float32) if g(model.opt_obj_tilts) is None
                   else g(model.opt_obj_tilts),
                   g_slice_thickness=np.float32(0.0) if g(model.opt_slice_thickness) is None
                   else g(model.opt_slice_thickness))
    if tilts is not None and np.asarray(tilts).size > 2:   # per-position tilts: H is the base one
        base = model.H if "slice_thickness" not in PROP_LR else \
            torch.exp(1j * model.opt_slice_thickness * model.Kz)   # case 1: exp(i dz Kz)
        out.update(H=base.detach().numpy(), tilt_each=True)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: loss={float(total):.7g} terms={[round(float(t), 7) for t in terms]}")


def run_trajectory(name, n, P, O, Nz, n_slow, n_fast, bsize, niter, grad_accumulation, seed, constraint_params=None,
                   shift_lr=5e-4):
    scan, probe, H, occu, obja, objp, gta, gtp = make_inputs(n, P, O, Nz, n_slow, n_fast, seed)
    meas = simulate_meas(scan, probe, H, occu, gta, gtp, shift_lr)
    iv = init_variables(obja, objp, probe, H, occu, scan.crop_pos, scan.shifts, meas,
                        scan.n_slow, scan.n_fast)
    model = build_model(iv, shift_lr)
    init_state = dict(obja=model.opt_obja.detach().numpy().copy(),
                      objp=model.opt_objp.detach().numpy().copy(),
                      probe=torch.view_as_complex(model.opt_probe.detach()).numpy().copy(),
                      shifts=model.opt_probe_pos_shifts.detach().numpy().copy())
    S = scan.crop_pos.shape[0]
    perm = np.random.default_rng(seed + 7).permutation(S)
    batches = np.array_split(perm, S // bsize)
    loss_fn = losses.CombinedLoss(DEFAULT_LOSS, device="cpu")
    opt = reconstruction.create_optimizer(model.optimizer_params, model.optimizable_params,
                                          verbose=False)
    hist = []
    if constraint_params is None:
        cfn = lambda m, i: None   # noqa: E731
    else:
        import ptyrad.constraints as cons
        cfn = cons.CombinedConstraint(constraint_params, device="cpu", verbose=False)
    for it in range(1, niter + 1):
        bl = reconstruction.recon_step(batches, grad_accumulation, model, opt, loss_fn,
                                       cfn, it, verbose=False)
        hist.append([float(np.mean(v)) for v in bl.values()])
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"),
        init_obja=init_state["obja"], init_objp=init_state["objp"],
        init_probe=init_state["probe"], init_shifts=init_state["shifts"],
        crop_pos=scan.crop_pos, H=model.H.numpy(), occu=model.omode_occu.numpy(), meas=meas,
        batches=np.concatenate(batches), batch_sizes=np.array([len(b) for b in batches]),
        niter=niter, grad_accumulation=grad_accumulation, lrs=json.dumps(model.lr_params),
        final_obja=model.opt_obja.detach().numpy(), final_objp=model.opt_objp.detach().numpy(),
        final_probe=torch.view_as_complex(model.opt_probe.detach()).numpy(),
        final_shifts=model.opt_probe_pos_shifts.detach().numpy(),
        loss_hist=np.array(hist), loss_params=json.dumps(DEFAULT_LOSS),
        probe_int_sum=np.float32(model.probe_int_sum.item()),
        constraint_params=json.dumps(constraint_params))
    print(f"{name}: loss_hist={np.array(hist).sum(1)}")


def run_otf_case(name, n, P, O, Nz, n_slow, n_fast, B, seed, Hm, pad_to=None, scale=None):
    """On-the-fly measurement padding / resampling (models.py:81-86, :384-412): the model holds
    (S, Hm, Hm) frames; get_measurements pastes them into the canvas and/or resamples to n."""
    scan, probe, H, occu, obja, objp, _, _ = make_inputs(n, P, O, Nz, n_slow, n_fast, seed)
    rng = np.random.default_rng(seed + 7)
    S = scan.crop_pos.shape[0]
    meas_small = rng.uniform(0.0, 2.0 / (Hm * Hm), (S, Hm, Hm)).astype(np.float32)
    iv = init_variables(obja, objp, probe, H, occu, scan.crop_pos, scan.shifts, meas_small, scan.n_slow, scan.n_fast)
    if pad_to is not None:
        h1 = (pad_to - Hm) // 2
        iv["on_the_fly_meas_padded"] = rng.uniform(0.0, 1e-4, (pad_to, pad_to)).astype(np.float32)
        iv["on_the_fly_meas_padded_idx"] = np.array([h1, h1 + Hm, h1, h1 + Hm], np.int32)
    if scale is not None:
        iv["on_the_fly_meas_scale_factors"] = [float(scale), float(scale)]
    model = build_model(iv, 5e-4)
    loss_fn = losses.CombinedLoss(DEFAULT_LOSS, device="cpu")
    batch = np.random.default_rng(seed + 100).permutation(S)[:B].astype(np.int64)
    dp = model(batch)
    mdp = model.get_measurements(batch)
    total, terms = loss_fn(dp, mdp, model._current_object_patches, model.omode_occu)
    total.backward()
    out = dict(obja=model.opt_obja.detach().numpy(), objp=model.opt_objp.detach().numpy(),
               probe=torch.view_as_complex(model.opt_probe.detach()).numpy(),
               shifts=model.opt_probe_pos_shifts.detach().numpy(),
               crop_pos=scan.crop_pos, H=model.H.numpy(), occu=model.omode_occu.numpy(), batch=batch,
               loss_params=json.dumps(DEFAULT_LOSS), shift_probes=True, meas_small=meas_small,
               meas_otf=mdp.detach().numpy(), dp=dp.detach().numpy(),
               loss_terms=np.array([float(t) for t in terms], np.float64), loss_total=np.float64(float(total)),
               g_obja=model.opt_obja.grad.numpy(), g_objp=model.opt_objp.grad.numpy(),
               g_probe=model.opt_probe.grad.numpy(), g_shifts=model.opt_probe_pos_shifts.grad.numpy())
    for k in ("on_the_fly_meas_padded", "on_the_fly_meas_padded_idx", "on_the_fly_meas_scale_factors"):
        if k in iv:
            out[k] = np.asarray(iv[k])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: loss={float(total):.7g} meas_otf {tuple(mdp.shape)}")


def constrained_trajectory():
    """3 iterations with the schema-default constraints (obj_rblur off: torchvision is absent)."""
    import copy

    from constraint_defaults import DEFAULTS
    cp = copy.deepcopy(DEFAULTS)
    cp["obj_rblur"]["freq"] = None
    run_trajectory("traj_n64_p2z2_cons", 64, 2, 1, 2, 4, 4, 4, 3, 1, seed=23, constraint_params=cp)


if __name__ == "__main__":
    torch.set_num_threads(4)
    if len(sys.argv) > 1 and sys.argv[1] == "--tilt-only":
        run_case("n64_p2o1z3_tilt", 64, 2, 1, 3, 3, 3, 6, seed=18, tilts=[3.0, -2.0])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--simlar-only":
        # loss_simlar (losses.py:106-141) blurs the patches with torchvision's gaussian_blur
        models.gaussian_blur = refimport.tv_gaussian_blur
        losses.gaussian_blur = refimport.tv_gaussian_blur
        sim = json.loads(json.dumps(DEFAULT_LOSS))
        sim["loss_simlar"].update(state=True, weight=0.2, obj_type="both", blur_std=1.0)
        run_case("n32_p1o2z2_simlar", 32, 1, 2, 2, 4, 4, 6, seed=81, loss_params=sim)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--pacbed-only":
        pac = json.loads(json.dumps(DEFAULT_LOSS))
        pac["loss_pacbed"].update(state=True, weight=0.5, dp_pow=0.2)
        run_case("n32_p2o1z2_pacbed", 32, 2, 1, 2, 4, 4, 7, seed=71, loss_params=pac)
        only = json.loads(json.dumps(pac))
        only["loss_single"].update(state=False)
        only["loss_sparse"].update(state=False)
        run_case("n64_p1o1z1_pacbedonly", 64, 1, 1, 1, 3, 3, 6, seed=72, loss_params=only)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--each-only":
        # per-position tilts (tilt_type 'each', models.py:330-356): fixed (case 2B) and optimised (2A)
        t16 = np.random.default_rng(61).uniform(-4.0, 4.0, (16, 2)).astype(np.float32)
        run_case("n32_p2o1z3_tilteach", 32, 2, 1, 3, 4, 4, 6, seed=61, tilts=t16)
        PROP_LR.update(obj_tilts=1e-3)
        t9 = np.random.default_rng(62).uniform(-4.0, 4.0, (9, 2)).astype(np.float32)
        run_case("n64_p1o2z2_opttilteach", 64, 1, 2, 2, 3, 3, 5, seed=62, tilts=t9)
        if len(sys.argv) > 2 and sys.argv[2] == "--with-dz":   # case 1 with per-position tilts
            PROP_LR.update(slice_thickness=1e-3)
            t16b = np.random.default_rng(63).uniform(-4.0, 4.0, (16, 2)).astype(np.float32)
            run_case("n32_p2o1z3_opttiltdzeach", 32, 2, 1, 3, 4, 4, 6, seed=63, tilts=t16b)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--otf-only":
        run_otf_case("otf_n32_pad", 32, 2, 1, 1, 4, 4, 6, seed=51, Hm=24, pad_to=32)
        run_otf_case("otf_n32_resample", 32, 1, 1, 2, 4, 4, 5, seed=52, Hm=16, scale=2.0)
        run_otf_case("otf_n32_pad_resample", 32, 1, 2, 1, 4, 4, 6, seed=53, Hm=20, pad_to=24, scale=1.3334)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--prop-only":
        PROP_LR.update(slice_thickness=1e-3)                         # case 3
        run_case("n32_p2o1z3_optdz", 32, 2, 1, 3, 4, 4, 6, seed=41)
        PROP_LR.clear()
        PROP_LR.update(obj_tilts=1e-3)                               # case 2A
        run_case("n32_p1o1z2_opttilt", 32, 1, 1, 2, 4, 4, 5, seed=42, tilts=[2.0, -1.0])
        PROP_LR.update(slice_thickness=1e-3)                         # case 1
        run_case("n64_p2o1z2_opttiltdz", 64, 2, 1, 2, 3, 3, 6, seed=43, tilts=[1.5, 2.5])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--blur-only":
        # detector blur (models.py:379-380) / object pre-blur (:275-284) call torchvision's
        # gaussian_blur, absent here: the reference runs with refimport.tv_gaussian_blur in its place
        models.gaussian_blur = refimport.tv_gaussian_blur
        BLUR.update(detector_blur_std=1.0, obj_preblur_std=None)
        run_case("n32_p2o1z2_detblur", 32, 2, 1, 2, 4, 4, 6, seed=31)
        BLUR.update(detector_blur_std=None, obj_preblur_std=0.8)
        run_case("n32_p1o2z1_preblur", 32, 1, 2, 1, 4, 4, 5, seed=32)
        BLUR.update(detector_blur_std=0.7, obj_preblur_std=1.2)
        run_case("n64_p2o1z1_bothblur", 64, 2, 1, 1, 3, 3, 6, seed=33)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--c1-traj":
        # BASELINE configs[0] shape: tBL_WSe2 params (demo/params/tBL_WSe2_reconstruct.yml:118-123:
        # obja / objp lr 5e-4, probe 1e-4, probe_pos_shifts 1e-4), N = 128, 8×8 scan, batch 32
        run_trajectory("traj_c1_n128", 128, 1, 1, 1, 8, 8, 32, 2, 1, seed=24, shift_lr=1e-4)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--constrained-only":
        constrained_trajectory()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--mixed-radix":
        # N with factors 3 and 5 (meas_crop / meas_resample / meas_pad output, init_params.py:53, 340,
        # 361): the general engine's mixed-radix Stockham passes, in LDS (96) and in global scratch
        run_case("n96_p2o1z2_mixed", 96, 2, 1, 2, 3, 3, 6, seed=101)
        run_case("n96_p1o1z1_single", 96, 1, 1, 1, 3, 3, 5, seed=102)
        run_case("n160_p1o1z1_mixed", 160, 1, 1, 1, 3, 3, 4, seed=103, big=True)
        run_case("n192_p2o2z1_mixed", 192, 2, 2, 1, 3, 3, 4, seed=104, big=True)
        run_trajectory("traj_n96_p2_ga1", 96, 2, 1, 1, 3, 3, 3, 3, 1, seed=105)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--both-terms":
        # loss_single + loss_poissn (+ loss_sparse) at the shapes of every engine that takes both
        # terms in two passes around k_finalize: k_fused3, k_fused3ms, the mixed-state engine, stripe
        both = json.loads(json.dumps(DEFAULT_LOSS))
        both["loss_poissn"].update(state=True, weight=0.5, dp_pow=1.0, eps=1e-6)
        run_case("n128_p1o1z1_both", 128, 1, 1, 1, 3, 3, 8, seed=121, loss_params=both)
        run_case("n128_p1o1z3_both", 128, 1, 1, 3, 3, 3, 8, seed=122, loss_params=both)
        run_case("n128_p3o1z2_both", 128, 3, 1, 2, 3, 3, 8, seed=123, loss_params=both)
        run_case("n256_p2o2z1_both", 256, 2, 2, 1, 3, 3, 6, seed=124, loss_params=both, big=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--smooth":
        # every 2·3·5-smooth N in [32, 256] runs the general engine: odd N (45, 125), a radix-15
        # LDS plan (120), and the radix > 16 plans on 512-thread workgroups (125 = 25·5 in LDS,
        # 216 = 18·12 and 250 = 25·10 in global scratch)
        run_case("n45_p1o1z2_odd", 45, 1, 1, 2, 3, 3, 5, seed=111)
        run_case("n120_p2o1z1_r15", 120, 2, 1, 1, 3, 3, 5, seed=112)
        run_case("n125_p1o1z1_odd", 125, 1, 1, 1, 3, 3, 4, seed=113, big=True)
        run_case("n216_p2o1z2_r18", 216, 2, 1, 2, 3, 3, 4, seed=114, big=True)
        run_case("n250_p1o2z1_r25", 250, 1, 2, 1, 3, 3, 4, seed=115, big=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--radix7":
        # 2·3·5·7-smooth N (round 5): radix 7 in LDS (112 = 16·7, 49 = 7·7 odd) and radix 14 / 21 in
        # global scratch (196 = 14·14, 189 = 27·7 on 512-thread workgroups)
        run_case("n112_p2o1z2_r7", 112, 2, 1, 2, 3, 3, 6, seed=131)
        run_case("n49_p1o2z1_r7", 49, 1, 2, 1, 3, 3, 5, seed=132)
        run_case("n196_p1o1z2_r14", 196, 1, 1, 2, 3, 3, 4, seed=133, big=True)
        run_case("n189_p2o1z1_r27x7", 189, 2, 1, 1, 3, 3, 4, seed=134, big=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--big-n":
        # N above 256 (round 5): the line-block two-pass plans with radices up to 49 on 512-thread
        # workgroups — 384 = 24·16, 343 = 49·7 (odd, the largest radix), 512 = 32·16 with two modes
        run_case("n384_p1o1z1_big", 384, 1, 1, 1, 3, 3, 4, seed=141, big=True)
        run_case("n343_p1o1z2_r49", 343, 1, 1, 2, 3, 3, 3, seed=142, big=True)
        run_case("n512_p2o1z1_big", 512, 2, 1, 1, 3, 3, 3, seed=143, big=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--large":
        # the (N, P, O, Nz) of BASELINE configs[2..4] and of both demos, so the engines that only
        # run at these sizes (N = 256 stripe / general stages, mixed-state multislice, Nz = 16)
        # are compared with PtyRAD's own output: 3x3 scans, meas kept at the batch rows as f16
        run_case("n256_p8o2z1_c3", 256, 8, 2, 1, 3, 3, 8, seed=91, big=True)               # c3
        run_case("n256_p4o1z1_c5f16", 256, 4, 1, 1, 3, 3, 8, seed=92, big=True, f16_storage=True)  # c5
        run_case("n128_p1o1z16_c4", 128, 1, 1, 16, 3, 3, 8, seed=93, big=True)             # c4
        run_case("n128_p6o1z6_tbl", 128, 6, 1, 6, 3, 3, 8, seed=94, big=True)              # tBL demo
        run_case("n256_p4o1z5_pso", 256, 4, 1, 5, 3, 3, 6, seed=95, big=True)              # PSO-like
        run_trajectory("traj_n256_p4_ga1", 256, 4, 1, 1, 3, 3, 3, 3, 1, seed=96)
        run_trajectory("traj_n128_p6z6_ga1", 128, 6, 1, 6, 3, 3, 3, 3, 1, seed=97)
        sys.exit(0)
    poisson = json.loads(json.dumps(DEFAULT_LOSS))
    poisson["loss_poissn"].update(state=True, weight=0.5, dp_pow=1.0, eps=1e-6)
    poisson["loss_sparse"].update(ln_order=2, weight=0.05)
    single_q1 = json.loads(json.dumps(DEFAULT_LOSS))
    single_q1["loss_single"].update(dp_pow=1.0, weight=2.0)
    single_q1["loss_sparse"].update(state=False)

    run_case("n32_p1o1z1_shift", 32, 1, 1, 1, 4, 4, 6, seed=11)
    run_case("n32_p2o2z3_shift", 32, 2, 2, 3, 4, 4, 5, seed=12)
    run_case("n64_p1o1z2_noshift", 64, 1, 1, 2, 3, 3, 5, seed=13, shift_lr=0.0)
    run_case("n32_p2o1z1_poisson", 32, 2, 1, 1, 4, 4, 7, seed=14, loss_params=poisson)
    run_case("n32_p1o2z1_q1", 32, 1, 2, 1, 3, 4, 4, seed=15, loss_params=single_q1)
    run_case("n64_p3o1z1_shift", 64, 3, 1, 1, 3, 3, 9, seed=16)
    run_case("n128_c1_b32", 128, 1, 1, 1, 8, 8, 32, seed=17, big=True)
    run_case("n64_p2o1z3_tilt", 64, 2, 1, 3, 3, 3, 6, seed=18, tilts=[3.0, -2.0])
    run_trajectory("traj_n64_b4_ga1", 64, 1, 1, 1, 4, 4, 4, 3, 1, seed=21)
    run_trajectory("traj_n32_p2_ga2", 32, 2, 1, 2, 4, 4, 4, 3, 2, seed=22)
    constrained_trajectory()
