"""Where the time of one optimizer step goes at the reference's default cadence (ga = 1).

    python tools/recon_overhead.py [--scan 256] [--steps 512]

c2 geometry, mini-batches of 32.  Each line times `steps` repetitions of one piece, synchronising
only at the end (so a line is host-bound when the host is slower than the GPU):
  engine_dev    Plan.forward_loss_grad on device-resident idx / offsets
  engine_host   the same with numpy idx / offsets (two host-to-device copies per call)
  fused_into    CombinedLoss.fused_into(model, [batch])  (recon_step's per-step engine path)
  adam          torch Adam.step() over obja / objp / probe / shifts (the model's param groups)
  recon_step    recon_step(..., grad_accumulation=1) over `steps` mini-batches
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return round(1e3 * (t1 - t0) / steps, 4), round(1e3 * (t2 - t0) / steps, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scan", type=int, default=256)
    ap.add_argument("--steps", type=int, default=512)
    a = ap.parse_args()
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, batch_offsets
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from ptyrad_amd.reconstruction import create_optimizer, make_batches, recon_step
    dev = torch.device("cuda", 0)
    N, S = 128, a.scan
    scan = syn.raster_scan(S, S, N, seed=0)
    n = S * S
    Ny, Nx = scan.obj_shape
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    meas = torch.rand((n, N, N), generator=g, device=dev)
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 1e-4}
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
          "loss_pacbed": {"state": False, "weight": 0.5, "dp_pow": 0.2},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1}, "loss_simlar": {"state": False}}
    iv = {"obja": np.ones((1, 1, Ny, Nx), np.float32), "objp": np.zeros((1, 1, Ny, Nx), np.float32), "obj": None,
          "probe": (syn.stem_probe(N) * np.float32(60.0))[None], "probe_pos_shifts": scan.shifts,
          "omode_occu": np.ones(1, np.float32), "H": syn.fresnel_propagator(N, syn.DX_ANG, 2.0),
          "measurements": meas, "crop_pos": scan.crop_pos, "N_scan_slow": S, "N_scan_fast": S,
          "slice_thickness": 2.0, "dx": syn.DX_ANG, "dk": 1.0, "lambd": 0.04, "obj_tilts": np.zeros((1, 2), np.float32)}
    mp = {"detector_blur_std": None, "obj_preblur_std": None,
          "update_params": {k: {"start_iter": 1 if v else None, "lr": v} for k, v in lrs.items()},
          "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}
    model = PtychoHIP(iv, mp, device=dev, verbose=False)
    opt = create_optimizer(model.optimizer_params, model.optimizable_params)
    loss_fn = CombinedLoss(lp, device=dev)
    batches = make_batches(np.arange(n), scan.crop_pos, 32, mode="random", rng=np.random.default_rng(3))
    plan = model.plan
    t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
         "shifts": model.opt_probe_pos_shifts.detach(), "H": model._H_rv().detach(), "tilts": None}
    t.update(model._base())
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    cfg = LossConfig.from_loss_params(lp)
    idx_dev = [torch.as_tensor(b, dtype=torch.int32, device=dev) for b in batches[:a.steps]]
    off_dev = [torch.as_tensor(batch_offsets([b]), device=dev) for b in batches[:a.steps]]
    out = {}
    out["engine_dev"] = timed(lambda i: plan.forward_loss_grad(t, idx_dev[i], off_dev[i], cfg, grads), a.steps)
    plan.profile_begin()      # per-kernel GPU time of a 32-pattern call (HIP events)
    for i in range(64):
        plan.forward_loss_grad(t, idx_dev[i], off_dev[i], cfg, grads)
    out["engine_kernels_ms_per_call"] = {k: round(v[1] / 64, 4) for k, v in plan.profile_end().items()}
    out["engine_host"] = timed(lambda i: plan.forward_loss_grad(t, batches[i], batch_offsets([batches[i]]), cfg,
                                                                grads), a.steps)
    for p in (model.opt_obja, model.opt_objp, model.opt_probe, model.opt_probe_pos_shifts):
        p.grad = torch.zeros_like(p)
    out["fused_into"] = timed(lambda i: loss_fn.fused_into(model, [batches[i]]), a.steps)
    out["adam"] = timed(lambda i: opt.step(), a.steps)
    ps = [model.opt_obja, model.opt_objp, model.opt_probe, model.opt_probe_pos_shifts]
    for label, kw, merge in (("adam_fused", {"fused": True}, False), ("adam_foreach_merged", {"foreach": True}, True),
                             ("adam_fused_merged", {"fused": True}, True)):
        if merge:   # one group per learning rate
            by = {}
            for gr in model.optimizable_params:
                by.setdefault(gr["lr"], []).extend(gr["params"])
            groups = [{"params": v, "lr": k} for k, v in by.items()]
        else:
            groups = [{"params": list(gr["params"]), "lr": gr["lr"]} for gr in model.optimizable_params]
        o2 = torch.optim.Adam(groups, **kw)
        out[label] = timed(lambda i: o2.step(), a.steps)
        del o2
    for p in ps:
        p.grad = torch.zeros_like(p)
    opt.zero_grad(set_to_none=True)
    sub = batches[:a.steps]
    out["recon_step"] = timed(lambda i: recon_step(sub, 1, model, opt, loss_fn, None, 1, verbose=False)
                              if i == 0 else None, 1)
    out["recon_step"] = [round(v / a.steps, 4) for v in out["recon_step"]]
    print(json.dumps({"ms_per_step_[host_issue, wall]": out, "steps": a.steps}), flush=True)


if __name__ == "__main__":
    main()
