"""Probe-gradient error of loss_single + loss_poissn vs one term, register vs general engine
(the tolerance note in tests/test_gpu_parity.py): python tools/diag_both_terms.py"""
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from oracle import ptyx_oracle as orc
from tests.test_gpu_parity import orc_default_loss, run_fused
from tests.test_oracle_golden import rel
from ptyrad_amd import synthetic as syn
device = torch.device("cuda", 0)
for nz, shift, q1, both in [(3, True, 0.5, True), (3, True, 0.5, False), (3, True, 1.0, True)]:
    pr = syn.random_problem(128, 6, 7, Nz=nz, seed=40 + nz)
    lp = orc_default_loss(); lp["loss_poissn"]["state"] = both; lp["loss_single"]["dp_pow"] = q1
    d = dict(obja=pr.obja, objp=(pr.objp / nz).astype(np.float32), probe=pr.probe * np.float32(60.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift, loss_params=lp)
    perm = np.random.default_rng(7).permutation(42)
    cuts = [0, 9, 10, 30, 42]
    batches = [perm[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, lp, shift_probes=shift, grad_scale=0.5)
    for eng in ("register", "general"):
        if eng == "general": os.environ["PTYX_OBJ_SCRATCH_MB"] = "0"
        else: os.environ.pop("PTYX_OBJ_SCRATCH_MB", None)
        ks = {}
        terms, dp, g, _ = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
        print(nz, shift, q1, both, eng, sorted(ks)[:3], {k: f"{rel(g[k], og[k]):.2e}" for k in ("obja", "objp", "probe", "shifts")}, flush=True)
