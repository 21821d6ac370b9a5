"""Per-size parity sweep of the general engine against the oracle (a quick GPU diagnostic).

    python tools/check_sizes.py [N ...]

For each N and a few (P, O, Nz, shift) configurations prints the relative errors of dp, the
loss terms and the obja / objp / probe gradients against oracle/ptyx_oracle.py.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ptyx_oracle as orc  # noqa: E402
from ptyrad_amd.csrc.build import GEN_SIZES  # noqa: E402
from tests.test_gpu_parity import orc_default_loss, run_fused  # noqa: E402
from tests.test_oracle_golden import rel  # noqa: E402


def one(N, P, O, Nz, shift, device):
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(N, 3, 3, P=P, O=O, Nz=Nz, seed=40 + 7 * P + O + Nz)
    d = dict(obja=pr.obja, objp=(pr.objp / Nz).astype(np.float32), probe=pr.probe * np.float32(30.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=orc_default_loss())
    perm = np.random.default_rng(P + O + Nz).permutation(9)
    batches = [perm[:4], perm[4:5], perm[5:]]
    ks = {}
    terms, dp, g, plan = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, d["loss_params"],
                                             shift_probes=shift, grad_scale=0.5)
    errs = [rel(dp, np.concatenate(odps)), float(np.max(np.abs(terms - oterms)))]
    errs += [rel(g[k], og[k]) for k in ("obja", "objp", "probe")]
    plan.close()
    eng = "k_adjoint1" if "k_adjoint1" in ks else "k_adjoint" if "k_adjoint" in ks else "+".join(sorted(ks))[:24]
    print(f"N={N:3d} P{P} O{O} Nz{Nz} shift={int(shift)} {eng:10s} dp {errs[0]:.1e} terms {errs[1]:.1e} "
          f"obja {errs[2]:.1e} objp {errs[3]:.1e} probe {errs[4]:.1e}", flush=True)


CFGS = [(1, 1, 1, True), (1, 1, 1, False), (1, 1, 2, True), (2, 1, 1, True), (2, 1, 1, False), (1, 2, 1, False),
        (2, 1, 2, False)]


def main():
    device = torch.device("cuda", 0)
    sizes = [int(a) for a in sys.argv[1:]] or GEN_SIZES
    for N in sizes:
        for cfg in CFGS:
            one(N, *cfg, device)


if __name__ == "__main__":
    main()
