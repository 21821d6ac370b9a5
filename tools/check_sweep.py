"""Seeded random sweep of engine configurations against the oracle (a GPU diagnostic for latent
path bugs: the kind the size sweep found in round 4).

    python tools/check_sweep.py [count] [seed]

Each case draws N (a supported size), P, O, Nz, shifted probes or not, one or both data terms,
the far-field cache on or off (PTYX_FFC_MB=0) and ragged mini-batches, runs one
ptyx_forward_loss_grad call and prints the relative errors of dp, loss terms and gradients; lines
marked FAIL exceed the GPU parity tolerances (tests/test_gpu_parity.py).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ptyx_oracle as orc  # noqa: E402
from tests.test_gpu_parity import TOL_DP, TOL_G, TOL_G_BOTH, TOL_SH, TOL_TERMS, orc_default_loss, run_fused  # noqa: E402
from tests.test_oracle_golden import rel  # noqa: E402

SIZES = [32, 48, 64, 96, 128, 160, 256]


def one(rng, device):
    from ptyrad_amd import synthetic as syn
    N = int(rng.choice(SIZES))
    P = int(rng.integers(1, 4))
    O = int(rng.integers(1, 3))
    Nz = int(rng.integers(1, 4)) if N <= 128 else int(rng.integers(1, 3))
    shift = bool(rng.integers(0, 2))
    both = bool(rng.integers(0, 2))
    cache = bool(rng.integers(0, 2))
    if cache:
        os.environ.pop("PTYX_FFC_MB", None)
    else:
        os.environ["PTYX_FFC_MB"] = "0"
    pr = syn.random_problem(N, 3, 3, P=P, O=O, Nz=Nz, seed=int(rng.integers(0, 1 << 30)))
    lp = orc_default_loss()
    lp["loss_poissn"]["state"] = both
    d = dict(obja=pr.obja, objp=(pr.objp / Nz).astype(np.float32), probe=pr.probe * np.float32(30.0),
             shifts=pr.shifts, crop_pos=pr.crop_pos, H=pr.H, occu=pr.occu, meas=pr.meas, shift_probes=shift,
             loss_params=lp)
    perm = rng.permutation(9)
    cut = sorted(set([0, 9] + [int(c) for c in rng.integers(1, 9, 2)]))
    batches = [perm[a:b] for a, b in zip(cut[:-1], cut[1:])]
    ks = {}
    terms, dp, g, plan = run_fused(d, device, batches, grad_scale=0.5, kernels=ks)
    plan.close()
    oterms, odps, og = orc.forward_loss_grad(d["obja"], d["objp"], d["probe"], d["shifts"], d["crop_pos"], d["H"],
                                             d["occu"], d["meas"], batches, lp, shift_probes=shift, grad_scale=0.5)
    e = {"dp": rel(dp, np.concatenate(odps)), "terms": float(np.max(np.abs(terms - oterms)))}
    e.update({k: rel(g[k], og[k]) for k in ("obja", "objp", "probe")})
    if shift:
        e["shifts"] = rel(g["shifts"], og["shifts"])
    tol = {"dp": TOL_DP, "terms": TOL_TERMS * 10, "obja": TOL_G, "objp": TOL_G,
           "probe": TOL_G_BOTH if both else TOL_G, "shifts": TOL_SH}
    bad = [k for k, v in e.items() if not v < tol[k]]
    eng = "+".join(k for k in ("k_fused", "k_fmm_fwd", "k_s1", "k_adjoint") if k in ks)
    print(f"{'FAIL' if bad else 'ok  '} N={N:3d} P{P} O{O} Nz{Nz} shift={int(shift)} both={int(both)} cache={int(cache)} "
          f"batches={[len(b) for b in batches]} {eng:10s} " + " ".join(f"{k} {v:.1e}" for k, v in e.items()) +
          (f"  BAD {bad}" if bad else ""), flush=True)
    return not bad


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    device = torch.device("cuda", 0)
    fails = sum(0 if one(rng, device) else 1 for _ in range(count))
    print(f"{count - fails} ok, {fails} fail")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
