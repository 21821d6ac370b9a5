"""Per-pattern throughput of the other BASELINE.json configs on ONE GPU (bench.py measures c2).

    python tools/bench_configs.py --config c3 [--patterns 16384] [--steps 3]

The scan is a contiguous block of the config's full raster (so overlap and object size are the
config's own: object side from SURVEY.md §8 geometry), `--patterns` positions of it, reference
mini-batch 32, loss_single + loss_sparse, shifts on, synthetic DPs.  Reports patterns/s, the
per-kernel milliseconds from HIP events, and both roofline fractions of the dominant kernel:
B_alg = N²(s_m + 16·O·Nz) bytes and F_alg = n_fft·5N²log2N² flops per pattern.

  c3  N=256, P=8, O=2, Nz=1            (512² scan)
  c4  N=128, P=1, O=1, Nz=16, dz 2 Å   (1024² scan; per GPU 1/8 of it in the 8-GPU config)
  c5  N=256, P=4, O=1, Nz=1, fp16 DPs  (4096² scan)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "c2": dict(N=128, P=1, O=1, Nz=1, scan=256, f16=False),
    "c3": dict(N=256, P=8, O=2, Nz=1, scan=512, f16=False),
    "c4": dict(N=128, P=1, O=1, Nz=16, scan=1024, f16=False),
    "c5": dict(N=256, P=4, O=1, Nz=1, scan=4096, f16=True),
}
HBM_PEAK_GBPS, FP32_PEAK_TFLOPS = 8000.0, 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--patterns", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    c = CONFIGS[a.config]
    import torch

    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets

    dev = torch.device("cuda", 0)
    N, P, O, Nz = c["N"], c["P"], c["O"], c["Nz"]
    step_px = syn.STEP_ANG / syn.DX_ANG
    side = syn.object_side(c["scan"], N, step_px)
    n_fast = min(c["scan"], a.patterns)
    n_slow = max(1, a.patterns // n_fast)
    # a block of n_slow × n_fast positions of the full raster, in the full-size object
    full = syn.raster_scan(n_slow, n_fast, N, obj_shape=(side, side), seed=0)
    n = full.crop_pos.shape[0]
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    obja = (1.0 + 0.05 * torch.randn((O, Nz, side, side), generator=g, device=dev)).float()
    objp = (0.1 / Nz * torch.randn((O, Nz, side, side), generator=g, device=dev)).float()
    base = syn.stem_probe(N) * np.float32(60.0)
    probe_c = syn.mixed_probe(base, P) if P > 1 else base[None]
    probe = torch.view_as_real(torch.tensor(probe_c.astype(np.complex64), device=dev)).contiguous()
    meas = torch.rand((n, N, N), generator=g, device=dev)
    if c["f16"]:
        meas = meas.half()
    t = {"obja": obja, "objp": objp, "probe": probe, "shifts": torch.tensor(full.shifts, device=dev),
         "H": torch.tensor(syn.fresnel_propagator(N, syn.DX_ANG, 2.0), device=dev),
         "occu": torch.tensor(syn.omode_occupancy(O), device=dev), "crop_pos": torch.tensor(full.crop_pos, device=dev),
         "meas": meas}
    plan = Plan(N, P, O, Nz, side, side, n, n, shift_probes=True, meas_f16=c["f16"], device=dev)
    rng = np.random.default_rng(7)
    batches = np.array_split(rng.permutation(n), max(1, n // a.batch))
    idx_t = torch.as_tensor(np.concatenate(batches), dtype=torch.int32, device=dev)
    off_t = batch_offsets(batches)      # host offsets: the engine may split the call at batch boundaries
    nb, mb = len(batches), max(len(b) for b in batches)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    terms = torch.empty((nb, 5), device=dev)

    def step():
        for v in grads.values():
            v.zero_()
        plan.forward_loss_grad(t, idx_t, off_t, LossConfig(), grads, grad_scale=1.0 / nb, loss_terms=terms,
                               max_batch=mb)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    plan.profile_begin()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ks = plan.profile_end()
    assert torch.isfinite(terms).all()
    s_m = 2 if c["f16"] else 4
    b_alg = N * N * (s_m + 16 * O * Nz)
    n_fft = 2 * P * O * (2 * Nz - 1) + 2 * P
    f_alg = n_fft * 5 * N * N * math.log2(N * N)
    dom = max(ks, key=lambda k: ks[k][1])
    dom_s = ks[dom][1] / a.steps / 1e3      # the kernel's time per step (all its launches)
    out = {"config": a.config, "N": N, "P": P, "O": O, "Nz": Nz, "meas": "f16" if c["f16"] else "f32",
           "object": [side, side], "patterns_per_step": n, "scan_block": [n_slow, n_fast],
           "patterns_per_s": round(n * a.steps / el, 1), "ms_per_step": round(1e3 * el / a.steps, 3),
           "dominant_kernel": dom, "dom_ms": round(dom_s * 1e3, 3),
           "hbm_frac": round(b_alg * n / dom_s / 1e9 / HBM_PEAK_GBPS, 4),
           "fp32_frac": round(f_alg * n / dom_s / 1e12 / FP32_PEAK_TFLOPS, 4),
           "B_alg": b_alg, "F_alg": f_alg,
           "kernels_ms_per_step": {k: round(v[1] / a.steps, 3) for k, v in ks.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
