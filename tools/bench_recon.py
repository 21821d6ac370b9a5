"""Time the caller contract (recon_step, reconstruction.py:658-781) end to end on one GPU.

    python tools/bench_recon.py [--scan 256] [--ga 1 16 2048] [--iters 1] [--rccl split|whole]

PtychoHIP + CombinedLoss.fused_into + torch Adam at the c2 geometry (N = 128, P = O = Nz = 1, the
scan² raster, mini-batches of 32, make_batches 'random', seeded uniform DPs): one iteration =
every mini-batch once, an optimizer step every `ga` mini-batches.  ga = 1 is the reference's
default cadence (params/recon_params.py:17): 2,048 optimizer steps per iteration at scan 256, each
on 32 patterns, so per-step host work and launch latency count.  Prints one JSON line per ga.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scan", type=int, default=256)
    ap.add_argument("--ga", type=int, nargs="+", default=[1, 16, 2048])
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--pmodes", type=int, default=1, help="probe modes (tBL_WSe2 demo: 6)")
    ap.add_argument("--slices", type=int, default=1, help="object slices (tBL_WSe2 demo: 6)")
    ap.add_argument("--omodes", type=int, default=1, help="object modes")
    ap.add_argument("--simlar", choices=["off", "call", "batch"], default="off",
                    help="loss_simlar (weight 0.1, both, blur 1): beside the engine call, or per mini-batch (A/B)")
    ap.add_argument("--tune", action="append", default=[], help="ptyx_set_tuning key=value (A/B runs)")
    ap.add_argument("--graphs", choices=["auto", "on", "off"], default="auto",
                    help="recon_step(graphs=...): hipGraph-replayed optimizer steps")
    ap.add_argument("--rccl", choices=["off", "split", "whole"], default="off",
                    help="init_process_group('nccl') at world size 1 with every collective of the data-parallel "
                         "step executed (DistContext(always_reduce=True)): mini-batches split over the ranks "
                         "(the default cadence on several GPUs) or dealt whole")
    ap.add_argument("--chunk", type=int, default=None, help="StepGraphs.CHUNK: same-shape steps a graph (A/B)")
    a = ap.parse_args()
    if a.chunk is not None:
        from ptyrad_amd.stepgraph import StepGraphs
        StepGraphs.CHUNK = a.chunk
    ctx = None
    if a.rccl != "off":
        import torch.distributed as dist
        from ptyrad_amd.reconstruction import DistContext
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        ctx = DistContext(split_batches=a.rccl == "split", always_reduce=True)
    from ptyrad_amd import _lib
    from ptyrad_amd import synthetic as syn
    for kv in a.tune:
        k, v = kv.split("=")
        _lib.set_tuning(k, int(v))
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from ptyrad_amd.reconstruction import create_optimizer, make_batches, recon_step
    dev = torch.device("cuda", 0)
    N, S = 128, a.scan
    scan = syn.raster_scan(S, S, N, seed=0)
    n = S * S
    rng = np.random.default_rng(0)
    Ny, Nx = scan.obj_shape
    P, Nz, O = a.pmodes, a.slices, a.omodes
    probe = np.stack([syn.stem_probe(N) * np.float32(60.0 / (1 + 2 * p)) for p in range(P)])
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    meas = torch.rand((n, N, N), generator=g, device=dev)
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 1e-4}
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
          "loss_pacbed": {"state": False, "weight": 0.5, "dp_pow": 0.2},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
          "loss_simlar": {"state": a.simlar != "off", "weight": 0.1, "obj_type": "both",
                          "scale_factor": [1, 1, 1], "blur_std": 1}}
    for ga in a.ga:
        iv = {"obja": np.ones((O, Nz, Ny, Nx), np.float32),
              "objp": (1e-8 * rng.random((O, Nz, Ny, Nx))).astype(np.float32), "obj": None,
              "probe": probe, "probe_pos_shifts": scan.shifts, "omode_occu": np.full(O, 1.0 / O, np.float32),
              "H": syn.fresnel_propagator(N, syn.DX_ANG, 2.0), "measurements": meas, "crop_pos": scan.crop_pos,
              "N_scan_slow": S, "N_scan_fast": S, "slice_thickness": 2.0, "dx": syn.DX_ANG, "dk": 1.0 / (N * syn.DX_ANG),
              "lambd": syn.electron_wavelength(syn.KV), "obj_tilts": np.zeros((1, 2), np.float32)}
        mp = {"detector_blur_std": None, "obj_preblur_std": None,
              "update_params": {k: {"start_iter": 1 if v else None, "lr": v} for k, v in lrs.items()},
              "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}
        model = PtychoHIP(iv, mp, device=dev, verbose=False)
        opt = create_optimizer(model.optimizer_params, model.optimizable_params)
        loss_fn = CombinedLoss(lp, device=dev)
        loss_fn.simlar_per_batch = a.simlar == "batch"
        batches = make_batches(np.arange(n), scan.crop_pos, 32, mode="random", rng=np.random.default_rng(3))
        graphs = {"auto": None, "on": True, "off": False}[a.graphs]
        recon_step(batches, ga, model, opt, loss_fn, None, 1, verbose=False, graphs=graphs,
                   dist_ctx=ctx)   # warm-up iteration
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(a.iters):
            recon_step(batches, ga, model, opt, loss_fn, None, 2 + it, verbose=False, graphs=graphs, dist_ctx=ctx)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        steps = -(-len(batches) // ga)
        sg = getattr(model, "_step_graphs", None)
        print(json.dumps({"ga": ga, "P": P, "O": O, "Nz": Nz, "simlar": a.simlar, "graphs": a.graphs, "rccl": a.rccl, "tune": a.tune, "chunk": a.chunk, "replays": sg.replays if sg else 0,
                          "mini_batches": len(batches), "optimizer_steps": steps,
                          "s_per_iter": round(dt, 4), "patterns_per_s": round(n / dt, 1),
                          "ms_per_optimizer_step": round(1e3 * dt / steps, 4),
                          "loss": float(model.loss_iters[-1][1])}), flush=True)
        del model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
