"""Benchmark: diffraction-patterns/sec/iter (fwd+loss+adjoint) on the MI355X engine.

Workload = BASELINE.json configs[1] ("c2"): synthetic 4D-STEM, 256x256 scan per GPU, 128x128 DPs,
1 probe mode, 1 object mode, single slice, sub-px probe shifts on (schema default), loss_single
(dp_pow 0.5) + loss_sparse (L1, w 0.1), reference mini-batch B = 32 with its own NRMSE
normalisation.  One step = one iteration over the GPU's whole shard (65,536 patterns = 2,048
mini-batches) through ptyx_forward_loss_grad, gradients of every mini-batch accumulated (the
reference's grad_accumulation over the iteration), followed - with N > 1 GPUs - by one RCCL
all-reduce(sum) of the object + probe gradients.  Weak scaling: the global scan is
(256·N) x 256 positions, GPU r owns rows [256 r, 256 r + 256) and its DPs; object and probe are
replicated.  Inputs are resident in HBM before the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...   (driver, one rank per GPU, RCCL)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="reference mini-batch size (BATCH_SIZE.size)")
    ap.add_argument("--scan", type=int, default=256, help="scan positions per side per GPU shard")
    ap.add_argument("--N", type=int, default=128)
    ap.add_argument("--cpu-sample", type=int, default=40960, help="patterns for the CPU baseline (about 10 s on 16 cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--geom-world", type=int, default=0,
                    help="diagnostic: build rank --geom-rank's shard of a W-GPU weak-scaling geometry on one GPU "
                         "(no collective) to check that per-rank work stays constant as W grows")
    ap.add_argument("--geom-rank", type=int, default=0)
    return ap.parse_args()


# ------------------------------------------------------------------ CPU baseline (oracle port)
def _cpu_worker(args):
    n, seed, nbatch, bsize = args
    from oracle import ptyx_oracle as orc
    from ptyrad_amd import synthetic as syn
    pr = syn.random_problem(n, 16, 16, seed=seed)
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False}, "loss_pacbed": {"state": False},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1}, "loss_simlar": {"state": False}}
    rng = np.random.default_rng(seed)
    batches = [rng.choice(256, bsize, replace=False) for _ in range(nbatch)]
    t = time.perf_counter()
    orc.forward_loss_grad(pr.obja, pr.objp, pr.probe * np.float32(60.0), pr.shifts, pr.crop_pos, pr.H, pr.occu,
                          pr.meas, batches, lp, cdt=np.complex64)
    return nbatch * bsize, time.perf_counter() - t


def cpu_baseline(n, bsize, sample):
    """Oracle (NumPy port of the reference path) on the host cores, before any GPU call."""
    import multiprocessing as mp
    cores = max(1, min(16, os.cpu_count() or 1))
    nb_total = max(cores, sample // bsize)
    per = [nb_total // cores + (1 if i < nb_total % cores else 0) for i in range(cores)]
    jobs = [(n, 100 + i, per[i], bsize) for i in range(cores) if per[i] > 0]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    pats = sum(r[0] for r in res)
    return {"value": pats / wall, "unit": "patterns/s", "cores": len(jobs), "kind": "port",
            "sample": f"{pats} patterns ({len(jobs)} processes x mini-batches of {bsize}), N={n}, P=O=Nz=1, "
                      f"shifts on, oracle/ptyx_oracle.py complex64 NumPy, wall {wall:.1f}s incl. pool start"}


# ------------------------------------------------------------------ GPU workload
def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and not a.quiet and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a.N, a.batch, a.cpu_sample)          # before the GPU is touched

    import torch
    import torch.distributed as dist
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets

    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    N, S = a.N, a.scan
    gw, gr = (a.geom_world, a.geom_rank) if a.geom_world else (world, rank)
    n_slow_g, n_fast = S * gw, S
    scan = syn.raster_scan(n_slow_g, n_fast, N, seed=0)
    sl = slice(gr * S * n_fast, (gr + 1) * S * n_fast)
    crop_pos, shifts = scan.crop_pos[sl], scan.shifts[sl]
    n_local = crop_pos.shape[0]
    Ny, Nx = scan.obj_shape
    g = torch.Generator(device=dev)
    g.manual_seed(1234)          # identical object / probe on every rank (replicas)
    obja = (1.0 + 0.05 * torch.randn((1, 1, Ny, Nx), generator=g, device=dev)).float()
    objp = (0.1 * torch.randn((1, 1, Ny, Nx), generator=g, device=dev)).float()
    probe = torch.view_as_real(torch.tensor(syn.stem_probe(N) * np.float32(60.0), device=dev)[None]).contiguous()
    gm = torch.Generator(device=dev)
    gm.manual_seed(4321 + rank)
    meas = torch.rand((n_local, N, N), generator=gm, device=dev)      # this GPU's DPs, HBM-resident
    t = {"obja": obja, "objp": objp, "probe": probe,
         "shifts": torch.tensor(shifts, device=dev), "H": torch.tensor(syn.fresnel_propagator(N, syn.DX_ANG, 2.0),
                                                                        device=dev),
         "occu": torch.ones(1, device=dev), "crop_pos": torch.tensor(crop_pos, device=dev), "meas": meas}
    plan = Plan(N, 1, 1, 1, Ny, Nx, n_local, n_local, shift_probes=True, device=dev)
    rng = np.random.default_rng(7 + rank)
    batches = np.array_split(rng.permutation(n_local), n_local // a.batch)     # make_batches 'random'
    idx_t = torch.as_tensor(np.concatenate(batches), dtype=torch.int32, device=dev)
    off_t = torch.as_tensor(batch_offsets(batches), device=dev)
    nb = len(batches)
    max_batch = max(len(b) for b in batches)
    cfg = LossConfig()
    n_obj = obja.numel()
    flat = torch.zeros(2 * n_obj + probe.numel(), device=dev)     # one all-reduce buffer
    grads = {"obja": flat[:n_obj].view_as(obja), "objp": flat[n_obj:2 * n_obj].view_as(objp),
             "probe": flat[2 * n_obj:].view_as(probe), "shifts": torch.zeros_like(t["shifts"])}
    terms = torch.empty((nb, 5), device=dev)

    def step():
        flat.zero_()
        grads["shifts"].zero_()
        plan.forward_loss_grad(t, idx_t, off_t, cfg, grads, grad_scale=1.0 / nb, loss_terms=terms,
                               max_batch=max_batch)
        if world > 1:
            dist.all_reduce(flat)          # object + probe gradients; positions are rank-local

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    plan.profile_begin()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kstats = plan.profile_end()
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    total_patterns = world * n_local * a.steps
    value = total_patterns / elapsed
    ms_per_step = 1e3 * elapsed / a.steps

    # roofline of the dominant kernel (k_fused: forward + loss + adjoint in one pass; k_adjoint on
    # the two-pass path).  SURVEY §8d per pattern: B_alg = N^2 (s_m + 16 O Nz) bytes,
    # F_alg = n_fft 5 N^2 log2 N^2 flops (n_fft = 2 P O (2 Nz - 1) + 2P with shifts).
    b_alg = N * N * (4 + 16 * 1 * 1)
    n_fft = 2 * 1 * 1 * (2 * 1 - 1) + 2
    flops = n_fft * 5 * N * N * math.log2(N * N)
    dom = "k_fused" if "k_fused" in kstats else "k_adjoint"
    launches, dom_ms = kstats.get(dom, (0, 0.0))
    roof = None
    if launches:
        avg_s = dom_ms / launches / 1e3
        achieved = b_alg * n_local / avg_s / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_c2.json")
        if os.path.exists(pmc):
            # PMC summary of the same workload (profiles/collect_pmc.sh → summarize_pmc.py); its
            # kernel names are the HIP symbols: k_fused3 (register engine) or k_fused2
            engine = "k_fused3" if "k_obj_prep" in kstats else "k_fused2"
            with open(pmc) as f:
                tb = json.load(f).get("hbm_bytes_per_launch", {})
            traffic = tb.get(engine) if dom == "k_fused" else tb.get(dom)
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "alg_bytes_per_launch": b_alg * n_local, "avg_launch_ms": round(avg_s * 1e3, 4),
                "fft_fp32_frac": round(flops * n_local / avg_s / 1e12 / FP32_PEAK_TFLOPS, 4)}
        g_launches, g_ms = kstats.get("k_obj_gather", (0, 0.0))
        if g_launches:
            # gather reads one N^2 complex g_O slot per pattern (+ the object tile, negligible)
            g_s = g_ms / g_launches / 1e3
            roof["gather"] = {"avg_launch_ms": round(g_s * 1e3, 4),
                              "achieved_GBps": round(8 * N * N * n_local / g_s / 1e9, 1)}
    out = {
        "metric": "diffraction-patterns/sec/iter (fwd+bwd), 256x256 probe positions, 128x128 DP",
        "value": round(value, 1), "unit": "patterns/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (seeded torch.rand DPs, random object, aperture STEM probe)",
        "config": {"workload": "c2: synthetic 4D-STEM, 256x256 scan per GPU, 128x128 DP, P=O=Nz=1, "
                               "sub-px shifts on, loss_single(q=0.5)+loss_sparse(L1), mini-batch 32",
                   "scan_per_gpu": [S, S], "N": N, "mini_batch": a.batch, "mini_batches_per_step": nb,
                   "patterns_per_gpu_per_step": n_local, "object": [Ny, Nx],
                   "parallelism": f"dp{world} (RCCL all-reduce of object+probe grads per step)",
                   **({"geometry_only": f"rank {gr} of a {gw}-GPU scan, no collective"} if a.geom_world else {})},
        "roofline": roof,
        "fft_tflops": round(value / world * flops / 1e12, 2) if world else None,
        "kernels_ms_per_step": {k: round(v[1] / a.steps, 3) for k, v in kstats.items()},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
