"""Benchmark: diffraction-patterns/sec/iter (fwd+loss+adjoint) on the MI355X engine.

Default workload = BASELINE.json configs[1] ("c2"): synthetic 4D-STEM, 256x256 scan per GPU,
128x128 DPs simulated by the engine's own forward model from a ground-truth atom-lattice object
(SURVEY §8d), 1 probe mode, 1 object mode, single slice, sub-px probe shifts on (schema
default), loss_single (dp_pow 0.5) + loss_sparse (L1, w 0.1), reference mini-batch B = 32 with
its own NRMSE normalisation.  One step = one iteration over the GPU's whole shard (65,536
patterns = 2,048 mini-batches) through ptyx_forward_loss_grad, the gradients of every
mini-batch accumulated into ONE flat buffer (the reference's grad_accumulation over the
iteration, grad_accumulation = 2,048), then - with N > 1 GPUs - one RCCL all-reduce(sum) of
that buffer (ptyrad_amd.reconstruction.DistContext, the replacement of the DDP wrapper), then the
torch Adam step on the object, probe and positions (reconstruction.py:756-760).  Weak scaling: the
global scan is (256·N) x 256 positions, GPU r owns rows [256 r, 256 r + 256) and holds only its
DPs; object and probe are replicated.  Inputs are resident in HBM before the timed region.

Other workloads (--config; all one process per GPU, same step structure):
  c2-strong  a fixed 256x256 scan split over the ranks (strong scaling of the c2 step)
  c3         N=256, P=8 probe x O=2 object modes, a --patterns block of the 512² raster per rank
  c4         N=128, Nz=16, position correction: the 1024² scan sharded over the ranks
             (one optimizer step per iteration, all-reduce of the 2x16x3679² object gradient)
  c5         N=256, P=4, fp16 DP storage: a resident sub-stripe (--patterns positions) of each
             rank's shard of the 4096² scan (the full shard is 275 GB of DPs per GPU)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
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
FP32_PEAK_TFLOPS = 157.3     # FP32 vector = FP32 MFMA rate on gfx950

from ptyrad_amd.synthetic import BENCH_CONFIGS as CONFIGS  # noqa: E402  (numpy only; no GPU)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=32, help="reference mini-batch size (BATCH_SIZE.size)")
    ap.add_argument("--scan", type=int, default=None, help="c2: scan positions per side per GPU shard")
    ap.add_argument("--patterns", type=int, default=16384, help="c3 / c5: positions per rank (a block of the raster)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="patterns for the CPU baseline (0: about 20 s of the host's cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--loss", default="single", choices=["single", "poissn", "both"],
                    help="data term(s) beside loss_sparse (both: the stripe engine runs k_s3 twice around "
                         "k_finalize, the N = 128 mixed-state engine applies both coefficients in k_fmm_adj; "
                         "k_fused3 / k_fused3ms calls run the general engine)")
    ap.add_argument("--exchange", default="allreduce", choices=["allreduce", "band"],
                    help="N > 1: object gradients by one flat all-reduce, or by row band (ObjectBands: halo "
                         "rows to their owners, Adam on the owned band, bands all-gathered)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--geom-world", type=int, default=0,
                    help="diagnostic (c2): build rank --geom-rank's shard of a W-GPU weak-scaling geometry on one GPU "
                         "(no collective) to check that per-rank work stays constant as W grows")
    ap.add_argument("--geom-rank", type=int, default=0)
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="engine variant for A/B runs (ptyx_set_tuning, include/ptyx.h); recorded in the output")
    return ap.parse_args()


# ------------------------------------------------------------------ CPU baseline (oracle port)
def host_cores() -> int:
    """CPU cores this process may use: the cgroup CPU quota when there is one (the GPU box gives a
    job a share of a large host; os.cpu_count() shows the whole machine), else the affinity mask.
    PTYX_CPU_CORES overrides."""
    if os.environ.get("PTYX_CPU_CORES"):
        return max(1, int(os.environ["PTYX_CPU_CORES"]))
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


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
    """Oracle (NumPy port of the reference path) on the host cores, one process per core, before
    any GPU call.  sample 0: about 20 s of work (≈ 110 patterns/s per core measured)."""
    import multiprocessing as mp
    cores = host_cores()
    if not sample:
        sample = 110 * 20 * cores
    nb_total = max(cores, sample // bsize)
    per = [nb_total // cores + (1 if i < nb_total % cores else 0) for i in range(cores)]
    jobs = [(n, 100 + i, per[i], bsize) for i in range(cores) if per[i] > 0]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    pats = sum(r[0] for r in res)
    busy = max(r[1] for r in res)     # the workers' compute (they run concurrently), pool start excluded
    out = {"value": round(pats / busy, 1), "unit": "patterns/s", "cores": len(jobs), "kind": "port",
           "sample": f"{pats} patterns of the c2 shape ({len(jobs)} processes x mini-batches of {bsize}), N={n}, "
                     f"P=O=Nz=1, shifts on, oracle/ptyx_oracle.py complex64 NumPy; rate over the slowest worker's "
                     f"compute time {busy:.1f}s (wall {wall:.1f}s incl. pool start: {pats / wall:.1f} patterns/s)"}
    ratio = os.path.join(ROOT, "tests", "golden", "cpu_ratio.json")
    if os.path.exists(ratio):   # reference CPU path vs this port, same cores, measured in the build container
        r = json.load(open(ratio))
        out["ratio_to_reference"] = r["ratio_reference_over_port"]
        out["reference_equivalent"] = round(out["value"] * r["ratio_reference_over_port"], 1)
        out["ratio_measured"] = f"{r['host']}: reference {r['reference_patterns_per_s']} / port " \
                                f"{r['port_patterns_per_s']} patterns/s (tests/golden/measure_cpu_ratio.py)"
    return out


# ------------------------------------------------------------------ GPU workload
def gt_object(shape, dev, seed=1):
    """Ground-truth object on the device: unit amplitude, Gaussian atoms (σ 1.5 px,
    peak 0.3 rad) on a 3.3 Å hexagonal lattice — ptyrad_amd.synthetic.atom_phase_object in torch."""
    import torch
    from ptyrad_amd import synthetic as syn
    O, Nz, ny, nx = shape
    rng = np.random.default_rng(seed)
    sp = 3.3 / syn.DX_ANG
    basis = torch.tensor([[0.0, sp], [sp * math.sqrt(3) / 2, sp / 2]], dtype=torch.float64, device=dev)
    inv = torch.linalg.inv(basis.T)
    phase = torch.empty(shape, dtype=torch.float32, device=dev)
    yy = torch.arange(ny, dtype=torch.float64, device=dev)[:, None]
    xx = torch.arange(nx, dtype=torch.float64, device=dev)[None, :]
    for z in range(Nz):
        off = rng.uniform(0, sp, size=2)
        fy, fx = torch.broadcast_tensors(yy - off[0], xx - off[1])
        c = torch.einsum("ij,jyx->iyx", inv, torch.stack([fy, fx]))
        c = c - torch.round(c)
        d = torch.einsum("ij,jyx->iyx", basis.T, c)
        phase[:, z] = ((0.3 / Nz) * torch.exp(-(d[0] ** 2 + d[1] ** 2) / (2 * 1.5 ** 2))).float()
    return torch.ones_like(phase), phase


def main():
    a = parse()
    cfg = CONFIGS[a.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and not a.quiet and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(128, a.batch, a.cpu_sample)          # before the GPU is touched

    import torch
    import torch.distributed as dist
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets
    from ptyrad_amd.reconstruction import DistContext

    tunings = {}
    if a.tune:
        from ptyrad_amd import _lib
        for kv in a.tune:
            k, v = kv.split("=")
            _lib.set_tuning(k, int(v))
            tunings[k] = int(v)
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = DistContext()
    N, P, O, Nz, f16 = cfg["N"], cfg["P"], cfg["O"], cfg["Nz"], cfg["f16"]
    gw, gr = (a.geom_world, a.geom_rank) if a.geom_world else (world, rank)

    # -------------------------------------------------- geometry: this rank's positions
    crop_pos, shifts, (Ny, Nx), desc, n_global = syn.bench_geometry(a.config, gw, gr, a.patterns, a.scan)
    n_local = crop_pos.shape[0]

    # -------------------------------------------------- parameters (replicated) and this rank's DPs
    g = torch.Generator(device=dev)
    g.manual_seed(1234)               # identical reconstruction init / probe on every rank
    base = syn.stem_probe(N) * np.float32(60.0 if N == 128 else 30.0)
    probe_c = syn.mixed_probe(base, P) if P > 1 else base[None]
    probe = torch.view_as_real(torch.tensor(probe_c.astype(np.complex64), device=dev)).contiguous()
    t = {"probe": probe, "shifts": torch.tensor(shifts, device=dev),
         "H": torch.tensor(syn.fresnel_propagator(N, syn.DX_ANG, 2.0), device=dev),
         "occu": torch.tensor(syn.omode_occupancy(O), device=dev), "crop_pos": torch.tensor(crop_pos, device=dev)}
    plan = Plan(N, P, O, Nz, Ny, Nx, n_local, n_local, shift_probes=True, meas_f16=f16, device=dev)
    if a.config in ("c2", "c2-strong"):
        # DPs = the forward model on the ground-truth object (+1e-10), then the reconstruction
        # starts from exp(1e-8 i U)
        gta, gtp = gt_object((O, Nz, Ny, Nx), dev)
        meas = torch.empty((n_local, N, N), dtype=torch.float32, device=dev)
        plan.forward({**t, "obja": gta, "objp": gtp}, np.arange(n_local, dtype=np.int32), dp_out=meas)
        del gta, gtp
        t["obja"] = torch.ones((O, Nz, Ny, Nx), device=dev)
        t["objp"] = (1e-8 * torch.rand((O, Nz, Ny, Nx), generator=g, device=dev)).float()
        data = "synthetic: DPs = engine forward model of a ground-truth atom-lattice object; recon init exp(1e-8 iU)"
    else:
        t["obja"] = (1.0 + 0.05 * torch.randn((O, Nz, Ny, Nx), generator=g, device=dev)).float()
        t["objp"] = (0.1 / Nz * torch.randn((O, Nz, Ny, Nx), generator=g, device=dev)).float()
        gm = torch.Generator(device=dev)
        gm.manual_seed(4321 + rank)
        meas = torch.rand((n_local, N, N), generator=gm, device=dev)
        data = "synthetic: seeded uniform DPs (SURVEY §8d allows random DPs for c3-c5), random object"
    t["meas"] = meas.half() if f16 else meas
    del meas
    rng = np.random.default_rng(7 + rank)
    batches = np.array_split(rng.permutation(n_local), max(1, n_local // a.batch))   # make_batches 'random'
    idx_t = torch.as_tensor(np.concatenate(batches), dtype=torch.int32, device=dev)
    off = batch_offsets(batches)       # host offsets: the Plan splits a call at mini-batch boundaries
    nb = len(batches)
    max_batch = max(len(b) for b in batches)
    lcfg = LossConfig(single_on=a.loss in ("single", "both"), poissn_on=a.loss in ("poissn", "both"))
    # every gradient of the step in ONE flat buffer (position gradients are rank-local)
    names = ("obja", "objp", "probe")
    flat = torch.zeros(sum(t[k].numel() for k in names), device=dev)
    grads, o_ = {}, 0
    for k in names:
        grads[k] = flat[o_:o_ + t[k].numel()].view_as(t[k])
        o_ += t[k].numel()
    grads["shifts"] = torch.zeros_like(t["shifts"])
    terms = torch.empty((nb, 5), device=dev)
    stream = torch.cuda.current_stream(dev)
    ar_ev = []
    # The optimizer step (reconstruction.py:756-760): Adam over the reconstruction's tensors,
    # per-tensor learning rates of demo/params/tBL_WSe2_reconstruct.yml:118-123, one step per
    # iteration (grad_accumulation = all of the rank's mini-batches).  The gradients are the views
    # of the flat all-reduced buffer; the next step's engine call sees the updated tensors.  The
    # optimizer is create_optimizer's default, ptyrad_amd.optim.Adam (torch.optim.Adam with its
    # update in one grid-filling HIP launch), one param group per tensor as the reference builds them.
    from ptyrad_amd.reconstruction import create_optimizer
    lrs = {"obja": 5e-4, "objp": 5e-4, "probe": 1e-4, "shifts": 1e-4}
    for k in lrs:
        t[k].grad = grads[k]
    opt = create_optimizer({"name": "Adam", "configs": {}}, [{"params": [t[k]], "lr": lr} for k, lr in lrs.items()])
    bands = None
    n_obj = t["obja"].numel() + t["objp"].numel()
    if world > 1 and a.exchange == "band":
        from ptyrad_amd.reconstruction import ObjectBands
        bands = ObjectBands(ctx, Ny, dev)
        bands.set_rows(int(crop_pos[:, 0].min()), int(crop_pos[:, 0].max()) + N)
        objs = [t["obja"], t["objp"]]
    # bytes each rank sends per step in the exchange (ring all-reduce / all-gather: (W-1)/W per pass)
    if bands is None:
        xbytes = 2 * (world - 1) / world * flat.numel() * 4 if world > 1 else 0
    else:
        row_b = t["obja"].shape[0] * t["obja"].shape[1] * Nx * 4
        xbytes = (2 * bands.sent_rows() * row_b + (world - 1) / world * n_obj * 4 +
                  2 * (world - 1) / world * (flat.numel() - n_obj) * 4)

    def step(timed=False):
        flat.zero_()
        grads["shifts"].zero_()
        plan.forward_loss_grad(t, idx_t, off, lcfg, grads, grad_scale=1.0 / nb, loss_terms=terms,
                               max_batch=max_batch)
        if world > 1:
            e0 = torch.cuda.Event(enable_timing=True) if timed else None
            e1 = torch.cuda.Event(enable_timing=True) if timed else None
            if timed:
                e0.record(stream)
            if bands is None:
                ctx.allreduce(flat)    # object + probe gradients: ONE RCCL all-reduce per step
            else:
                ctx.allreduce(flat[n_obj:])                   # probe
                bands.reduce([grads["obja"], grads["objp"]])  # halo rows to their owners
            if timed:
                e1.record(stream)
                ar_ev.append((e0, e1))
        if bands is None:
            opt.step()
        else:
            for p_ in objs:
                p_.grad = None
            opt.step()                                        # probe, positions
            t["obja"].grad, t["objp"].grad = grads["obja"], grads["objp"]
            bands.step(opt, objs)                             # Adam on the owned rows
            if timed:
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record(stream)
            bands.gather(objs)
            if timed:
                e3 = torch.cuda.Event(enable_timing=True)
                e3.record(stream)
                ar_ev.append((e2, e3))

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    plan.profile_begin()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(timed=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kstats = plan.profile_end()
    assert bool(torch.isfinite(terms).all()), "non-finite loss terms"
    ar_ms = sum(e0.elapsed_time(e1) for e0, e1 in ar_ev) / a.steps if ar_ev else 0.0
    engine_ms = sum(v[1] for v in kstats.values()) / a.steps
    if world > 1:
        e = torch.tensor([elapsed, engine_ms, ar_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed, engine_max, ar_max = (float(x) for x in e.tolist())
    else:
        engine_max, ar_max = engine_ms, ar_ms
    total_patterns = world * n_local * a.steps if cfg["mode"] != "strong" else n_global * a.steps
    if a.geom_world:
        total_patterns = n_local * a.steps
    value = total_patterns / elapsed
    ms_per_step = 1e3 * elapsed / a.steps

    # roofline.  SURVEY §8d per pattern: B_alg = N^2 (s_m + 16 O Nz) bytes (DP read once, object patch
    # read and patch-gradient write), F_alg = n_fft 5 N^2 log2 N^2 flops, n_fft = 2 P O (2 Nz - 1) + 2P.
    s_m = 2 if f16 else 4
    b_alg = N * N * (s_m + 16 * O * Nz)
    n_fft = 2 * P * O * (2 * Nz - 1) + 2 * P
    f_alg = n_fft * 5 * N * N * math.log2(N * N)
    roof = None
    stripe = [k for k in kstats if k in ("k_s1", "k_s2", "k_s3", "k_s4", "k_s5")]
    # HBM traffic of the dominant kernel from its PMC passes (FETCH_SIZE x2 + WRITE_SIZE, separate
    # rocprofv3 --pmc runs of this bench command; tools/gpu_profile.sh -> profiles/make_traffic.py):
    # measured at the commit named in `traffic_source`, not inside this run
    tr = {}
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        tr = json.load(open(tpath)).get(a.config, {})
    tsrc = f"{tr['source']} (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE at {tr['measured_at']})" if tr else None
    if "k_fused" in kstats:
        # the register engines (k_fused3 / k_fused3ms): forward + loss + adjoint in one launch per call
        launches, dom_ms = kstats["k_fused"]
        avg_s = dom_ms / launches / 1e3
        per_launch = n_local / max(1, launches // a.steps)       # patterns per launch
        achieved = b_alg * per_launch / avg_s / 1e9
        traffic = round(tr["bytes_per_pattern"] * per_launch) if tr.get("bytes_per_pattern") else None
        roof = {"kernel": "k_fused3" if Nz == 1 else "k_fused3ms", "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "alg_bytes_per_launch": int(b_alg * per_launch), "avg_launch_ms": round(avg_s * 1e3, 4),
                "fft_fp32_frac": round(f_alg * per_launch / avg_s / 1e12 / FP32_PEAK_TFLOPS, 4)}
        g_launches, g_ms = kstats.get("k_obj_gather", (0, 0.0))
        if g_launches:
            g_s = g_ms / g_launches / 1e3
            roof["gather"] = {"avg_launch_ms": round(g_s * 1e3, 4),
                              "achieved_GBps": round(8 * N * N * Nz * per_launch / g_s / 1e9, 1)}
    elif stripe:
        # the N = 256 stripe engine (k_s1..k_s5): FP32-FFT bound (c3 AI 107, c5 AI 71 flop/B)
        s_ms = sum(kstats[k][1] for k in stripe) / a.steps
        achieved = f_alg * n_local / (s_ms / 1e3) / 1e12
        traffic, fabric = None, None
        if tr.get("bytes_per_pattern"):   # PMC bytes per pattern of the five passes, per step
            traffic = round(tr["bytes_per_pattern"] * n_local)
            fabric = round(traffic / (s_ms / 1e3) / 1e9, 1)
        roof = {"kernel": "stripe engine k_s1..k_s5", "bound": "fp32-valu", "achieved": round(achieved, 2),
                "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                "traffic": traffic, "traffic_unit": "bytes per step", "traffic_GBps": fabric,
                "traffic_source": tsrc, "alg_flops_per_step": f_alg * n_local,
                "engine_ms_per_step": round(s_ms, 3),
                "note": "the FFTs run on the vector ALUs (no MFMA); FP32 vector peak 157.3 TF",
                "hbm_alg_frac": round(b_alg * n_local / (s_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)}
    par = f"dp{world} (RCCL all-reduce of object+probe grads per step)" if world > 1 else "dp1"
    out = {
        "metric": "diffraction-patterns/sec/iter (fwd+bwd), 256x256 probe positions, 128x128 DP"
        if a.config.startswith("c2") else f"diffraction-patterns/sec/iter (fwd+bwd), BASELINE {a.config}",
        "value": round(value, 1), "unit": "patterns/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong" if cfg["mode"] == "strong" else "weak", "vs_baseline": None,
        "dtype": "f32", "data": data,
        "config": {"workload": desc + ", sub-px shifts on, " + {"single": "loss_single(q=0.5)", "poissn": "loss_poissn",
                                                                "both": "loss_single(q=0.5)+loss_poissn"}[a.loss]
                   + "+loss_sparse(L1), mini-batch "
                   f"{a.batch}, one Adam step per iteration (grad_accumulation = all mini-batches; all-reduce first)",
                   "N": N, "P": P, "O": O, "Nz": Nz, "dp_storage": "f16" if f16 else "f32",
                   "mini_batch": a.batch, "mini_batches_per_step": nb, "patterns_per_gpu_per_step": n_local,
                   "object": [Ny, Nx], "parallelism": par,
                   **({"tunings": tunings} if tunings else {}),
                   **({"capacity_env": {k: os.environ[k] for k in ("PTYX_STRIPE_MB", "PTYX_OBJ_SCRATCH_MB", "PTYX_FFC_MB")
                                        if k in os.environ}} if any(k in os.environ for k in
                                                                   ("PTYX_STRIPE_MB", "PTYX_OBJ_SCRATCH_MB", "PTYX_FFC_MB"))
                      else {}),
                   **({"geometry_only": f"rank {gr} of a {gw}-GPU scan, no collective"} if a.geom_world else {})},
        "roofline": roof,
        "per_rank_ms": {"engine": round(engine_max, 3), "allreduce": round(ar_max, 3),
                        "allreduce_bytes": int(flat.numel() * 4), "exchange": a.exchange if world > 1 else None,
                        "exchange_bytes_sent_per_rank": int(xbytes)},
        "fft_tflops": round(value / world * f_alg / 1e12, 2) if cfg["mode"] != "strong" else
        round(value * f_alg / 1e12 / world, 2),
        "kernels_ms_per_step": {k: round(v[1] / a.steps, 3) for k, v in kstats.items()},
        "launches_per_step": {k: v[0] // a.steps for k, v in kstats.items()},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
