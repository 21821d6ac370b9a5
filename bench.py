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

  --cadence reference  recon_step at grad_accumulation = 1 (the reference's default cadence), c2 scan,
             mini-batches split over the ranks, graph-replayed steps with captured RCCL collectives

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
       torchrun --nproc-per-node N bench.py --gpus N ...   (driver, one rank per GPU, RCCL)
  Without torchrun, --gpus N > 1 starts the N rank processes itself (launch_ranks: fresh
  processes, rank 0's JSON line only, non-zero exit when a rank fails or fewer GPUs are visible).
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
    ap.add_argument("--exchange", default="auto", choices=["auto", "allreduce", "band"],
                    help="N > 1: object gradients by one flat all-reduce, or by row band (ObjectBands: halo "
                         "rows to their owners, Adam on the owned band, updated halo rows back to their "
                         "readers; no all-gather); auto (default) = band when the ranks' touched object rows "
                         "line up by rank within a window (every weak-scaling config), as recon_step's "
                         "DistContext decides.  With --geom-world W the band bytes of rank --geom-rank are "
                         "computed from the W ranks' geometry (no collective)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--geom-world", type=int, default=0,
                    help="diagnostic (c2): build rank --geom-rank's shard of a W-GPU weak-scaling geometry on one GPU "
                         "(no collective) to check that per-rank work stays constant as W grows")
    ap.add_argument("--geom-rank", type=int, default=0)
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="engine variant for A/B runs (ptyx_set_tuning, include/ptyx.h); recorded in the output")
    ap.add_argument("--cadence", default="iteration", choices=["iteration", "reference"],
                    help="iteration: one optimizer step per pass over the shard (default, the headline); "
                         "reference: recon_step at grad_accumulation = 1 (the reference's default cadence) on "
                         "the c2 scan, every mini-batch split over the ranks, graph-replayed steps with their "
                         "RCCL collectives captured; one bench step = one recon_step iteration")
    ap.add_argument("--flat-exchange", action="store_true",
                    help="--cadence reference: all-reduce the whole flat gradient in split steps instead of the "
                         "slot exchange (DistContext(slot_exchange=False))")
    ap.add_argument("--rank-timeout", type=float, default=3000.0,
                    help="--gpus N > 1 without torchrun: seconds before the launcher stops a job that has not ended")
    ap.add_argument("--always-reduce", action="store_true",
                    help="--cadence reference at one GPU: init RCCL anyway and run every collective of the "
                         "multi-rank step (split mini-batches), as an 8-GPU job would")
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


def _alg_flops(cfg):
    """SURVEY §8d F_alg per pattern: n_fft 5 N² log2 N², n_fft = 2 P O (2 Nz - 1) + 2 P (shifts on)."""
    N, P, O, Nz = cfg["N"], cfg["P"], cfg["O"], cfg["Nz"]
    return (2 * P * O * (2 * Nz - 1) + 2 * P) * 5 * N * N * math.log2(N * N)


def _cpu_worker(args):
    config, seed, nbatch, bsize = args
    from oracle import ptyx_oracle as orc
    from ptyrad_amd import synthetic as syn
    cfg = CONFIGS[config]
    N = cfg["N"]
    pr = syn.random_problem(N, 16, 16, P=cfg["P"], O=cfg["O"], Nz=cfg["Nz"], seed=seed)
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False}, "loss_pacbed": {"state": False},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1}, "loss_simlar": {"state": False}}
    rng = np.random.default_rng(seed)
    batches = [rng.choice(256, bsize, replace=False) for _ in range(nbatch)]
    t = time.perf_counter()
    orc.forward_loss_grad(pr.obja, pr.objp, pr.probe * np.float32(60.0 if N == 128 else 30.0), pr.shifts,
                          pr.crop_pos, pr.H, pr.occu, pr.meas, batches, lp, cdt=np.complex64)
    return nbatch * bsize, time.perf_counter() - t


def cpu_baseline(config, bsize, sample):
    """Oracle (NumPy port of the reference path) at the config's own shape (N, P, O, Nz) on the
    host cores, one process per core, before any GPU call.  sample 0: about 20 s of work (≈ 110
    patterns/s per core at the c2 shape, scaled by the shape's FFT work, at least one mini-batch
    per core)."""
    import multiprocessing as mp
    cfg = CONFIGS[config]
    cores = host_cores()
    if not sample:
        per_core_rate = 110.0 * _alg_flops(CONFIGS["c2"]) / _alg_flops(cfg)
        sample = int(per_core_rate * 20 * cores)
    nb_total = max(cores, sample // bsize)
    per = [nb_total // cores + (1 if i < nb_total % cores else 0) for i in range(cores)]
    jobs = [(config, 100 + i, per[i], bsize) for i in range(cores) if per[i] > 0]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    pats = sum(r[0] for r in res)
    busy = max(r[1] for r in res)     # the workers' compute (they run concurrently), pool start excluded
    shape = f"N={cfg['N']}, P={cfg['P']}, O={cfg['O']}, Nz={cfg['Nz']}"
    out = {"value": round(pats / busy, 1), "unit": "patterns/s", "cores": len(jobs), "kind": "port",
           "shape": f"{config}: {shape}",
           "sample": f"{pats} patterns of the {config} shape ({shape}, f32 DPs; {len(jobs)} processes x mini-batches "
                     f"of {bsize}), shifts on, loss_single(q=0.5)+loss_sparse(L1), oracle/ptyx_oracle.py complex64 "
                     f"NumPy; rate over the slowest worker's compute time {busy:.1f}s (wall {wall:.1f}s incl. pool "
                     f"start: {pats / wall:.1f} patterns/s)"}
    r = cpu_ratio(config)
    if r:   # reference CPU path vs this port at the same shape, same cores, measured in the build container
        out["ratio_to_reference"] = r["ratio_reference_over_port"]
        out["reference_equivalent"] = round(out["value"] * r["ratio_reference_over_port"], 1)
        out["ratio_measured"] = f"{r['host']}: reference {r['reference_patterns_per_s']} / port " \
                                f"{r['port_patterns_per_s']} patterns/s at the {config} shape " \
                                f"(tests/golden/measure_cpu_ratio.py)"
    return out


def cpu_ratio(key):
    """tests/golden/cpu_ratio.json's entry for `key` (a config, or 'c2_refcad': recon_step with
    Adam at grad_accumulation = 1), or None."""
    path = os.path.join(ROOT, "tests", "golden", "cpu_ratio.json")
    if not os.path.exists(path):
        return None
    r = json.load(open(path))
    e = r.get("configs", {}).get(key)
    return {**e, "host": r["host"]} if e else None


def cpu_adam_ms(shapes, reps=5):
    """One torch.optim.Adam step (single-tensor arithmetic, NumPy fp32) over tensors of the given
    shapes on one host core: the per-optimizer-step cost a CPU run of the reference's default
    cadence pays on top of the mini-batch's forward / loss / gradient."""
    rng = np.random.default_rng(0)
    ts = [(rng.random(s, dtype=np.float32), rng.random(s, dtype=np.float32) - np.float32(0.5),
           np.zeros(s, np.float32), np.zeros(s, np.float32)) for s in shapes]
    b1, b2, lr, eps = np.float32(0.9), np.float32(0.999), 5e-4, np.float32(1e-8)
    best = float("inf")
    for r in range(reps):
        t = time.perf_counter()
        step = r + 1
        bc1, bc2s = 1.0 - 0.9 ** step, math.sqrt(1.0 - 0.999 ** step)
        for p, g, m, v in ts:
            m += (g - m) * (np.float32(1.0) - b1)
            v *= b2
            v += (np.float32(1.0) - b2) * g * g
            p += np.float32(-lr / bc1) * m / (np.sqrt(v) / np.float32(bc2s) + eps)
        best = min(best, time.perf_counter() - t)
    return 1e3 * best


def with_adam(cpu, shapes, bsize):
    """cpu_baseline at the reference's default cadence: every mini-batch of `bsize` also pays one
    Adam step over the full parameter set (each worker process its own, as independent replicas)."""
    if not cpu:
        return cpu
    ms = cpu_adam_ms(shapes)
    per_core = cpu["value"] / cpu["cores"]                  # patterns/s of one process
    t_batch = bsize / per_core
    out = dict(cpu)
    out["value"] = round(cpu["cores"] * bsize / (t_batch + ms / 1e3), 1)
    out["value_without_adam"] = cpu["value"]
    out["adam_ms_per_optimizer_step"] = round(ms, 2)
    out["sample"] = cpu["sample"] + (f"; plus one NumPy fp32 Adam step (torch single-tensor order) over the c2 "
                                     f"parameters {[list(s) for s in shapes]} per mini-batch of {bsize}, "
                                     f"{ms:.1f} ms on one core (grad_accumulation = 1, like for like)")
    for k in ("ratio_to_reference", "reference_equivalent", "ratio_measured"):
        out.pop(k, None)
    r = cpu_ratio("c2_refcad")
    if r:   # the reference's own recon_step WITH Adam at grad_accumulation = 1 vs this Adam-inclusive port
        out["ratio_to_reference"] = r["ratio_reference_over_port"]
        out["reference_equivalent"] = round(out["value"] * r["ratio_reference_over_port"], 1)
        out["ratio_measured"] = f"{r['host']}: reference recon_step + Adam {r['reference_patterns_per_s']} / port + " \
                                f"Adam {r['port_patterns_per_s']} patterns/s (tests/golden/measure_cpu_ratio.py)"
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


def reference_cadence(a, world, rank, local, cpu):
    """--cadence reference: what a PtyRAD user's multi-GPU job runs.  recon_step
    (reconstruction.py:658-781) at the reference's default grad_accumulation = 1
    (params/recon_params.py:17) on the c2 geometry: the 256x256 scan, make_batches 'random' with 32
    positions a mini-batch (identical on every rank), every mini-batch split over the ranks
    (accelerate's split_batches, utils/common.py:63 — the global mini-batch stays 32, so this is
    strong scaling), each rank holding only its parts' DPs, hipGraph-replayed optimizer steps with
    the loss-sum and gradient RCCL all-reduces captured inside them, the HIP Adam.  One bench step
    = one recon_step iteration = 2,048 optimizer steps over all 65,536 positions."""
    import torch
    import torch.distributed as dist
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import Plan
    from ptyrad_amd.losses import CombinedLoss
    from ptyrad_amd.models import PtychoHIP
    from ptyrad_amd.reconstruction import DistContext, create_optimizer, make_batches, recon_step
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or a.always_reduce:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    ctx = DistContext(split_batches=True if a.always_reduce else None, always_reduce=a.always_reduce,
                      slot_exchange=not a.flat_exchange)
    N = 128
    crop_pos, shifts, (Ny, Nx), _, _ = syn.bench_geometry("c2", 1, 0, scan=a.scan)
    n = crop_pos.shape[0]
    lrs = {"obja": 5e-4, "objp": 5e-4, "obj_tilts": 0.0, "slice_thickness": 0.0, "probe": 1e-4,
           "probe_pos_shifts": 1e-4}
    lp = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
          "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
          "loss_pacbed": {"state": False, "weight": 0.5, "dp_pow": 0.2},
          "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1}, "loss_simlar": {"state": False}}
    probe = syn.stem_probe(N) * np.float32(60.0)
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    # DPs: the engine's forward model of the ground-truth object (as the default cadence)
    plan = Plan(N, 1, 1, 1, Ny, Nx, n, n, shift_probes=True, device=dev)
    gta, gtp = gt_object((1, 1, Ny, Nx), dev)
    t = {"obja": gta, "objp": gtp, "probe": torch.view_as_real(torch.tensor(probe[None], device=dev)).contiguous(),
         "shifts": torch.tensor(shifts, device=dev), "H": torch.tensor(H, device=dev),
         "occu": torch.ones(1, device=dev), "crop_pos": torch.tensor(crop_pos, device=dev)}
    meas = torch.empty((n, N, N), dtype=torch.float32, device=dev)
    plan.forward(t, np.arange(n, dtype=np.int32), dp_out=meas)
    del gta, gtp, t, plan
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    iv = {"obja": np.ones((1, 1, Ny, Nx), np.float32),
          "objp": (1e-8 * torch.rand((1, 1, Ny, Nx), generator=g, device=dev)).cpu().numpy(), "obj": None,
          "probe": probe[None], "probe_pos_shifts": shifts, "omode_occu": np.ones(1, np.float32), "H": H,
          "crop_pos": crop_pos, "N_scan_slow": int(round(math.sqrt(n))), "N_scan_fast": int(round(math.sqrt(n))),
          "slice_thickness": 2.0, "dx": syn.DX_ANG, "dk": 1.0 / (N * syn.DX_ANG),
          "lambd": syn.electron_wavelength(syn.KV), "obj_tilts": np.zeros((1, 2), np.float32)}
    mp_ = {"detector_blur_std": None, "obj_preblur_std": None,
           "update_params": {k: {"start_iter": 1 if v else None, "lr": v} for k, v in lrs.items()},
           "optimizer_params": {"name": "Adam", "configs": {}, "load_state": None}}
    batches = make_batches(np.arange(n), crop_pos, a.batch, mode="random", verbose=False,
                           rng=np.random.default_rng(3))
    loss_fn = CombinedLoss(lp, device=dev)
    mi = ctx.local_indices(batches, 1, loss_fn=loss_fn, model_params=mp_, init_variables=iv)
    iv["measurements"] = meas[torch.as_tensor(mi, device=dev)].contiguous()
    iv["measurements_index"] = mi
    del meas
    model = PtychoHIP(iv, mp_, device=dev, verbose=False)
    opt = create_optimizer(model.optimizer_params, model.optimizable_params)
    it = 0
    for _ in range(a.warmup):
        it += 1
        recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, dist_ctx=ctx)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        it += 1
        recon_step(batches, 1, model, opt, loss_fn, None, it, verbose=False, dist_ctx=ctx)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    sg = getattr(model, "_step_graphs", None)
    n_steps = len(batches)
    last = float(model.loss_iters[-1][1])
    # bytes a rank sends per optimizer step in the gradient exchange of a W-rank job (ring
    # collectives: an all-reduce sends 2(W-1)/W of its buffer, an all-gather (W-1) x the rank's
    # share).  Slot exchange: ⌈B/W⌉ slots (N² complex64) + table rows all-gathered, the probe
    # gradient and loss terms all-reduced; flat: the object, probe and position gradients all-reduced
    W_x = a.geom_world or world
    n_obj, n_pr, n_sh = 2 * Ny * Nx, 2 * N * N, 2 * n
    cap_x = -(-a.batch // W_x)
    ring = 2 * (W_x - 1) / W_x
    slot_b = (W_x - 1) * cap_x * (2 * N * N + 8) * 4 + ring * (n_pr + 5) * 4
    flat_b = ring * (n_obj + n_pr + n_sh + 5) * 4
    use_slots = bool(ctx.slot_exchange) and (world > 1 or a.always_reduce or a.geom_world > 1)
    assert math.isfinite(last), "non-finite loss"
    out = {
        "metric": "diffraction-patterns/sec/iter (fwd+bwd), 256x256 probe positions, 128x128 DP",
        "value": round(n * a.steps / elapsed, 1), "unit": "patterns/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: DPs = engine forward model of a ground-truth atom-lattice object; recon init exp(1e-8 iU)",
        "config": {"workload": f"c2 scan {int(round(math.sqrt(n)))}^2 at the reference's default cadence: recon_step, "
                               f"grad_accumulation = 1, mini-batches of {a.batch} ('random') split over the ranks, "
                               "loss_single(q=0.5)+loss_sparse(L1), HIP Adam; one bench step = one iteration",
                   "cadence": "reference", "N": N, "P": 1, "O": 1, "Nz": 1, "mini_batch": a.batch,
                   "optimizer_steps_per_iteration": n_steps, "object": [Ny, Nx],
                   "parallelism": f"dp{world} (split mini-batches; per optimizer step an RCCL loss-sum all-reduce, then "
                                  + ("the slot exchange: object-gradient slots all-gathered, probe gradient and "
                                     "loss terms all-reduced" if use_slots else "the flat gradient all-reduce")
                                  + f"{', forced at world size 1' if a.always_reduce and world == 1 else ''})"},
        "ms_per_optimizer_step": round(1e3 * elapsed / a.steps / n_steps, 4),
        "exchange": {"mode": ("slots" if use_slots else "allreduce") if (world > 1 or a.always_reduce) else None,
                     "world_for_bytes": W_x,
                     "bytes_sent_per_rank_per_step": int(slot_b if use_slots else flat_b),
                     "slot_exchange_bytes": int(slot_b), "flat_allreduce_bytes": int(flat_b),
                     **({"geometry_only": f"bytes of a {W_x}-rank job; this run has {world} rank(s)"}
                        if a.geom_world else {})},
        "graphs": {"captures": sg.captures, "replays": sg.replays, "eager": sg.eager} if sg else None,
        "loss_last_iteration": last,
        "roofline": None,
        "roofline_note": "32-pattern optimizer steps are launch / latency bound; the kernel roofline is the "
                         "default (--cadence iteration) line's",
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


# ------------------------------------------------------------------ rank launcher
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus() -> int:
    """GPUs this process could use, counted without initialising the GPU (torch.cuda.device_count
    does not create a HIP context on this image; is_available() would)."""
    import torch
    return int(torch.cuda.device_count())


def launch_ranks(n, cmd, timeout=None, env=None, poll_s=0.2, out=None):
    """Run ``cmd`` as ``n`` fresh rank processes of one job (one per GPU, the launch torchrun would
    make: RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR 127.0.0.1 / MASTER_PORT in
    their environment) and forward rank 0's stdout only; every rank's stderr passes through.  The
    launcher itself never touches the GPU.  The first rank that exits non-zero, or a job still
    running after ``timeout`` seconds, ends the job: the other ranks' process groups are killed and
    the exit status returned is non-zero (the failing rank's code, 124 on a timeout).  Returns 0
    when every rank exits 0."""
    import signal
    import subprocess
    out = out if out is not None else sys.stdout
    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(_free_port())})
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True, text=True))

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    import threading
    lines = []

    def pump():                        # rank 0's stdout, forwarded as it arrives
        for line in procs[0].stdout:
            lines.append(line)
            out.write(line)
            out.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t0 = time.monotonic()
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[bench] rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr)
                status = c if c > 0 else 128 - c
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"[bench] the {n}-rank job exceeded {timeout:.0f} s; stopping it", file=sys.stderr)
                status = 124
                break
            time.sleep(poll_s)
    finally:
        kill_all()
        th.join(timeout=5)
    return status


def main():
    a = parse()
    cfg = CONFIGS[a.config]
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: start the N ranks here, one fresh process per
        # GPU, and never touch the GPU in this process
        have = visible_gpus()
        if have < a.gpus:
            print(f"[bench] --gpus {a.gpus} needs {a.gpus} visible GPUs, this host shows {have}", file=sys.stderr)
            raise SystemExit(2)
        raise SystemExit(launch_ranks(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      timeout=a.rank_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE {world}: the launcher must start one rank per GPU",
              file=sys.stderr)
        raise SystemExit(2)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline("c2" if a.cadence == "reference" or a.config == "c2-strong" else a.config,
                           a.batch, a.cpu_sample)                # before the GPU is touched
    if a.cadence == "reference":
        if a.config != "c2":
            raise SystemExit("--cadence reference runs the c2 geometry")
        if cpu:
            from ptyrad_amd import synthetic as syn
            crop_pos, _, (Ny, Nx), _, _ = syn.bench_geometry("c2", 1, 0, scan=a.scan)
            cpu = with_adam(cpu, [(1, 1, Ny, Nx), (1, 1, Ny, Nx), (1, 128, 128, 2), (crop_pos.shape[0], 2)], a.batch)
        return reference_cadence(a, world, rank, local, cpu)

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
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
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
    row_b = t["obja"].shape[0] * t["obja"].shape[1] * Nx * 4 * 2      # one object row, amplitude + phase
    exchange = a.exchange
    if world > 1 and exchange != "allreduce":
        from ptyrad_amd.reconstruction import ObjectBands, exchange_ranges
        rows = exchange_ranges(ctx, int(crop_pos[:, 0].min()), int(crop_pos[:, 0].max()) + N, dev)
        if exchange == "band" or ObjectBands.disjoint(rows, Ny, world, N):
            exchange = "band"
            bands = ObjectBands(ctx, Ny, dev, rows)
            objs = [t["obja"], t["objp"]]
        else:
            exchange = "allreduce"
    # bytes each rank sends per step in the exchange (ring all-reduce: 2(W-1)/W of the buffer; band:
    # its touched rows outside its band to their owners + its band rows others read back to them,
    # + the ring all-reduce of the probe part)
    W_x = gw if a.geom_world else world
    xb = bands
    if a.geom_world and W_x > 1 and exchange != "allreduce":
        # --geom-world: the W ranks' touched rows from the geometry alone
        from ptyrad_amd.reconstruction import ObjectBands

        class _Ctx:
            rank, world, group = gr, gw, None
        rows = []
        for r_ in range(gw):
            cp_ = syn.bench_geometry(a.config, gw, r_, a.patterns, a.scan)[0]
            rows.append((int(cp_[:, 0].min()), int(cp_[:, 0].max()) + N))
        if exchange == "band" or ObjectBands.disjoint(rows, Ny, gw, N):
            exchange = "band"
            xb = ObjectBands(_Ctx(), Ny, "cpu", rows)
        else:
            exchange = "allreduce"
    if xb is not None:
        xbytes = ((xb.sent_rows() + xb.halo_rows()) * row_b +
                  2 * (W_x - 1) / W_x * (flat.numel() - n_obj) * 4)
    else:
        xbytes = 2 * (W_x - 1) / W_x * flat.numel() * 4 if W_x > 1 else 0

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
            bands.halo(objs)                                  # updated rows back to their readers
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
                        "allreduce_bytes": int(flat.numel() * 4),
                        "exchange": exchange if (world > 1 or a.geom_world) else None,
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
