"""Speed ratio of the oracle port (bench.py's cpu_baseline leg) to the reference's own CPU path,
measured in THIS container with the same workload.

    python tests/golden/measure_cpu_ratio.py [c2 c3 c4 c5 c2_refcad]   (build container only: imports
                                                                        /root/reference)

Per bench config shape (N, P, O, Nz of BENCH_CONFIGS; sub-pixel shifts on, loss_single q = 0.5 +
loss_sparse L1, mini-batches of 32) both legs run on the same number of host cores:
  reference  PtychoAD.forward + CombinedLoss + backward (models.py:422, losses.py:143, autograd),
             torch CPU with torch.set_num_threads(cores);
  port       bench.cpu_baseline(): oracle/ptyx_oracle.py complex64 NumPy in `cores` processes, the
             SAME function and the same default sample per core (110 · 20 patterns) as on the GPU
             box, its rate taken over the workers' compute time (pool start excluded) on both.
Harness: one warm-up pass, then the median of 3 timed passes of the whole sample.
'c2_refcad' times the reference's own recon_step WITH its Adam step at grad_accumulation = 1 (the
--cadence reference line's like-for-like) against the port plus bench.with_adam's per-mini-batch
Adam.  Writes tests/golden/cpu_ratio.json (numbers only, one entry per config), which bench.py
reports as cpu_baseline.ratio_to_reference: reference patterns/s ≈ port patterns/s × ratio.
"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

from refimport import import_reference  # noqa: E402

LOSS = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
        "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
        "loss_pacbed": {"state": False, "weight": 0.5, "dp_pow": 0.2},
        "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
        "loss_simlar": {"state": False, "weight": 0.1, "obj_type": "both", "scale_factor": [1, 1, 1],
                        "blur_std": 1}}


def reference_rate(cores, config="c2", n_batches=None, bsize=32):
    """PtychoAD.forward + CombinedLoss + backward at the config's shape (16 x 16 scan)."""
    models, losses, _ = import_reference()
    import bench
    import make_golden as mg
    cfg = bench.CONFIGS[config]
    N, P, O, Nz = cfg["N"], cfg["P"], cfg["O"], cfg["Nz"]
    if n_batches is None:   # about 2-3 s a pass at the reference's measured rates
        n_batches = max(4, int(64 * bench._alg_flops(bench.CONFIGS["c2"]) / bench._alg_flops(cfg)))
    torch.set_num_threads(cores)
    scan, probe, H, occu, obja, objp, _, _ = mg.make_inputs(N, P, O, Nz, 16, 16, seed=100)
    S = scan.crop_pos.shape[0]
    meas = np.random.default_rng(0).random((S, N, N), dtype=np.float32)
    iv = mg.init_variables(obja, objp, probe, H, occu, scan.crop_pos, scan.shifts, meas, 16, 16)
    model = models.PtychoAD(iv, mg.model_params(5e-4), device="cpu", verbose=False)
    loss_fn = losses.CombinedLoss(LOSS, device="cpu")
    rng = np.random.default_rng(1)
    batches = [rng.choice(S, bsize, replace=False) for _ in range(n_batches)]

    def one_pass():
        t = time.perf_counter()
        for b in batches:
            dp = model(b)
            total, _ = loss_fn(dp, model.get_measurements(b), model._current_object_patches, model.omode_occu)
            total.backward()
        return time.perf_counter() - t

    one_pass()
    ts = [one_pass() for _ in range(3)]
    return n_batches * bsize / statistics.median(ts)


def reference_recon_rate(cores, n_batches=48, bsize=32):
    """The reference's own recon_step (reconstruction.py:658-781) WITH its Adam step at
    grad_accumulation = 1, on the c2 object (the bench's c2 raster, 1033² object, so Adam updates
    the real parameter sizes) over a block of the raster's positions, constraints a no-op (as the
    bench's --cadence reference line runs it)."""
    models, losses, _ = import_reference()
    import make_golden as mg
    import ptyrad.reconstruction as rec
    from ptyrad_amd import synthetic as syn
    torch.set_num_threads(cores)
    crop_pos, shifts, (Ny, Nx), _, _ = syn.bench_geometry("c2", 1, 0)
    S = n_batches * bsize
    crop_pos, shifts = crop_pos[:S], shifts[:S]
    N = 128
    rng = np.random.default_rng(5)
    obja = np.ones((1, 1, Ny, Nx), np.float32)
    objp = (1e-8 * rng.random((1, 1, Ny, Nx))).astype(np.float32)
    probe = (syn.stem_probe(N) * np.float32(60.0))[None]
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    meas = rng.random((S, N, N), dtype=np.float32)
    iv = mg.init_variables(obja, objp, probe, H, np.ones(1, np.float32), crop_pos, shifts, meas, n_batches, bsize)
    model = models.PtychoAD(iv, mg.model_params(1e-4), device="cpu", verbose=False)
    loss_fn = losses.CombinedLoss(LOSS, device="cpu")
    opt = rec.create_optimizer(model.optimizer_params, model.optimizable_params, verbose=False)
    batches = np.array_split(np.random.default_rng(3).permutation(S), n_batches)
    it = [0]

    def one_pass():
        it[0] += 1
        t = time.perf_counter()
        rec.recon_step(batches, 1, model, opt, loss_fn, lambda m, n: None, it[0], verbose=False)
        return time.perf_counter() - t

    one_pass()
    ts = [one_pass() for _ in range(3)]
    return S / statistics.median(ts), [(1, 1, Ny, Nx), (1, 1, Ny, Nx), (1, N, N, 2), (65536, 2)]


def port_rate(cores, config="c2", sample=0, adam_shapes=None):
    import bench
    bench_cores = os.environ.get("PTYX_CPU_CORES")
    os.environ["PTYX_CPU_CORES"] = str(cores)
    try:
        bench.cpu_baseline(config, 32, cores * 32)   # warm-up (pool start, imports)
        rs = []
        for _ in range(3):
            c = bench.cpu_baseline(config, 32, sample)
            if adam_shapes:
                c = bench.with_adam(c, adam_shapes, 32)
            rs.append(c["value"])
    finally:
        if bench_cores is None:
            os.environ.pop("PTYX_CPU_CORES", None)
        else:
            os.environ["PTYX_CPU_CORES"] = bench_cores
    return statistics.median(rs)


def main():
    import bench
    cores = len(os.sched_getaffinity(0))
    path = os.path.join(HERE, "cpu_ratio.json")
    out = {"host": f"{cores} cores (build container)", "cores": cores,
           "workload": "loss_single q=0.5 + loss_sparse L1, shifts on, mini-batch 32; reference = PtyRAD CPU "
                       "(torch threads = cores), port = bench.cpu_baseline (one process per core, default sample, "
                       "compute-time rate); median of 3 passes after a warm-up",
           "configs": {}}
    for config in [a for a in sys.argv[1:] if not a.startswith("-")] or ["c2", "c3", "c4", "c5", "c2_refcad"]:
        if config == "c2_refcad":
            ref, shapes = reference_recon_rate(cores)
            port = port_rate(cores, "c2", 0, adam_shapes=shapes)
            what = "reference recon_step with torch Adam at grad_accumulation = 1 on the c2 object (1033^2) vs " \
                   "the port with bench.with_adam's NumPy Adam per mini-batch"
        else:
            ref = reference_rate(cores, config)
            port = port_rate(cores, config, 0)
            c = bench.CONFIGS[config]
            what = f"N={c['N']}, P={c['P']}, O={c['O']}, Nz={c['Nz']} (f32 DPs on both legs)"
        out["configs"][config] = {"shape": what, "reference_patterns_per_s": round(ref, 1),
                                  "port_patterns_per_s": round(port, 1),
                                  "ratio_reference_over_port": round(ref / port, 4)}
        print(config, json.dumps(out["configs"][config]), flush=True)
    if os.path.exists(path):   # keep entries measured earlier that this run did not redo
        old = json.load(open(path)).get("configs", {})
        out["configs"] = {**old, **out["configs"]}
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
