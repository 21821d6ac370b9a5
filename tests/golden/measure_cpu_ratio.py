"""Speed ratio of the oracle port (bench.py's cpu_baseline leg) to the reference's own CPU path,
measured in THIS container with the same workload.

    python tests/golden/measure_cpu_ratio.py        (build container only: imports /root/reference)

Both legs run the c2 hot path shape (N = 128, P = O = Nz = 1, sub-pixel shifts on, loss_single
q = 0.5 + loss_sparse L1, mini-batches of 32) on the same number of host cores:
  reference  PtychoAD.forward + CombinedLoss + backward (models.py:422, losses.py:143, autograd),
             torch CPU with torch.set_num_threads(cores);
  port       bench.cpu_baseline(): oracle/ptyx_oracle.py complex64 NumPy in `cores` processes, the
             SAME function and the same default sample per core (110 · 20 patterns) as on the GPU
             box, its rate taken over the workers' compute time (pool start excluded) on both.
Harness: one warm-up pass, then the median of 3 timed passes of the whole sample.
Writes tests/golden/cpu_ratio.json (numbers only), which bench.py reports as
cpu_baseline.ratio_to_reference: reference patterns/s ≈ port patterns/s × ratio.
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


def reference_rate(cores, n_batches=64, bsize=32):
    models, losses, _ = import_reference()
    import make_golden as mg
    from ptyrad_amd import synthetic as syn
    torch.set_num_threads(cores)
    scan, probe, H, occu, obja, objp, _, _ = mg.make_inputs(128, 1, 1, 1, 16, 16, seed=100)
    S = scan.crop_pos.shape[0]
    meas = np.random.default_rng(0).random((S, 128, 128), dtype=np.float32)
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
    return n_batches * bsize / statistics.median(ts), syn


def port_rate(cores, sample):
    import bench
    bench_cores = os.environ.get("PTYX_CPU_CORES")
    os.environ["PTYX_CPU_CORES"] = str(cores)
    try:
        bench.cpu_baseline(128, 32, max(1024, sample // 4))   # warm-up (pool start, imports)
        rs = [bench.cpu_baseline(128, 32, sample)["value"] for _ in range(3)]
    finally:
        if bench_cores is None:
            os.environ.pop("PTYX_CPU_CORES", None)
        else:
            os.environ["PTYX_CPU_CORES"] = bench_cores
    return statistics.median(rs)


def main():
    cores = len(os.sched_getaffinity(0))
    ref, _ = reference_rate(cores)
    port = port_rate(cores, 0)          # 0: bench.py's default sample (110 · 20 patterns per core)
    out = {"host": f"{cores} cores (build container)", "cores": cores, "workload": "c2 shape: N=128, P=O=Nz=1, "
           "shifts on, loss_single q=0.5 + loss_sparse L1, mini-batch 32",
           "port_sample": "bench.cpu_baseline default (110 x 20 patterns per core), compute-time rate",
           "reference_patterns_per_s": round(ref, 1), "port_patterns_per_s": round(port, 1),
           "ratio_reference_over_port": round(ref / port, 4)}
    with open(os.path.join(HERE, "cpu_ratio.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
