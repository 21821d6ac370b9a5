"""Diagnostic: graph-replayed recon_step with and without PTYX_PREP_GRAD_STORE against eager steps,
on a reference trajectory fixture (default traj_n32_p2_ga2: the general engine, two probe modes).
    python tools/diag_store.py [traj name] [iterations]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_helpers import gpu_recon  # noqa: E402
from ptyrad_amd.stepgraph import StepGraphs  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


name = sys.argv[1] if len(sys.argv) > 1 else "traj_n32_p2_ga2"
nit = int(sys.argv[2]) if len(sys.argv) > 2 else 1
z = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
out = {}
for tag, graphs, store in (("eager", False, True), ("graph_store", True, True), ("graph_nostore", True, False)):
    StepGraphs.STORE = store
    m = gpu_recon(z, graphs=graphs, niter=nit)
    out[tag] = {k: getattr(m, k).detach().cpu().numpy() for k in ("opt_obja", "opt_objp", "opt_probe")}
    sg = getattr(m, "_step_graphs", None)
    print(tag, "captures/replays/eager", (sg.captures, sg.replays, sg.eager) if sg else None, flush=True)
for tag in ("graph_store", "graph_nostore"):
    print(tag, {k: rel(out[tag][k], out["eager"][k]) for k in out["eager"]}, flush=True)
