"""GPU: the on-device CombinedConstraint (ptyrad_amd/constraints.py → libptyx HIP kernels) against
the reference's own outputs (tests/golden/cons_*.npz) and the oracle at larger sizes."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle import constraints_oracle as co
from tests.golden.constraint_defaults import DEFAULTS

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLD, "cons_*.npz")))


class Model:
    """The attributes CombinedConstraint reads (constraints.py:34-224), on cuda:0."""

    def __init__(self, obja, objp, probe, probe_int_sum, dev):
        self.opt_obja = torch.nn.Parameter(torch.tensor(obja, device=dev))
        self.opt_objp = torch.nn.Parameter(torch.tensor(objp, device=dev))
        self.opt_probe = torch.nn.Parameter(torch.view_as_real(torch.tensor(probe, device=dev)).contiguous())
        self.opt_obj_tilts = torch.nn.Parameter(torch.zeros(1, 2, device=dev))
        self.probe_int_sum = torch.tensor(probe_int_sum, dtype=torch.float32, device=dev)
        self.device = dev
        self.N_scan_slow = self.N_scan_fast = 1

    def get_complex_probe_view(self):
        return torch.view_as_complex(self.opt_probe)


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("name", CASES)
def test_hip_constraints_match_reference(name, dev):
    from ptyrad_amd.constraints import CombinedConstraint
    z = np.load(os.path.join(GOLD, f"cons_{name}.npz"))
    cp = json.loads(str(z["constraint_params"]))
    m = Model(z["obja"], z["objp"], z["probe"], float(z["probe_int_sum"]), dev)
    CombinedConstraint(cp, device=dev, verbose=False)(m, int(z["niter"]))
    torch.cuda.synchronize()
    a, p = m.opt_obja.detach().cpu().numpy(), m.opt_objp.detach().cpu().numpy()
    pr = torch.view_as_complex(m.opt_probe.detach()).cpu().numpy()
    # fp32 tolerance (values O(1)): 2e-6 absolute on the object, 2e-5 relative L2 on the probe
    assert np.max(np.abs(a - z["out_obja"])) < 2e-6, (name, np.max(np.abs(a - z["out_obja"])))
    assert np.max(np.abs(p - z["out_objp"])) < 2e-6, (name, np.max(np.abs(p - z["out_objp"])))
    assert rel(pr, z["out_probe"]) < 2e-5, (name, rel(pr, z["out_probe"]))


def test_default_chain_large_multislice(dev):
    """c4-like object (16 slices, 2 object modes, 640² here) through the one-pass default chain."""
    from ptyrad_amd.constraints import CombinedConstraint
    rng = np.random.default_rng(11)
    obja = (1 + 0.05 * rng.standard_normal((2, 16, 640, 640))).astype(np.float32)
    objp = (0.02 + 0.1 * rng.standard_normal((2, 16, 640, 640))).astype(np.float32)
    probe = (rng.standard_normal((1, 64, 64)) + 1j * rng.standard_normal((1, 64, 64))).astype(np.complex64)
    m = Model(obja, objp, probe, 123.0, dev)
    CombinedConstraint(DEFAULTS, device=dev, verbose=False)(m, 1)
    want = co.combined(DEFAULTS, {"obja": obja, "objp": objp, "probe": probe, "probe_int_sum": 123.0}, 1)
    assert np.max(np.abs(m.opt_obja.detach().cpu().numpy() - want["obja"])) < 2e-6
    assert np.max(np.abs(m.opt_objp.detach().cpu().numpy() - want["objp"])) < 2e-6
    got_pr = torch.view_as_complex(m.opt_probe.detach()).cpu().numpy()
    assert abs(float((np.abs(got_pr.astype(np.complex128)) ** 2).sum()) - 123.0) < 1e-3   # fix_probe_int
    assert rel(got_pr, want["probe"]) < 1e-6


def test_ortho_eight_modes_orthonormal_and_deterministic(dev):
    """c3's 8 probe modes at N = 256: V^H M is orthogonal, sorted, and bitwise reproducible."""
    from ptyrad_amd.constraints import CombinedConstraint
    rng = np.random.default_rng(12)
    probe = (rng.standard_normal((8, 256, 256)) + 1j * rng.standard_normal((8, 256, 256))).astype(np.complex64)
    probe *= (0.7 ** np.arange(8))[:, None, None].astype(np.float32)
    cp = {"ortho_pmode": {"freq": 1}}
    outs = []
    for _ in range(2):
        m = Model(np.ones((1, 1, 8, 8), np.float32), np.zeros((1, 1, 8, 8), np.float32), probe, 1.0, dev)
        CombinedConstraint(cp, device=dev, verbose=False)(m, 1)
        outs.append(torch.view_as_complex(m.opt_probe.detach()).cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    want = co.orthogonalize_modes(probe.astype(np.complex128))
    assert rel(outs[0], want) < 2e-5
    M = outs[0].reshape(8, -1).astype(np.complex128)
    G = M @ M.conj().T
    d = np.real(np.diag(G))
    assert np.all(np.diff(d) <= 0)
    assert np.abs(G - np.diag(np.diag(G))).max() < 1e-5 * d.max()


@pytest.mark.parametrize("P", [17, 24, 40, 64])
def test_ortho_many_modes_vs_oracle(dev, P):
    """ortho_pmode beyond 16 probe modes (the wave-parallel Jacobi and the padded apply kernels):
    against the oracle's orthogonalize_modes (numpy eig), orthogonal, sorted, bitwise repeatable."""
    from ptyrad_amd.constraints import CombinedConstraint
    rng = np.random.default_rng(100 + P)
    probe = (rng.standard_normal((P, 64, 64)) + 1j * rng.standard_normal((P, 64, 64))).astype(np.complex64)
    probe *= (0.93 ** np.arange(P))[:, None, None].astype(np.float32)
    cp = {"ortho_pmode": {"freq": 1}}
    outs = []
    for _ in range(2):
        m = Model(np.ones((1, 1, 8, 8), np.float32), np.zeros((1, 1, 8, 8), np.float32), probe, 1.0, dev)
        CombinedConstraint(cp, device=dev, verbose=False)(m, 1)
        outs.append(torch.view_as_complex(m.opt_probe.detach()).cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    want = co.orthogonalize_modes(probe.astype(np.complex128))
    assert rel(outs[0], want) < 5e-5
    M = outs[0].reshape(P, -1).astype(np.complex128)
    G = M @ M.conj().T
    d = np.real(np.diag(G))
    assert np.all(np.diff(d) <= 0)
    assert np.abs(G - np.diag(np.diag(G))).max() < 2e-5 * d.max()
