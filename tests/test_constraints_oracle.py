"""CPU: the constraints oracle (oracle/constraints_oracle.py) against the reference's own
CombinedConstraint outputs (tests/golden/cons_*.npz, made by make_golden_constraints.py)."""
import glob
import json
import os

import numpy as np
import pytest

from oracle import constraints_oracle as co

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLD, "cons_*.npz")))


def load_case(name):
    z = np.load(os.path.join(GOLD, f"cons_{name}.npz"))
    cp = json.loads(str(z["constraint_params"]))
    return z, cp


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(np.asarray(b)), 1e-30))


def test_cases_present():
    assert {"default_p1", "default_p4o2z6", "options", "freq", "fourier", "rblur", "rblur_k7"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    z, cp = load_case(name)
    st = {"obja": z["obja"], "objp": z["objp"], "probe": z["probe"], "probe_int_sum": z["probe_int_sum"]}
    out = co.combined(cp, st, int(z["niter"]))
    # f32 reference vs f64 oracle: object values are O(1)
    assert np.max(np.abs(out["obja"] - z["out_obja"])) < 2e-6, name
    assert np.max(np.abs(out["objp"] - z["out_objp"])) < 2e-6, name
    # probe: orthogonalisation runs in complex64 LAPACK in the reference
    assert rel(out["probe"], z["out_probe"]) < 2e-5, name


def test_gaussian_kernels():
    k = co.gaussian1d_scipy(5, 1.0)
    assert abs(float(k.sum()) - 1.0) < 1e-6 and k[2] == k.max()
    t = co.gaussian1d_torchvision(5, 0.5)
    assert abs(float(t.sum()) - 1.0) < 1e-6 and np.allclose(t, t[::-1])


def test_ortho_modes_orthogonal():
    _, cp = load_case("default_p4o2z6")
    z, _ = load_case("default_p4o2z6")
    o = co.orthogonalize_modes(z["probe"].astype(np.complex128))
    M = o.reshape(o.shape[0], -1)
    G = M @ M.conj().T
    off = G - np.diag(np.diag(G))
    assert np.abs(off).max() < 1e-9 * np.abs(np.diag(G)).max()
    w = np.real(np.diag(G))
    assert np.all(np.diff(w) <= 0)


def test_host_config_marshalling():
    """CombinedConstraint's frequency gating and the ptyx_obj_constraints struct (no GPU call)."""
    import copy

    from ptyrad_amd.constraints import CombinedConstraint
    from tests.golden.constraint_defaults import DEFAULTS
    cp = copy.deepcopy(DEFAULTS)
    cp["objp_postiv"].update(mode="subtract_min", relax=0.25)
    cp["obj_zblur"].update(freq=2, obj_type="phase", kernel_size=7, std=1.5)
    cc = CombinedConstraint(cp, device="cpu", verbose=False)
    c1 = cc._obj_cfg(1, zblur=True, pointwise=True)
    assert (c1.zblur_a, c1.zblur_p) == (0, 0)                  # freq 2 skips iteration 1
    assert c1.mir_on == 1 and abs(c1.mir_relax - 0.1) < 1e-7 and c1.mir_power == 4.0
    assert c1.thr_on == 1 and abs(c1.thr_lo - 0.98) < 1e-7 and abs(c1.thr_hi - 1.02) < 1e-7
    assert c1.pos_on == 1 and c1.pos_subtract_min == 1 and c1.pos_relax == 0.25
    assert c1.cr_a == 0 and c1.cr_p == 0                        # complex_ratio off by default
    c2 = cc._obj_cfg(2, zblur=True, pointwise=False)
    assert (c2.zblur_a, c2.zblur_p, c2.zblur_ks) == (0, 1, 7) and c2.mir_on == 0
