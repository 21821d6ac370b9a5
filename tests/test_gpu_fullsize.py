"""The bench workload at its full size on MI355X (c2: 256×256 scan = 65,536 patterns, N = 128,
object 1033², mini-batches of 32, one engine call), checked through size-independent properties:

* determinism: two identical calls give bitwise-identical loss terms and gradients (fixed-order
  reductions, no atomics on this path);
* linearity: grad_scale 0.5 halves every gradient (rel ≤ 1e-6) and leaves the loss terms alone;
* split invariance: the same batches in two calls give bitwise-identical per-batch loss terms and
  the same summed gradients (rel ≤ 1e-6; only the summation order differs);
* locality: each mini-batch's loss terms depend on its own 32 patterns only, so sampled batches
  of the full call match the oracle run on just those patterns (rtol 1e-5).
"""
import numpy as np
import pytest
import torch

from oracle import ptyx_oracle as orc
from tests.test_oracle_golden import rel

pytestmark = pytest.mark.gpu
LP = {"loss_single": {"state": True, "weight": 1.0, "dp_pow": 0.5},
      "loss_poissn": {"state": False, "weight": 1.0, "dp_pow": 1.0, "eps": 1e-6},
      "loss_pacbed": {"state": False}, "loss_sparse": {"state": True, "weight": 0.1, "ln_order": 1},
      "loss_simlar": {"state": False}}


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("gather_rows", [-1, 1], ids=["default_gather", "row_gather"])
def test_c2_full_call_properties(gather_rows):
    """gather_rows 1: every unsplit object gather is k_obj_gather_rows (one compensated sequential
    sum per pixel over its ≈ 2,000 hits; the default for small mixed-state calls) — the same
    properties hold at the full c2 call."""
    device = dev()
    from ptyrad_amd import _lib
    _lib.set_tuning("gather_rows", gather_rows)
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets
    N, S = 128, 256
    scan = syn.raster_scan(S, S, N, seed=0)
    Ny, Nx = scan.obj_shape
    n = S * S
    g = torch.Generator(device=device)
    g.manual_seed(1234)
    obja = (1.0 + 0.05 * torch.randn((1, 1, Ny, Nx), generator=g, device=device)).float()
    objp = (0.1 * torch.randn((1, 1, Ny, Nx), generator=g, device=device)).float()
    probe_c = (syn.stem_probe(N) * np.float32(60.0)).astype(np.complex64)
    gm = torch.Generator(device=device)
    gm.manual_seed(4321)
    meas = torch.rand((n, N, N), generator=gm, device=device)
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    t = {"obja": obja, "objp": objp, "probe": torch.view_as_real(torch.tensor(probe_c, device=device)[None]).contiguous(),
         "shifts": torch.tensor(scan.shifts, device=device), "H": torch.tensor(H, device=device),
         "occu": torch.ones(1, device=device), "crop_pos": torch.tensor(scan.crop_pos, device=device), "meas": meas}
    plan = Plan(N, 1, 1, 1, Ny, Nx, n, n, shift_probes=True, device=device)
    rng = np.random.default_rng(7)
    batches = np.array_split(rng.permutation(n), n // 32)
    cfg = LossConfig.from_loss_params(LP)

    def run(bs, scale=1.0, grads=None):
        grads = grads if grads is not None else {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
        idx_t = torch.as_tensor(np.concatenate(bs), dtype=torch.int32, device=device)
        off_t = torch.as_tensor(batch_offsets(bs), device=device)
        terms = plan.forward_loss_grad(t, idx_t, off_t, cfg, grads, grad_scale=scale, max_batch=32)
        return terms.cpu().numpy(), grads

    t1, g1 = run(batches)
    t2, g2 = run(batches)
    np.testing.assert_array_equal(t1, t2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    del g2
    t3, g3 = run(batches, scale=0.5)
    np.testing.assert_array_equal(t1, t3)
    for k in g1:
        assert rel(g3[k].cpu().numpy(), 0.5 * g1[k].cpu().numpy()) < 1e-6, k
    del g3
    half = len(batches) // 2
    ta, gs = run(batches[:half])
    tb, gs = run(batches[half:], grads=gs)
    np.testing.assert_array_equal(np.concatenate([ta, tb]), t1)
    for k in g1:
        assert rel(gs[k].cpu().numpy(), g1[k].cpu().numpy()) < 1e-6, k
    del gs
    oa, op = obja.cpu().numpy(), objp.cpu().numpy()
    for k in rng.choice(len(batches), 3, replace=False):
        b = batches[k]
        mb = meas[torch.as_tensor(b, device=device)].cpu().numpy()
        oterms, _, _ = orc.forward_loss_grad(oa, op, probe_c[None], scan.shifts[b], scan.crop_pos[b], H,
                                             np.ones(1, np.float32), mb, [np.arange(len(b))], LP)
        np.testing.assert_allclose(t1[k], oterms[0], rtol=1e-5, atol=1e-7)


def test_c2_geometry_gradients_of_2048_patterns_vs_oracle():
    """Object / probe / position gradients at the full c2 geometry (1033² object, positions spread
    over the whole 256² raster) for 64 random mini-batches of 32 (2,048 patterns; the register
    engine with segments crossing mini-batch and workgroup boundaries) vs the complex64 oracle on
    the same inputs."""
    device = dev()
    from ptyrad_amd import synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets
    N, S = 128, 256
    scan = syn.raster_scan(S, S, N, seed=0)
    Ny, Nx = scan.obj_shape
    n = S * S
    rng = np.random.default_rng(11)
    oa = (1.0 + 0.05 * rng.standard_normal((1, 1, Ny, Nx))).astype(np.float32)
    op = (0.1 * rng.standard_normal((1, 1, Ny, Nx))).astype(np.float32)
    probe_c = (syn.stem_probe(N) * np.float32(60.0)).astype(np.complex64)
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    sel = rng.choice(n, 2048, replace=False)
    batches = np.array_split(sel, 64)
    # DPs only for the selected positions (the rest are never read); rows in scan order
    meas = torch.zeros((n, N, N), device=device)
    m_sel = rng.random((sel.size, N, N), dtype=np.float32)
    meas[torch.as_tensor(sel, device=device)] = torch.tensor(m_sel, device=device)
    t = {"obja": torch.tensor(oa, device=device), "objp": torch.tensor(op, device=device),
         "probe": torch.view_as_real(torch.tensor(probe_c, device=device)[None]).contiguous(),
         "shifts": torch.tensor(scan.shifts, device=device), "H": torch.tensor(H, device=device),
         "occu": torch.ones(1, device=device), "crop_pos": torch.tensor(scan.crop_pos, device=device), "meas": meas}
    plan = Plan(N, 1, 1, 1, Ny, Nx, n, 2048, shift_probes=True, device=device)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    plan.profile_begin()
    terms = plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                                   LossConfig.from_loss_params(LP), grads, grad_scale=1.0 / 64)
    torch.cuda.synchronize()
    assert "k_fused" in plan.profile_end()          # the register engine (k_fused3)
    # the oracle on the sub-problem: the 2,048 positions re-indexed 0..2047, full object
    loc = [np.searchsorted(np.sort(sel), b) for b in batches]
    order = np.sort(sel)
    m_sorted = np.empty_like(m_sel)
    m_sorted[np.searchsorted(order, sel)] = m_sel
    oterms, _, og = orc.forward_loss_grad(oa, op, probe_c[None], scan.shifts[order], scan.crop_pos[order], H,
                                          np.ones(1, np.float32), m_sorted, loc, LP, cdt=np.complex64,
                                          grad_scale=1.0 / 64)
    np.testing.assert_allclose(terms.cpu().numpy(), oterms, rtol=1e-5, atol=1e-7)
    assert rel(grads["obja"].cpu().numpy(), og["obja"]) < 5e-5
    assert rel(grads["objp"].cpu().numpy(), og["objp"]) < 5e-5
    gp = grads["probe"].cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], og["probe"]) < 5e-5
    assert rel(grads["shifts"].cpu().numpy()[order], og["shifts"]) < 2e-4


@pytest.mark.parametrize("gather_rows", [0, 1], ids=["wave_partials", "row_gather"])
def test_dense_block_gather_vs_oracle(gather_rows):
    """Both object-gradient gathers where every object tile has hundreds of hits: 2,048 patterns of
    a compact 32 × 64 block of the c2 raster (≈ 180 × 310 px of windows' origins, so an object
    tile sees ≈ 500 windows), vs the complex64 oracle on the same inputs (rel 5e-5, as the
    spread-out 2,048-pattern test)."""
    device = dev()
    from ptyrad_amd import _lib, synthetic as syn
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets
    _lib.set_tuning("gather_rows", gather_rows)
    N, S = 128, 256
    scan = syn.raster_scan(S, S, N, seed=0)
    Ny, Nx = scan.obj_shape
    n = S * S
    rng = np.random.default_rng(12)
    oa = (1.0 + 0.05 * rng.standard_normal((1, 1, Ny, Nx))).astype(np.float32)
    op = (0.1 * rng.standard_normal((1, 1, Ny, Nx))).astype(np.float32)
    probe_c = (syn.stem_probe(N) * np.float32(60.0)).astype(np.complex64)
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    rows, cols = np.arange(100, 132), np.arange(80, 144)
    sel = (rows[:, None] * S + cols[None, :]).reshape(-1)
    sel = sel[rng.permutation(sel.size)]
    batches = np.array_split(sel, 64)
    meas = torch.zeros((n, N, N), device=device)
    m_sel = rng.random((sel.size, N, N), dtype=np.float32)
    meas[torch.as_tensor(sel, device=device)] = torch.tensor(m_sel, device=device)
    t = {"obja": torch.tensor(oa, device=device), "objp": torch.tensor(op, device=device),
         "probe": torch.view_as_real(torch.tensor(probe_c, device=device)[None]).contiguous(),
         "shifts": torch.tensor(scan.shifts, device=device), "H": torch.tensor(H, device=device),
         "occu": torch.ones(1, device=device), "crop_pos": torch.tensor(scan.crop_pos, device=device), "meas": meas}
    plan = Plan(N, 1, 1, 1, Ny, Nx, n, 2048, shift_probes=True, device=device)
    grads = {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}
    terms = plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                                   LossConfig.from_loss_params(LP), grads, grad_scale=1.0 / 64)
    torch.cuda.synchronize()
    cy = scan.crop_pos[sel, 0]
    cx = scan.crop_pos[sel, 1]
    # hits of the busiest 64 x 16 tile: windows overlapping it
    ty, tx = int(np.median(cy)) // 16 * 16, int(np.median(cx)) // 64 * 64
    hits = int(np.sum((cy > ty - N) & (cy < ty + 16) & (cx > tx - N) & (cx < tx + 64)))
    assert hits >= 400, hits
    order = np.sort(sel)
    loc = [np.searchsorted(order, b) for b in batches]
    m_sorted = np.empty_like(m_sel)
    m_sorted[np.searchsorted(order, sel)] = m_sel
    oterms, _, og = orc.forward_loss_grad(oa, op, probe_c[None], scan.shifts[order], scan.crop_pos[order], H,
                                          np.ones(1, np.float32), m_sorted, loc, LP, cdt=np.complex64,
                                          grad_scale=1.0 / 64)
    np.testing.assert_allclose(terms.cpu().numpy(), oterms, rtol=1e-5, atol=1e-7)
    assert rel(grads["obja"].cpu().numpy(), og["obja"]) < 5e-5
    assert rel(grads["objp"].cpu().numpy(), og["objp"]) < 5e-5
