"""The c3 / c4 / c5 bench workloads at their full bench geometry on MI355X.

The paths only the bench sizes reach: c5's 14418² object with f32 object-gradient
atomics and four stripe calls sharing PTYX_PREP_REUSE; c3's sixteen 1,024-pattern stripe calls with
per-pattern slots + k_obj_gather (two object modes); c4's calls of up to 32,768 patterns through
k_fused3ms and the tile-binned gather over the 3679² object with 16 slices.

1. The full bench call (tools/bench.py's geometry, ptyrad_amd.synthetic.bench_geometry), through
   size-independent properties: determinism where promised (c3 slots, c4 gather: bitwise; c5's
   atomics: to summation order), grad_scale linearity, split invariance (the same mini-batches in two
   engine calls: bitwise-identical loss terms, the same summed gradients), and locality (sampled
   mini-batches' loss terms equal the oracle run on just their patterns).
2. Gradients of a subset of mini-batches spread over the whole bench block, run through the same
   multi-call path (the per-call capacity forced down so the subset takes four calls with prep
   reuse and, for c3 / c4, the binned gather), against the complex64 oracle on the same inputs.

Reference: forward.py:57-79 (forward model), models.py:251-265 (patch gather and its scatter-add).
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


def bench_problem(config, device, seed=1234, world=1, rank=0):
    """bench.py's inputs for one GPU (rank `rank` of a `world`-GPU job's geometry): geometry, seeded
    random object, probe modes, uniform DPs."""
    from ptyrad_amd import synthetic as syn
    cfg = syn.BENCH_CONFIGS[config]
    N, P, O, Nz = cfg["N"], cfg["P"], cfg["O"], cfg["Nz"]
    crop_pos, shifts, (Ny, Nx), _, _ = syn.bench_geometry(config, world, rank)
    n = crop_pos.shape[0]
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    base = syn.stem_probe(N) * np.float32(60.0 if N == 128 else 30.0)
    probe_c = (syn.mixed_probe(base, P) if P > 1 else base[None]).astype(np.complex64)
    H = syn.fresnel_propagator(N, syn.DX_ANG, 2.0)
    t = {"obja": (1.0 + 0.05 * torch.randn((O, Nz, Ny, Nx), generator=g, device=device)).float(),
         "objp": (0.1 / Nz * torch.randn((O, Nz, Ny, Nx), generator=g, device=device)).float(),
         "probe": torch.view_as_real(torch.tensor(probe_c, device=device)).contiguous(),
         "shifts": torch.tensor(shifts, device=device), "H": torch.tensor(H, device=device),
         "occu": torch.tensor(syn.omode_occupancy(O), device=device), "crop_pos": torch.tensor(crop_pos, device=device)}
    gm = torch.Generator(device=device)
    gm.manual_seed(seed + 1)
    meas = torch.rand((n, N, N), generator=gm, device=device)
    t["meas"] = meas.half() if cfg["f16"] else meas
    return cfg, t, probe_c, H, crop_pos, shifts


def zero_grads(t):
    return {k: torch.zeros_like(t[k]) for k in ("obja", "objp", "probe", "shifts")}


def run_call(plan, t, batches, cfg_loss, scale=1.0, grads=None):
    from ptyrad_amd.engine import batch_offsets
    grads = grads if grads is not None else zero_grads(t)
    idx = torch.as_tensor(np.concatenate(batches), dtype=torch.int32, device=t["obja"].device)
    terms = plan.forward_loss_grad(t, idx, batch_offsets(batches), cfg_loss, grads, grad_scale=scale, max_batch=32)
    return terms.cpu().numpy(), grads


def grel(a, b):
    return rel(a.cpu().numpy(), b.cpu().numpy())


@pytest.mark.parametrize("config", ["c5", "c3", "c4"])
def test_full_bench_call_properties(config):
    device = dev()
    from ptyrad_amd.engine import LossConfig, Plan
    cfg, t, probe_c, H, crop_pos, shifts = bench_problem(config, device)
    n = crop_pos.shape[0]
    O, Nz, Ny, Nx = t["obja"].shape
    plan = Plan(cfg["N"], cfg["P"], O, Nz, Ny, Nx, n, n, shift_probes=True, meas_f16=cfg["f16"], device=device)
    rng = np.random.default_rng(7)
    batches = np.array_split(rng.permutation(n), n // 32)
    lcfg = LossConfig.from_loss_params(LP)
    plan.profile_begin()
    t1, g1 = run_call(plan, t, batches, lcfg)
    ks = plan.profile_end()
    calls = -(-n // plan.register_capacity)               # c5: 4, c3: 16, c4: 32 with the default capacities
    assert calls > 1
    engine = "k_fused" if config == "c4" else "k_s3"
    assert ks[engine][0] == calls, ks                     # the bench's call split
    if config in ("c3", "c4"):
        assert "k_obj_gather" in ks, ks
    t2, g2 = run_call(plan, t, batches, lcfg)
    np.testing.assert_array_equal(t1, t2)
    for k in g1:
        if config == "c5" and k in ("obja", "objp"):      # f32 atomics: the same sum in another order
            assert grel(g2[k], g1[k]) < 1e-6, k
        else:                                             # slots / gathers / fixed-order slabs
            assert torch.equal(g1[k], g2[k]), k
    del g2
    t3, g3 = run_call(plan, t, batches, lcfg, scale=0.5)
    np.testing.assert_array_equal(t1, t3)
    for k in g1:
        assert rel(g3[k].cpu().numpy(), 0.5 * g1[k].cpu().numpy()) < 1e-6, k
    del g3
    half = len(batches) // 2
    ta, gs = run_call(plan, t, batches[:half], lcfg)
    tb, gs = run_call(plan, t, batches[half:], lcfg, grads=gs)
    np.testing.assert_array_equal(np.concatenate([ta, tb]), t1)
    for k in g1:
        assert grel(gs[k], g1[k]) < 1e-6, k
    del gs
    assert all(bool(torch.isfinite(g1[k]).all()) for k in g1)
    # locality: a mini-batch's loss terms depend on its own patterns only
    oa, op = t["obja"].cpu().numpy(), t["objp"].cpu().numpy()
    occu = t["occu"].cpu().numpy()
    for k in rng.choice(len(batches), 2, replace=False):
        b = batches[k]
        mb = t["meas"][torch.as_tensor(b, device=device)].float().cpu().numpy()
        oterms, _, _ = orc.forward_loss_grad(oa, op, probe_c, shifts[b], crop_pos[b], H, occu, mb,
                                             [np.arange(len(b))], LP, cdt=np.complex64)
        np.testing.assert_allclose(t1[k], oterms[0], rtol=1e-5, atol=1e-7)


# per config: the subset's patterns and the capacity override that makes it four engine calls
SUBSET = {"c5": (512, "PTYX_STRIPE_MB", "512"),        # 4 MiB of stripe intermediates a pattern → 128 a call
          "c3": (256, "PTYX_STRIPE_MB", "1024"),       # 16 MiB a pattern → 64 a call
          "c4": (512, "PTYX_OBJ_SCRATCH_MB", "256")}   # 16 slot planes = 2 MiB a pattern → 128 a call


@pytest.mark.parametrize("config,world,rank", [("c5", 1, 0), ("c3", 1, 0), ("c4", 1, 0),
                                               ("c5", 8, 7), ("c3", 8, 3), ("c4", 8, 7)],
                         ids=["c5", "c3", "c4", "c5_rank7of8", "c3_rank3of8", "c4_rank7of8"])
def test_bench_geometry_subset_gradients_vs_oracle(config, world, rank, monkeypatch):
    """Also one rank's shard of the 8-GPU job (bench_geometry(config, 8, r): c4's rows split by rank,
    c3 / c5's block starting at the rank's first scan row): the replicated object, of which the
    shard's windows touch one band (the engines' bounding box / tile skips), the last rank's band
    at the object's bottom edge."""
    device = dev()
    from ptyrad_amd.engine import LossConfig, Plan, batch_offsets
    n_sub, env, mb_cap = SUBSET[config]
    monkeypatch.setenv(env, mb_cap)
    cfg, t, probe_c, H, crop_pos, shifts = bench_problem(config, device, seed=99, world=world, rank=rank)
    if world > 1:   # the shard's rows are its own band, away from the single-rank block's
        assert int(crop_pos[:, 0].min()) > 0
    n = crop_pos.shape[0]
    O, Nz, Ny, Nx = t["obja"].shape
    rng = np.random.default_rng(11)
    sel = rng.choice(n, n_sub, replace=False)            # spread over the whole bench block
    batches = np.array_split(sel, n_sub // 32)
    plan = Plan(cfg["N"], cfg["P"], O, Nz, Ny, Nx, n, n_sub, shift_probes=True, meas_f16=cfg["f16"], device=device)
    assert plan.register_capacity == n_sub // 4, plan.register_capacity
    grads = zero_grads(t)
    plan.profile_begin()
    terms = plan.forward_loss_grad(t, np.concatenate(batches).astype(np.int32), batch_offsets(batches),
                                   LossConfig.from_loss_params(LP), grads, grad_scale=1.0 / len(batches))
    torch.cuda.synchronize()
    ks = plan.profile_end()
    engine = "k_fused" if config == "c4" else "k_s3"
    assert ks[engine][0] == 4, ks                        # four calls: PTYX_PREP_FULL then three REUSE
    assert ks["k_obj_prep"][0] == 1, ks                  # the object prepared once for the four
    if config in ("c3", "c4"):
        assert "k_obj_gather" in ks, ks
    # the oracle on the sub-problem: the positions re-indexed 0..n_sub-1, the full object
    order = np.sort(sel)
    loc = [np.searchsorted(order, b) for b in batches]
    m = t["meas"][torch.as_tensor(order, device=device)].float().cpu().numpy()
    oterms, _, og = orc.forward_loss_grad(t["obja"].cpu().numpy(), t["objp"].cpu().numpy(), probe_c, shifts[order],
                                          crop_pos[order], H, t["occu"].cpu().numpy(), m, loc, LP,
                                          cdt=np.complex64, grad_scale=1.0 / len(batches))
    np.testing.assert_allclose(terms.cpu().numpy(), oterms, rtol=1e-5, atol=1e-7)
    assert rel(grads["obja"].cpu().numpy(), og["obja"]) < 5e-5
    assert rel(grads["objp"].cpu().numpy(), og["objp"]) < 5e-5
    gp = grads["probe"].cpu().numpy()
    assert rel(gp[..., 0] + 1j * gp[..., 1], og["probe"]) < 5e-5
    assert rel(grads["shifts"].cpu().numpy()[order], og["shifts"]) < 2e-4
