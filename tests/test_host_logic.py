"""Host-side logic that needs no GPU: batching, index selection, loss-config mapping."""
import numpy as np
import pytest

from ptyrad_amd.engine import LossConfig, batch_offsets
from ptyrad_amd.reconstruction import make_batches, select_scan_indices, toggle_grad_requires


def test_batch_offsets():
    b = [np.arange(3), np.arange(3, 5), np.arange(5, 9)]
    assert batch_offsets(b).tolist() == [0, 3, 5, 9]
    assert batch_offsets(b).dtype == np.int32


def test_make_batches_random_is_a_partition():
    idx = np.arange(100)
    bs = make_batches(idx, None, 32, rng=np.random.default_rng(0))
    assert len(bs) == 3                               # len // batch_size groups (array_split)
    flat = np.sort(np.concatenate(bs))
    assert np.array_equal(flat, idx)
    assert sorted(len(b) for b in bs) == [33, 33, 34]


def test_select_scan_indices_modes():
    assert np.array_equal(select_scan_indices(4, 5), np.arange(20))
    c = select_scan_indices(4, 4, 2, 2, mode="center")
    assert sorted(c.tolist()) == [5, 6, 9, 10]
    s = select_scan_indices(4, 4, 2, 2, mode="sub")
    assert sorted(s.tolist()) == [0, 3, 12, 15]
    with pytest.raises(ValueError):
        select_scan_indices(4, 4, mode="bogus")


def test_loss_config_mapping_and_out_of_scope_terms():
    lp = {"loss_single": {"state": True, "weight": 2.0, "dp_pow": 0.4},
          "loss_poissn": {"state": True, "weight": 0.5, "dp_pow": 1.0, "eps": 1e-5},
          "loss_pacbed": {"state": False}, "loss_sparse": {"state": True, "weight": 0.2, "ln_order": 2},
          "loss_simlar": {"state": False}}
    c = LossConfig.from_loss_params(lp)
    assert (c.single_on, c.single_w, c.single_q) == (True, 2.0, 0.4)
    assert (c.poissn_on, c.poissn_w, c.poissn_eps) == (True, 0.5, 1e-5)
    assert (c.sparse_on, c.sparse_n) == (True, 2)
    cs = c.to_c(0.25)
    assert abs(cs.grad_scale - 0.25) < 1e-9
    lp["loss_pacbed"] = {"state": True, "weight": 0.3, "dp_pow": 0.25}     # HIP ptyx_loss_pacbed
    c = LossConfig.from_loss_params(lp)
    assert (c.pacbed_on, c.pacbed_w, c.pacbed_q) == (True, 0.3, 0.25)
    only = LossConfig(single_on=False, poissn_on=False, pacbed_on=True).to_c(1.0)
    assert (only.single_on, only.single_w) == (1, 0.0)      # zero-weight data term for the engine
    lp["loss_simlar"]["state"] = True
    with pytest.raises(NotImplementedError):
        LossConfig.from_loss_params(lp)


def test_toggle_grad_requires_follows_start_iter():
    import torch

    class M:
        pass
    m = M()
    m.start_iter = {"obja": 1, "probe": 3, "obj_tilts": None}
    m.optimizable_tensors = {k: torch.zeros(1, requires_grad=False) for k in m.start_iter}
    toggle_grad_requires(m, 2)
    assert [m.optimizable_tensors[k].requires_grad for k in ("obja", "probe", "obj_tilts")] == [True, False, False]
    toggle_grad_requires(m, 3)
    assert m.optimizable_tensors["probe"].requires_grad


def test_make_batches_sparse_matches_reference_greedy_rule():
    """'sparse' grouping (reconstruction.py:548-587): seeds nearest the compact centroids, then
    each remaining index joins the group whose nearest member is farthest.  Checked against a
    direct restatement with the reference's full pairwise-distance matrix on the same clusters."""
    from scipy.spatial.distance import cdist
    from ptyrad_amd.reconstruction import sparse_groups
    rng = np.random.default_rng(3)
    yy, xx = np.meshgrid(np.arange(9), np.arange(9), indexing="ij")
    pos = np.stack([yy.ravel(), xx.ravel()], 1) * 2.87 + rng.normal(0, 0.15, (81, 2))
    idx = np.arange(81)
    compact = make_batches(idx, pos, 10, mode="compact", random_state=0)
    got = sparse_groups(idx, pos, compact)
    # reference rule, literally
    pw = cdist(pos, pos)
    pos_s = pos[idx]
    groups, used = [], []
    for cb in compact:
        c = np.mean(pos[cb], axis=0)
        j = int(np.argmin(np.linalg.norm(pos_s - c, axis=1)))
        groups.append([idx[j]])
        used.append(j)
    for i in np.delete(idx.copy(), used):
        g = int(np.argmax([np.min(pw[grp, i]) for grp in groups]))
        groups[g].append(i)
    assert [list(g) for g in got] == [list(map(int, g)) for g in groups]
    assert np.array_equal(np.sort(np.concatenate(got)), idx)
    bs = make_batches(idx, pos, 10, mode="sparse", random_state=0)
    assert np.array_equal(np.sort(np.concatenate(bs)), idx)


def test_hip_adam_class_is_torch_adam_and_runs_torch_step_on_cpu():
    """ptyrad_amd.optim.Adam is a torch.optim.Adam; on CPU tensors (no kernel) its step() is
    torch's own, bit for bit."""
    import torch
    from ptyrad_amd import optim
    g = torch.Generator().manual_seed(0)
    a = torch.randn(5, 7, generator=g)
    p1, p2 = a.clone().requires_grad_(), a.clone().requires_grad_()
    o1, o2 = optim.Adam([p1], lr=1e-2, weight_decay=0.1), torch.optim.Adam([p2], lr=1e-2, weight_decay=0.1)
    assert isinstance(o1, torch.optim.Adam)
    for _ in range(3):
        gr = torch.randn(5, 7, generator=g)
        p1.grad, p2.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    assert torch.equal(p1, p2)
    o3 = torch.optim.Adam([p2], lr=1e-2)
    o3.load_state_dict(o1.state_dict())


def test_stepgraph_tables_and_eligibility_on_cpu():
    """StepGraphs' per-iteration tables (first pattern / first mini-batch of every optimizer step,
    per rank: whole groups, parts of split groups or the rank's whole mini-batches), the
    persistent buffers a reshuffled batching is copied into, and recon_step's refusal of
    graphs=True without a HIP device."""
    import numpy as np
    import torch
    from ptyrad_amd.reconstruction import DistContext
    from ptyrad_amd.stepgraph import StepGraphs, _local_steps, ineligible_reason
    batches = [np.array([5, 1, 9]), np.array([2, 7]), np.array([0, 3, 4]), np.array([8, 6])]
    sg = StepGraphs()
    steps = _local_steps(None, batches, 3)
    assert [(s[1], s[2], s[3]) for s in steps] == [(3, False, (0, 1, 2)), (1, False, (0,))]
    idx_all, istart, rstart = sg._tables(steps, 3, torch.device("cpu"))
    assert idx_all.tolist() == [5, 1, 9, 2, 7, 0, 3, 4, 8, 6]
    assert istart.tolist() == [0, 8] and rstart.tolist() == [0, 3]       # steps of 3 and 1 mini-batches
    assert sg._tables(steps, 3, torch.device("cpu"))[0] is idx_all       # cached while the batches stay
    shuffled = [np.array([9, 5, 1]), np.array([7, 2]), np.array([4, 0, 3]), np.array([6, 8])]
    again = sg._tables(_local_steps(None, shuffled, 3), 3, torch.device("cpu"))
    assert again[0] is idx_all and idx_all.tolist() == [9, 5, 1, 7, 2, 4, 0, 3, 6, 8]   # same buffers, new table
    # two ranks: ga = 1 splits each mini-batch (rank 1 takes the second part), ga = 2 deals whole ones
    ctx = DistContext()
    ctx.rank, ctx.world, ctx.always_reduce = 1, 2, True
    st1 = _local_steps(ctx, batches, 1)
    assert [p.tolist() for s in st1 for p in s[0]] == [[9], [7], [4], [6]] and all(s[2] and s[3] == () for s in st1)
    st2 = _local_steps(ctx, batches, 2)
    assert [p.tolist() for s in st2 for p in s[0]] == [[2, 7], [8, 6]] and [s[3] for s in st2] == [(1,), (1,)]
    tab = StepGraphs()._tables(st2, 2, torch.device("cpu"))
    assert tab[1].tolist() == [0, 2] and tab[2].tolist() == [0, 2]

    class M:
        opt_obja = torch.zeros(1)
    assert ineligible_reason(M(), None, None, None, batches, 1) == "no HIP device"


def test_check_plans_names_the_iteration():
    """recon_step surfaces device-flagged input errors after the iteration's sync (graph-replayed
    steps bypass Plan's per-call check), naming the iteration; plans without errors pass."""
    import pytest
    from ptyrad_amd.reconstruction import check_plans

    class _Plan:
        def __init__(self, bad):
            self.bad, self.calls = bad, 0

        def _prev_errors(self):
            self.calls += 1
            if self.bad:
                raise IndexError("scan index 70000 out of range [0, 65536)")

    class _Model:
        pass
    m = _Model()
    m._plan, m._stack_plans = _Plan(False), {32: _Plan(False)}
    check_plans(m, 3)
    assert m._plan.calls == 1 and m._stack_plans[32].calls == 1
    m._stack_plans[64] = _Plan(True)
    with pytest.raises(IndexError, match=r"recon_step iteration 7: scan index 70000"):
        check_plans(m, 7)
    m2 = _Model()
    m2._plan = None
    check_plans(m2, 1)          # a pre-blur model without its main plan yet
