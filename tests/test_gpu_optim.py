"""ptyrad_amd.optim.Adam / AdamW (one ptyx_adam_step launch for every group) against torch's own
Adam / AdamW on the CPU — the single-tensor path PtyRAD's CPU runs take and the optimizer the
reference trajectories (tests/golden/traj_*.npz) were made with."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _groups(shapes_lrs, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    ts = [torch.randn(s, generator=g) for s, _ in shapes_lrs]
    return ts, [(t.clone().to(dev).requires_grad_(), lr) for t, (_, lr) in zip(ts, shapes_lrs)]


@pytest.mark.parametrize("name,wd", [("Adam", 0.0), ("Adam", 0.01), ("AdamW", 0.01)])
def test_hip_adam_matches_torch_cpu_adam(name, wd):
    dev = need_gpu()
    from ptyrad_amd import optim
    shapes = [((1, 1, 257, 263), 5e-4), ((1, 1, 257, 263), 5e-4), ((1, 128, 128, 2), 1e-4), ((4096, 2), 1e-4),
              ((1,), 1e-3)]
    cpu_t, dev_t = _groups(shapes, dev)
    cpu_p = [t.clone().requires_grad_() for t in cpu_t]
    ref = getattr(torch.optim, name)([{"params": [p], "lr": lr} for p, (_, lr) in zip(cpu_p, shapes)],
                                     weight_decay=wd, foreach=False)
    hip = getattr(optim, name)([{"params": [p], "lr": lr} for p, lr in dev_t], weight_decay=wd)
    assert isinstance(hip, getattr(torch.optim, name))
    g = torch.Generator().manual_seed(7)
    start = [t.clone() for t in cpu_t]
    for it in range(6):
        grads = [torch.randn(t.shape, generator=g) * (10.0 ** (it % 3 - 1)) for t in cpu_t]
        for p, gr in zip(cpu_p, grads):
            p.grad = gr.clone()
        for (p, _), gr in zip(dev_t, grads):
            p.grad = gr.to(dev)
        if it == 3:   # a frozen tensor this step (no .grad): skipped, its step count stays
            cpu_p[2].grad = None
            dev_t[2][0].grad = None
        ref.step()
        hip.step()
    # the parameters' displacement over the six steps agrees to fp32 rounding of the update
    # (relative L2 and elementwise against the step size)
    for p, (q, lr), p0 in zip(cpu_p, dev_t, start):
        d_ref = (p.detach() - p0).double().numpy()
        d_hip = (q.detach().cpu() - p0).double().numpy()
        assert np.linalg.norm(d_hip - d_ref) <= 1e-5 * np.linalg.norm(d_ref), name
        ulp = np.spacing(np.abs(p.detach().numpy())).astype(np.float64)   # one fp32 ulp of the parameter
        assert np.all(np.abs(d_hip - d_ref) <= 2 * ulp + 1e-4 * lr), name
    for p, (q, _) in zip(cpu_p, dev_t):
        sr, sh = ref.state[p], hip.state[q]
        assert float(sr["step"]) == float(sh["step"].cpu())
        np.testing.assert_allclose(sh["exp_avg"].cpu().numpy(), sr["exp_avg"].numpy(), rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(sh["exp_avg_sq"].cpu().numpy(), sr["exp_avg_sq"].numpy(), rtol=1e-6, atol=1e-12)


def test_hip_adam_state_dict_moves_to_torch_adam_and_graph_replay():
    """The state_dict loads into torch.optim.Adam (and back) and continues identically; a step
    captured in a hipGraph and replayed equals eager steps."""
    dev = need_gpu()
    from ptyrad_amd import optim
    shapes = [((1, 1, 300, 300), 5e-4), ((1, 64, 64, 2), 1e-4)]
    _, a_t = _groups(shapes, dev, seed=1)
    _, b_t = _groups(shapes, dev, seed=1)
    A = optim.Adam([{"params": [p], "lr": lr} for p, lr in a_t])
    B = optim.Adam([{"params": [p], "lr": lr} for p, lr in b_t])
    gen = torch.Generator(device=dev).manual_seed(3)
    grads = [[torch.randn(p.shape, generator=gen, device=dev) for p, _ in a_t] for _ in range(8)]

    def set_grads(ts, k):
        for (p, _), gr in zip(ts, grads[k]):
            p.grad = gr.clone()

    for k in range(2):                      # eager steps on both (creates the state)
        set_grads(a_t, k)
        set_grads(b_t, k)
        A.step()
        B.step()
    # A: state → torch.optim.Adam (foreach) for two steps → back to ptyrad_amd.optim.Adam
    T = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in a_t], foreach=False)
    T.load_state_dict(A.state_dict())
    for k in (2, 3):
        set_grads(a_t, k)
        T.step()
    A2 = optim.Adam([{"params": [p], "lr": lr} for p, lr in a_t])
    A2.load_state_dict(T.state_dict())
    for k in (4, 5):
        set_grads(a_t, k)
        A2.step()
    # B: steps 2..5 with steps 4, 5 replayed from one captured graph
    for k in (2, 3):
        set_grads(b_t, k)
        B.step()
    static = [torch.zeros_like(p) for p, _ in b_t]
    for (p, _), s in zip(b_t, static):
        p.grad = s
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        B.step()
    for k in (4, 5):
        for s, gr in zip(static, grads[k]):
            s.copy_(gr)
        graph.replay()
    torch.cuda.synchronize()
    for (pa, _), (pb, _) in zip(a_t, b_t):
        np.testing.assert_allclose(pa.detach().cpu().numpy(), pb.detach().cpu().numpy(), rtol=2e-6, atol=1e-9)
    assert float(A2.state[a_t[0][0]]["step"].cpu()) == float(B.state[b_t[0][0]]["step"].cpu()) == 6.0
