"""Graph-replayed optimizer steps for recon_step (HIP graphs instead of a tracing compiler).

At the reference's default cadence (grad_accumulation = 1, params/recon_params.py:17) an iteration
of recon_step (reconstruction.py:658-781) is one optimizer step per 32-pattern mini-batch: 2,048
steps per iteration at the c2 geometry.  Each step is ~18 small engine launches plus the fused
Adam kernels, and issuing them from Python costs more than the GPU needs to run them
(0.47 ms per step, 0.18 ms of it GPU time).  ``StepGraphs`` captures ONE optimizer
step — ptyx_step_select (the step's indices by a device counter, and the flat gradient buffer
zeroed), the ptyx_forward_loss_grad call, ``optimizer.step()``, ptyx_step_store (the loss terms,
then the counter advances) — into a hipGraph
(torch.cuda.CUDAGraph is hipGraph on ROCm) and replays it for every later step with the same
shape.  The step's inputs are selected on the device from a per-iteration index table by a
step counter that the graph itself advances, so a replay needs no host work besides the launch.

Same kernels, same order, same arguments as the eager step: the trajectory is bitwise identical
(tests/test_gpu_stepgraph.py).  The first step of every new shape runs eagerly through the same
body (it creates the optimizer state a capture must not allocate), the next is captured.

Eligible: one rank (no collectives inside the step), the plain fused engine path (no autograd
stages, no loss_pacbed, no optimised propagator), ``ptyrad_amd.optim.Adam`` / ``AdamW``
(``create_optimizer``'s default) or torch's Adam / AdamW with ``fused=True``, and every step small
enough for one engine call.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .engine import LossConfig, _ptr, batch_offsets


def ineligible_reason(model, optimizer, loss_fn, ctx, batches, grad_accumulation):
    """None when recon_step's steps can be graph-replayed, else why not (a short string)."""
    if not torch.cuda.is_available() or model.opt_obja.device.type != "cuda":
        return "no HIP device"
    if ctx is not None and (ctx._collective() or ctx.band_exchange):
        return "collectives inside the step"
    if not (hasattr(loss_fn, "_special") and hasattr(loss_fn, "supports_batch_split")):
        return "loss_fn is not ptyrad_amd.losses.CombinedLoss"
    if loss_fn._special(model) or loss_fn.loss_params.get("loss_pacbed", {}).get("state", False):
        return "autograd stages or loss_pacbed"
    if getattr(model, "prop_opt", False) or model._dz_t() is not None:
        return "optimised propagator (autograd through H)"
    from .optim import _HipAdamMixin, _eligible
    hip_adam = isinstance(optimizer, _HipAdamMixin) and all(
        _eligible(g, [p for p in g["params"] if p.grad is not None or p.requires_grad]) for g in optimizer.param_groups)
    if not hip_adam and (not isinstance(optimizer, (torch.optim.Adam, torch.optim.AdamW)) or
                         not all(g.get("fused") for g in optimizer.param_groups)):
        return "optimizer is not ptyrad_amd.optim.Adam / AdamW or a fused torch Adam / AdamW"
    cap = model.plan.register_capacity
    cap = min(cap, int(model.plan.dims.max_patterns)) if cap > 0 else int(model.plan.dims.max_patterns)
    ga = max(1, int(grad_accumulation))
    for g0 in range(0, len(batches), ga):
        if sum(len(np.asarray(b).reshape(-1)) for b in batches[g0:g0 + ga]) > cap:
            return "a step larger than one engine call"
    return None


class StepGraphs:
    """Captured optimizer steps of one (model, optimizer, loss_fn), keyed by step shape."""

    MAX_GRAPHS = 16               # captured steps kept (insertion order; the oldest is dropped)

    def __init__(self):
        self.graphs = {}          # key -> CUDAGraph
        self.static = {}          # key -> (idx (n,) i32, off (nb+1,) i32 device, terms (nb, 5))
        self.pool = None
        self._table = None        # (batches fingerprint, idx_all, istart, rstart)
        self._seen = set()        # keys whose first (eager) step has run
        self._cnt = None          # (1,) i64: the step the next replay runs
        self._terms = None        # (n_batches, 5) loss terms of the iteration
        self.captures = 0
        self.replays = 0
        self.eager = 0

    # ---------------------------------------------------------------- per-iteration tables
    def _tables(self, batches, ga, dev):
        sizes = [len(np.asarray(b).reshape(-1)) for b in batches]
        flat = np.concatenate([np.asarray(b).reshape(-1) for b in batches]).astype(np.int32)
        fp = (ga, tuple(sizes), hash(flat.tobytes()))
        if self._table is None or self._table[0] != fp:
            off = np.concatenate([[0], np.cumsum(sizes)])
            istart = off[0:len(batches):ga].astype(np.int64)                 # first pattern of each step
            rstart = np.arange(0, len(batches), ga, dtype=np.int64)          # first mini-batch of each step
            self._table = (fp, torch.as_tensor(flat).to(dev), torch.as_tensor(istart).to(dev),
                           torch.as_tensor(rstart).to(dev))
        return self._table[1:]

    # ---------------------------------------------------------------- one step
    def _body(self, model, optimizer, loss_fn, flat_grad, grads, key, grad_scale, cnt, idx_all, istart, rstart,
              terms_all):
        """Exactly recon_step's step, on static buffers: captured or run eagerly."""
        sidx, soff, sterms = self.static[key]
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream(flat_grad.device).cuda_stream)
        # the step's indices (device counter) + zeroed gradient buffer, one launch
        _lib.check(lib.ptyx_step_select(st, _ptr(idx_all), _ptr(istart), _ptr(cnt), int(sidx.numel()), _ptr(sidx),
                                        _ptr(flat_grad), int(flat_grad.numel())))
        t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
             "shifts": model.opt_probe_pos_shifts.detach(), "H": model._H_rv().detach(),
             "tilts": None if model._tilts() is None else model._tilts().detach().contiguous()}
        t.update(model._base())
        cfg = LossConfig.from_loss_params(loss_fn.loss_params)
        model.plan.forward_loss_grad(t, sidx, soff, cfg, grads, grad_scale=grad_scale, loss_terms=sterms,
                                     max_batch=max(key[0]), _rows_checked=True)
        optimizer.step()
        # the loss terms into the iteration's table, then the counter advances (one launch)
        _lib.check(lib.ptyx_step_store(st, _ptr(sterms), int(sterms.shape[0]), _ptr(rstart), _ptr(cnt),
                                       _ptr(terms_all)))

    def run(self, model, optimizer, loss_fn, batches, ga, live, flat_grad):
        """All optimizer steps of one recon_step iteration; returns the (n_batches, 5) loss terms.
        ``live``: the parameters whose ``.grad`` are views of ``flat_grad`` (DistContext.grad_views)."""
        dev = model.opt_obja.device
        ga = max(1, int(ga))
        idx_all, istart, rstart = self._tables(batches, ga, dev)
        # every position must be held (checked once per iteration on the host, as fused_into does)
        flat_np = np.concatenate([np.asarray(b).reshape(-1) for b in batches])
        model._check_indices(flat_np)
        loss_fn._check_held(model, flat_np)
        # persistent step counter and loss-term table (the graphs hold their addresses)
        if self._cnt is None or self._cnt.device != dev:
            self._cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        if self._terms is None or self._terms.shape[0] != len(batches) or self._terms.device != dev:
            self._terms = torch.zeros((len(batches), 5), dtype=torch.float32, device=dev)
        cnt, terms_all = self._cnt, self._terms
        cnt.zero_()
        grads = {}
        for k, p in (("obja", model.opt_obja), ("objp", model.opt_objp), ("probe", model.opt_probe),
                     ("tilts", model._tilts())):
            if p is not None and any(p is q for q in live):
                grads[k] = p.grad
        if model.shift_probes and any(model.opt_probe_pos_shifts is q for q in live):
            grads["shifts"] = model.opt_probe_pos_shifts.grad
        base = model._base()
        # the graph bakes in every pointer the step reads or writes (H is a fixed buffer here)
        ptrs = tuple(int(v.data_ptr()) for v in (model.opt_obja, model.opt_objp, model.opt_probe,
                                                  model.opt_probe_pos_shifts, flat_grad, cnt,
                                                  idx_all, istart, rstart, terms_all)) + \
            tuple(int(v.data_ptr()) for v in base.values() if isinstance(v, torch.Tensor))
        lrs = tuple(float(g["lr"]) for g in optimizer.param_groups)
        live_ids = tuple(id(p) for p in live)
        saved = [g.get("capturable", False) for g in optimizer.param_groups]
        for g in optimizer.param_groups:
            g["capturable"] = True            # fused Adam keeps its step counts on the device already
        def state_ptrs():   # the optimizer state a captured step reads and writes (replaced by a load)
            return tuple(int(v.data_ptr()) for p in live for v in optimizer.state.get(p, {}).values()
                         if isinstance(v, torch.Tensor))

        try:
            for g0 in range(0, len(batches), ga):
                sizes = tuple(len(np.asarray(b).reshape(-1)) for b in batches[g0:g0 + ga])
                key = (sizes, live_ids, lrs, ptrs, id(optimizer), state_ptrs())
                if key not in self.static:
                    n, nb = sum(sizes), len(sizes)
                    self.static[key] = (torch.zeros(n, dtype=torch.int32, device=dev),
                                        torch.as_tensor(batch_offsets([np.zeros(s) for s in sizes])).to(dev),
                                        torch.zeros((nb, 5), dtype=torch.float32, device=dev))
                args = (model, optimizer, loss_fn, flat_grad, grads, key, 1.0 / ga, cnt, idx_all, istart, rstart,
                        terms_all)
                gr = self.graphs.get(key)
                if gr is not None:
                    gr.replay()
                    self.replays += 1
                elif key in self._seen:
                    # second step of this shape: capture it (the optimizer state exists by now)
                    gr = torch.cuda.CUDAGraph()
                    if self.pool is None:
                        self.pool = torch.cuda.graph_pool_handle()
                    torch.cuda.synchronize(dev)
                    with torch.cuda.graph(gr, pool=self.pool):
                        self._body(*args)
                    self.graphs[key] = gr
                    self.captures += 1
                    while len(self.graphs) > self.MAX_GRAPHS:   # oldest first (e.g. a learning-rate schedule)
                        old = next(iter(self.graphs))
                        del self.graphs[old]
                        self.static.pop(old, None)
                        self._seen.discard(old)
                    gr.replay()
                    self.replays += 1
                else:
                    self._body(*args)
                    self.eager += 1
                    self._seen.add(key)
        finally:
            for g, c in zip(optimizer.param_groups, saved):
                g["capturable"] = c
        return terms_all.clone()
