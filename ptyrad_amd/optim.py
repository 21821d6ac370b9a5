"""torch.optim.Adam / AdamW whose update runs as one grid-filling HIP launch (ptyx_adam_step).

``create_optimizer`` (reconstruction.py:285-368 of the reference) builds ``torch.optim.Adam`` with
one parameter group per optimisable tensor.  torch's fused Adam then launches one
multi_tensor_apply kernel per group with one workgroup per 65,536-element chunk — 17 workgroups
for a 1033² object — so at the reference's default cadence (one optimizer step per 32-pattern
mini-batch) the update is latency-bound and costs more GPU time than the engine call
(ptyrad_amd/csrc/ptyx_optim.hip).  These classes ARE torch.optim.Adam / AdamW (same constructor,
param_groups, state layout — 'step', 'exp_avg', 'exp_avg_sq' — and state_dict, so checkpoints
move between them and torch's own classes); only ``step()`` differs: the step counts advance in
one ``torch._foreach_add_`` and every group's update runs in one ``ptyx_adam_step`` launch, in
torch's single-tensor arithmetic (fp32, same operation order; bias corrections in fp64).

Cases the kernel does not cover (amsgrad, complex or non-fp32 or sparse gradients, CPU tensors,
tensor-valued lr / betas, differentiable) run torch's own ``step()``.  Both step paths are
graph-capturable once the state exists (ptyrad_amd/stepgraph.py).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _eligible(group, params):
    if group.get("amsgrad") or group.get("differentiable") or group.get("foreach") or group.get("fused"):
        return False
    if any(isinstance(group[k], torch.Tensor) for k in ("lr", "eps", "weight_decay")) or \
            any(isinstance(b, torch.Tensor) for b in group["betas"]):
        return False
    return all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and
               (p.grad is None or (not p.grad.is_sparse and p.grad.dtype == torch.float32 and p.grad.is_contiguous()))
               for p in params)


class _HipAdamMixin:
    _decoupled = False
    # set by a graph-replayed recon_step around step(): its ptyx_step_select launch has already
    # advanced the step counts _step_tensors() returned (ptyrad_amd/stepgraph.py)
    _external_step_inc = False
    # set likewise: (terms, nb, rstart, cnt, terms_all) pointers of the step's ptyx_step_store, done
    # by the first Adam launch instead (ptyx_adam_step_store); _step_store_done tells the caller
    _step_store = None
    _step_store_done = False

    def _step_tensors(self):
        """The step counts the next step() advances (one per eligible parameter with a gradient),
        or [] while any of them does not exist yet (step() creates the state and increments)."""
        out = []
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params or not _eligible(group, params):
                continue
            for p in params:
                st = self.state.get(p)
                if not st or "step" not in st or st["step"].device != p.device:
                    return []
                out.append(st["step"])
        return out

    def _hip_batches(self, create=True):
        """(batches, plain): the eligible groups' (param, state, lr) by Adam hyperparameter key, and
        the groups torch's own step() takes.  ``create``: make missing state as step() does; else
        None while any eligible parameter has no state yet."""
        plain = []
        batches = {}
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if not _eligible(group, params):
                plain.append(group)
                continue
            decoupled = bool(group.get("decoupled_weight_decay", self._decoupled))
            key = (float(group["betas"][0]), float(group["betas"][1]), float(group["eps"]),
                   float(group["weight_decay"]), decoupled, bool(group.get("maximize", False)), params[0].device)
            b = batches.setdefault(key, [])
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    if not create:
                        return None
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif st["step"].device != p.device:   # a state loaded from a non-capturable torch Adam
                    if not create:
                        return None
                    st["step"] = st["step"].to(p.device, torch.float32)
                b.append((p, st, float(group["lr"])))
        return batches, plain

    @staticmethod
    def _launch_args(key, items):
        """ptyx_adam_step's arguments after the stream: (n, params, grads, exp_avgs, exp_avg_sqs,
        steps, numels, lrs, beta1, beta2, eps, weight_decay, flags)."""
        b1, b2, eps, wd, decoupled, maximize, _ = key
        n = len(items)
        P = (ctypes.c_void_p * n)(*[p.data_ptr() for p, _, _ in items])
        G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p, _, _ in items])
        M = (ctypes.c_void_p * n)(*[st["exp_avg"].data_ptr() for _, st, _ in items])
        V = (ctypes.c_void_p * n)(*[st["exp_avg_sq"].data_ptr() for _, st, _ in items])
        S = (ctypes.c_void_p * n)(*[st["step"].data_ptr() for _, st, _ in items])
        NE = (ctypes.c_int64 * n)(*[p.numel() for p, _, _ in items])
        LR = (ctypes.c_double * n)(*[lr for _, _, lr in items])
        flags = (1 if decoupled else 0) | (2 if maximize else 0)
        return (n, P, G, M, V, S, NE, LR, b1, b2, eps, wd, flags)

    def fused_step_args(self):
        """ptyx_plan_set_adam's arguments (after the plan) when ONE HIP launch is the whole step:
        every group eligible, one hyperparameter batch, every state created — what a graph-replayed
        recon_step folds into its engine call (PTYX_PREP_FUSED_ADAM, ptyrad_amd/stepgraph.py) —
        else None.  The step counts are the caller's to advance (ptyx_step_select)."""
        got = self._hip_batches(create=False)
        if got is None:
            return None
        batches, plain = got
        if plain or len(batches) != 1:
            return None
        key, items = next(iter(batches.items()))
        return self._launch_args(key, items)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches, plain = self._hip_batches()
        for key, items in batches.items():
            if not self._external_step_inc:
                torch._foreach_add_([st["step"] for _, st, _ in items], 1)
            args = self._launch_args(key, items)
            stream = ctypes.c_void_p(torch.cuda.current_stream(key[-1]).cuda_stream)
            if self._step_store is not None and not self._step_store_done:
                _lib.check(_lib.load().ptyx_adam_step_store(stream, *args, *self._step_store))
                self._step_store_done = True
            else:
                _lib.check(_lib.load().ptyx_adam_step(stream, *args))
        if plain:
            saved = self.param_groups
            try:
                self.param_groups = plain
                super().step()
            finally:
                self.param_groups = saved
        return loss


class Adam(_HipAdamMixin, torch.optim.Adam):
    """torch.optim.Adam with a one-launch HIP update (see the module docstring)."""


class AdamW(_HipAdamMixin, torch.optim.AdamW):
    """torch.optim.AdamW with a one-launch HIP update (decoupled weight decay)."""
    _decoupled = True
