"""Reconstruction loop on the HIP engine: PtyRAD's recon_step contract + RCCL data parallelism.

Mirrors ``src/ptyrad/reconstruction.py``:
  select_scan_indices :441-477, make_batches :479-587 ('random' and 'compact'),
  recon_step :658-781 (Adam / SGD branch), toggle_grad_requires :783-790, loss_logger :808-832.

Hot loop: every optimizer step's group of ``grad_accumulation`` mini-batches is ONE
``CombinedLoss.fused`` engine call (each batch keeps its own NRMSE normalisation; the summed
gradient / grad_accumulation equals the reference's accumulated ``.grad``).

Multi-GPU (replaces the accelerate/DDP wrapper, utils/common.py:58-90): ``DistContext``.  The
mini-batches of a group are dealt round-robin to ranks, each rank runs its share, then ONE
all-reduce(sum) over a flat buffer of every gradient gives all ranks the exact single-device
accumulated gradient (up to fp32 summation order); every rank then takes the same optimizer
step, so replicas stay identical.  No per-forward buffer broadcast, no loss averaging.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from .engine import LOSS_TERM_NAMES


# ------------------------------------------------------------------ indices and batches
def select_scan_indices(N_scan_slow, N_scan_fast, subscan_slow=None, subscan_fast=None, mode="full",
                        verbose=True):
    n = int(N_scan_slow) * int(N_scan_fast)
    if mode == "full":
        return np.arange(n)
    if subscan_slow is None and subscan_fast is None:
        subscan_slow, subscan_fast = N_scan_slow // 2, N_scan_fast // 2
    grid = np.arange(n).reshape(N_scan_slow, N_scan_fast)
    if mode == "center":
        r0 = (N_scan_slow - subscan_slow) // 2
        c0 = (N_scan_fast - subscan_fast) // 2
        return grid[r0:r0 + subscan_slow, c0:c0 + subscan_fast].reshape(-1)
    if mode == "sub":
        rs = np.linspace(0, N_scan_slow - 1, num=subscan_slow, dtype=int)
        cs = np.linspace(0, N_scan_fast - 1, num=subscan_fast, dtype=int)
        return grid[np.ix_(rs, cs)].reshape(-1)
    raise ValueError(f"Indices selection mode {mode} not implemented, use 'full', 'center' or 'sub'")


def make_batches(indices, pos, batch_size, mode="random", verbose=True, rng=None):
    """Mini-batches of ~batch_size indices (reference :479-587).  'random' = shuffled array_split."""
    indices = np.asarray(indices)
    num_batch = max(1, len(indices) // batch_size)
    if mode == "random":
        rng = rng if rng is not None else np.random.default_rng()
        return np.array_split(rng.permutation(indices), num_batch)
    if mode == "compact":
        from sklearn.cluster import MiniBatchKMeans
        km = MiniBatchKMeans(init="k-means++", n_init=10, n_clusters=num_batch, max_iter=10, batch_size=3072)
        km.fit(np.asarray(pos)[indices])
        return [indices[km.labels_ == b] for b in range(num_batch) if np.any(km.labels_ == b)]
    raise NotImplementedError(f"GROUP_MODE '{mode}' is not implemented on this path (use 'random' or 'compact')")


def toggle_grad_requires(model, niter, verbose=False):
    for name, start in model.start_iter.items():
        model.optimizable_tensors[name].requires_grad = start is not None and niter >= start


def time_sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    return time.perf_counter()


def loss_logger(batch_losses, niter, iter_t, verbose=True):
    avg = {k: float(np.mean(v)) if len(v) else 0.0 for k, v in batch_losses.items()}
    total = sum(avg.values())
    if verbose:
        s = ", ".join(f"{k}: {v:.4f}" for k, v in avg.items())
        print(f"Iter: {niter}, Total Loss: {total:.4f}, {s}, in {iter_t:.3f} sec", flush=True)
    return total


# ------------------------------------------------------------------ data parallel context
class DistContext:
    """Rank/world of a torch.distributed job (backend 'nccl' = RCCL on ROCm, or 'gloo' on CPU)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def my_batches(self, group_batches):
        """Round-robin deal of a group's mini-batches to ranks (positions of batch b on rank b % world)."""
        return [i for i in range(len(group_batches)) if i % self.world == self.rank]

    def allreduce_grads(self, params):
        """ONE all-reduce(sum) over a flat buffer of all gradients (zeros where a rank had none)."""
        if self.world == 1:
            return
        grads = []
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, group=self.group)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def gather_terms(self, terms_local, idx_local, n_total, device):
        """All ranks get the (n_total, 5) loss terms of the group (rows filled by their owners)."""
        buf = torch.zeros((n_total, 5), dtype=torch.float32, device=device)
        if len(idx_local):
            buf[torch.as_tensor(idx_local, device=device)] = terms_local.to(device)
        if self.world > 1:
            dist.all_reduce(buf, group=self.group)
        return buf


# ------------------------------------------------------------------ the reference step
def recon_step(batches, grad_accumulation, model, optimizer, loss_fn, constraint_fn, niter, verbose=True,
               acc=None, dist_ctx=None):
    """One iteration over ``batches`` (reconstruction.py:658-781, non-LBFGS branch).

    Optimizer steps happen every ``grad_accumulation`` batches and after the last one; each step's
    group of batches runs as one fused engine call (sharded over ranks when ``dist_ctx`` is given).
    """
    if acc is not None:
        raise NotImplementedError("accelerate is replaced by DistContext (RCCL) on this path")
    if isinstance(optimizer, torch.optim.LBFGS):
        raise NotImplementedError("LBFGS closure branch is outside the hot path")
    ctx = dist_ctx or DistContext()
    batch_losses = {name: [] for name in loss_fn.loss_params.keys()}
    t0 = time_sync()
    toggle_grad_requires(model, niter, verbose)
    params = [p for g in optimizer.param_groups for p in g["params"]]
    optimizer.zero_grad()
    ga = max(1, int(grad_accumulation))
    dev = model.opt_obja.device
    for g0 in range(0, len(batches), ga):
        group = batches[g0:g0 + ga]
        mine = ctx.my_batches(group)
        if mine:
            total, terms = loss_fn.fused(model, [group[i] for i in mine])
            (total / ga).backward()
        else:
            terms = torch.zeros((0, 5), device=dev)
        ctx.allreduce_grads(params)
        optimizer.step()
        optimizer.zero_grad()
        all_terms = ctx.gather_terms(terms, mine, len(group), dev).cpu().numpy()   # one sync per step
        for row in all_terms:
            for name, v in zip(LOSS_TERM_NAMES, row):
                if name in batch_losses:
                    batch_losses[name].append(v)
        model.clear_cache()
    if constraint_fn is not None:
        constraint_fn(model, niter)
    iter_t = time_sync() - t0
    model.loss_iters.append((niter, loss_logger(batch_losses, niter, iter_t, verbose=verbose)))
    model.iter_times.append(iter_t)
    model.dz_iters.append((niter, model.opt_slice_thickness.detach().cpu().numpy()))
    model.avg_tilt_iters.append((niter, model.opt_obj_tilts.detach().mean(0).cpu().numpy()))
    return batch_losses


def recon_loop(model, optimizer, loss_fn, constraint_fn, batches, NITER, grad_accumulation=1, verbose=True,
               dist_ctx=None):
    """Minimal recon_loop (reconstruction.py:589-656) without saving/plotting."""
    for niter in range(1, NITER + 1):
        recon_step(batches, grad_accumulation, model, optimizer, loss_fn, constraint_fn, niter, verbose=verbose,
                   dist_ctx=dist_ctx)
    return model.loss_iters


def create_optimizer(optimizer_params, optimizable_params, verbose=True):
    """torch.optim.<name>(param groups with per-tensor lr, **configs) (reconstruction.py:285-368)."""
    name = optimizer_params.get("name", "Adam")
    cls = getattr(torch.optim, name, None)
    if cls is None:
        raise ValueError(f"Optimizer '{name}' is not supported.")
    return cls(optimizable_params, **(optimizer_params.get("configs") or {}))
