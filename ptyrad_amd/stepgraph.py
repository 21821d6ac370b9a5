"""Graph-replayed optimizer steps for recon_step (HIP graphs instead of a tracing compiler).

At the reference's default cadence (grad_accumulation = 1, params/recon_params.py:17) an iteration
of recon_step (reconstruction.py:658-781) is one optimizer step per 32-pattern mini-batch: 2,048
steps per iteration at the c2 geometry.  Each step is ~18 small engine launches plus the fused
Adam kernels, and issuing them from Python costs more than the GPU needs to run them
(0.47 ms per step, 0.18 ms of it GPU time).  ``StepGraphs`` captures ONE optimizer
step — ptyx_step_select (the step's indices by a device counter, the flat gradient buffer zeroed,
and the HIP Adam's step counts advanced), the ptyx_forward_loss_grad call, ``optimizer.step()``, ptyx_step_store (the loss terms,
then the counter advances; done by the HIP Adam's first launch when it runs one) — into a hipGraph
(torch.cuda.CUDAGraph is hipGraph on ROCm) and replays it for every later step with the same
shape.  The step's inputs are selected on the device from a per-iteration index table by a
step counter that the graph itself advances, so a replay needs no host work besides the launch.

Same kernels, same order, same arguments as the eager step: the trajectory is bitwise identical
(tests/test_gpu_stepgraph.py).  With one rank and one HIP Adam batch the optimizer step rides in
the engine call (PTYX_PREP_FUSED_ADAM, ABI 209: the k_fused3 engine's small calls fold the object
gather, the probe gradient's rows and the update into one launch), bitwise the separate launch.  The first step of every new shape runs eagerly through the same
body (it creates the optimizer state a capture must not allocate), the next is captured.

Eligible: the plain fused engine path (no autograd stages, no loss_pacbed, no optimised
propagator), ``ptyrad_amd.optim.Adam`` / ``AdamW`` (``create_optimizer``'s default) or torch's
Adam / AdamW with ``fused=True``, and every step small enough for one engine call.  With several
ranks (or ``always_reduce``) the step's RCCL collectives are captured too: the all-reduce of a
split step's per-mini-batch loss sums (between ptyx_forward_loss_grad_begin and _end) and the
gradient all-reduce, which also carries the step's loss terms — one or two collectives a step,
replayed with the kernels.  Needs the 'nccl' (RCCL) backend, no band exchange, and every rank
holding a part of every mini-batch of a split step.
"""
from __future__ import annotations

import ctypes
from dataclasses import astuple

import numpy as np
import torch

from . import _lib
from .engine import LossConfig, _ptr, batch_offsets


def ineligible_reason(model, optimizer, loss_fn, ctx, batches, grad_accumulation):
    """None when recon_step's steps can be graph-replayed, else why not (a short string).  The
    answer depends only on the job's shapes and settings, never on the rank, so every rank takes
    the same path."""
    if not torch.cuda.is_available() or model.opt_obja.device.type != "cuda":
        return "no HIP device"
    if ctx is not None and (ctx.band_exchange is True or ctx.bands is not None):
        return "band exchange (point-to-point collectives per step)"
    if not (hasattr(loss_fn, "_special") and hasattr(loss_fn, "supports_batch_split")):
        return "loss_fn is not ptyrad_amd.losses.CombinedLoss"
    ga = max(1, int(grad_accumulation))
    coll = ctx is not None and ctx._collective()
    if coll:
        import torch.distributed as dist
        if dist.get_backend(ctx.group) != "nccl":
            return "collectives on a backend graphs cannot capture (RCCL 'nccl' only)"
        split_ok = loss_fn.supports_batch_split(model)
        for g0 in range(0, len(batches), ga):
            group = batches[g0:g0 + ga]
            if ctx.splits(group):
                if not split_ok:
                    return "a split step with a loss that cannot be split"
                if min(len(np.asarray(b).reshape(-1)) for b in group) < ctx.world:
                    return "a mini-batch with fewer positions than ranks (empty parts)"
            elif len(group) < ctx.world:
                return "a step that leaves ranks without a mini-batch"
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
    cap = model.plan.call_capacity
    for g0 in range(0, len(batches), ga):
        group = batches[g0:g0 + ga]
        sizes = [len(np.asarray(b).reshape(-1)) for b in group]
        if coll and ctx.splits(group):
            load = sum(-(-n // ctx.world) for n in sizes)                     # rank 0's parts (the largest)
        elif coll:
            load = max(sum(sizes[r::ctx.world]) for r in range(ctx.world))   # whole batches round-robin
        else:
            load = sum(sizes)
        if load > cap:
            return "a step larger than one engine call"
    return None


def _local_steps(ctx, batches, ga):
    """Per optimizer step of the iteration: (this rank's mini-batch pieces, the group size, whether
    the group is split, the group rows this rank's terms fill, the slot-exchange rows per rank of a
    split group).  One rank: the whole groups."""
    out = []
    for g0 in range(0, len(batches), ga):
        group = batches[g0:g0 + ga]
        if ctx is None or not ctx._collective():
            out.append(([np.asarray(b).reshape(-1) for b in group], len(group), False, tuple(range(len(group))), 0))
        elif ctx.splits(group):
            out.append(([ctx.my_part(b) for b in group], len(group), True,
                        tuple(range(len(group))) if ctx.rank == 0 else (), ctx.slot_cap(group)))
        else:
            mine = ctx.my_batches(group)
            out.append(([np.asarray(group[i]).reshape(-1) for i in mine], len(group), False, tuple(mine), 0))
    return out


class StepGraphs:
    """Captured optimizer steps of one (model, optimizer, loss_fn), keyed by step shape."""

    MAX_GRAPHS = 16               # captured steps kept (insertion order; the oldest is dropped)
    STORE = True                  # whole-batch steps' calls overwrite the object gradient (A/B switch)
    FUSE_ADAM = True              # one-rank steps fold the optimizer step into the engine call (A/B switch)
    SELECT = True                 # whole-batch steps' calls pick their own indices (PTYX_PREP_SELECT; A/B switch)
    CHUNK = 16                    # consecutive steps of one shape replayed as one graph (1: one step a graph)

    def __init__(self):
        self.graphs = {}          # key -> CUDAGraph
        self.static = {}          # key -> (idx (n,) i32, off (nb+1,) i32 device, terms (nb, 5))
        self.pool = None
        self._table = None        # persistent device buffers (idx_all, istart, rstart)
        self._host = None         # the host tables last copied into them
        self._seen = set()        # keys whose first (eager) step has run
        self._sptr = {}           # key -> (step-count pointers, their device array) for ptyx_step_select
        self._cnt = None          # (1,) i64: the step the next replay runs
        self._terms = None        # (n_batches, 5) loss terms of the iteration
        self.captures = 0
        self.replays = 0
        self.eager = 0
        self._store_from = 0      # floats at the flat buffer's head a whole-batch step's call overwrites

    # ---------------------------------------------------------------- per-iteration tables
    def _tables(self, steps, ga, dev):
        """The iteration's index table (every step's positions on this rank, back to back) and the
        first pattern / mini-batch of each step, in PERSISTENT device buffers: a new batching (the
        reference's hypertune loop reshuffles every iteration, reconstruction.py:1059) is copied
        into them, so the captured graphs' pointers stay valid and no step is recaptured.  The
        buffers grow (and the graphs are dropped) only when a table outgrows them."""
        pieces = [p for st in steps for p in st[0]]
        flat = (np.concatenate(pieces) if pieces else np.zeros(0)).astype(np.int32)
        n_step = np.array([sum(len(p) for p in st[0]) for st in steps], np.int64)
        istart = np.concatenate([[0], np.cumsum(n_step)[:-1]]).astype(np.int64)   # first pattern of each step
        rstart = np.arange(0, len(steps) * ga, ga, dtype=np.int64)                 # first mini-batch of each step
        host = (flat, istart, rstart)
        bufs = self._table
        if bufs is None or bufs[0].device != dev or any(b.numel() < h.size for b, h in zip(bufs, host)):
            bufs = tuple(torch.zeros(max(h.size, 1), dtype=torch.int32 if h.dtype == np.int32 else torch.int64,
                                     device=dev) for h in host)
            self._table = bufs
            self._host = None
            self._drop_graphs()   # (their pointers were the old buffers')
        if self._host is None or not all(h0.shape == h.shape and np.array_equal(h0, h)
                                         for h0, h in zip(self._host, host)):
            for b, h in zip(bufs, host):
                b[:h.size].copy_(torch.from_numpy(h), non_blocking=False)
            self._host = tuple(h.copy() for h in host)
        return bufs

    def _evict(self, gkey):
        """Drop one captured graph; a single step's also takes its chunk graphs (they replay its
        static buffers) and its static state."""
        self.graphs.pop(gkey, None)
        if gkey and gkey[0] == "chunk":
            return
        for k in [k for k in self.graphs if k and k[0] == "chunk" and k[2] == gkey]:
            del self.graphs[k]
        self.static.pop(gkey, None)
        self._sptr.pop(gkey, None)
        self._seen.discard(gkey)

    def _drop_graphs(self):
        self.graphs.clear()
        self.static.clear()
        self._seen.clear()
        self._sptr.clear()

    def _step_ptrs(self, key, step_ts, dev):
        """Device array of the step-count pointers ptyx_step_select advances (kept per step shape:
        a captured graph holds its address; the key already holds the state's pointers)."""
        want = [int(t.data_ptr()) for t in step_ts]
        cur = self._sptr.get(key)
        if cur is None or cur[0] != want:
            cur = (want, torch.tensor(want, dtype=torch.int64, device=dev))
            self._sptr[key] = cur
        return cur[1]

    # ---------------------------------------------------------------- one step
    def _body(self, model, optimizer, loss_fn, flat_grad, grads, key, grad_scale, cnt, idx_all, istart, rstart,
              terms_all, ctx, extra, G, split, scap=0, ar_skip=0):
        """Exactly recon_step's step, on static buffers: captured or run eagerly.  With collectives
        (RCCL, captured into the graph like the kernels): a split step all-reduces the engine's
        per-mini-batch loss sums between its halves, and the gradient all-reduce carries the
        step's loss terms in the flat buffer's tail."""
        sidx, soff, sterms, mine_t = self.static[key]
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream(flat_grad.device).cuda_stream)
        # the HIP Adam's step counts advance in the same launch (its own increment launch skipped)
        step_ts = optimizer._step_tensors() if hasattr(optimizer, "_step_tensors") else []
        sp = self._step_ptrs(key, step_ts, flat_grad.device) if 0 < len(step_ts) <= 256 else None
        # the step's indices (device counter) + zeroed gradient buffer (and terms tail), one launch;
        # a whole-batch step's engine call overwrites the object gradient at the buffer's head
        # (PTYX_PREP_GRAD_STORE): only the rest is zeroed.  A whole-batch step's call does the
        # selection itself (PTYX_PREP_SELECT: inside the small call's preparation launch).
        z0 = 0 if split else self._store_from
        zbuf = flat_grad[z0:]
        sel = (_ptr(idx_all), _ptr(istart), _ptr(cnt), _ptr(zbuf), int(zbuf.numel()),
               None if sp is None else _ptr(sp), 0 if sp is None else len(step_ts))
        fold = self.SELECT and not split
        done = [False]   # the step counts have advanced
        if not fold:
            _lib.check(lib.ptyx_step_select(st, sel[0], sel[1], sel[2], int(sidx.numel()), _ptr(sidx), *sel[3:]))
            done[0] = True
        try:
            self._body_rest(model, optimizer, loss_fn, flat_grad, grads, key, grad_scale, cnt, rstart, terms_all,
                            ctx, extra, G, split, sp, lib, st, scap, ar_skip, sel if fold else None, done)
        except BaseException:
            # an eager step that raised after its step counts advanced (an engine-call check, the
            # optimizer itself): take them back, so Adam's bias correction stays in step with the
            # updates it really made (a capture only records the launch; nothing ran)
            if sp is not None and done[0] and not torch.cuda.is_current_stream_capturing():
                with torch.no_grad():
                    for t_ in step_ts:
                        t_.sub_(1)
            raise

    def _body_rest(self, model, optimizer, loss_fn, flat_grad, grads, key, grad_scale, cnt, rstart, terms_all,
                   ctx, extra, G, split, sp, lib, st, scap=0, ar_skip=0, sel=None, done=None):
        sidx, soff, sterms, mine_t = self.static[key]
        t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
             "shifts": model.opt_probe_pos_shifts.detach(), "H": model._H_rv().detach(),
             "tilts": None if model._tilts() is None else model._tilts().detach().contiguous()}
        t.update(model._base())
        cfg = LossConfig.from_loss_params(loss_fn.loss_params)
        terms = sterms
        sx = None
        if split:
            from .reconstruction import SlotExchange
            # with the slot exchange and one HIP Adam launch for the step, the gather waits for the
            # probe / loss-term all-reduce below and takes the optimizer step in its launch
            fargs = optimizer.fused_step_args() if (self.FUSE_ADAM and scap and extra and sp is not None and
                                                    hasattr(optimizer, "fused_step_args")) else None
            sx = SlotExchange(ctx, scap, defer=fargs is not None) if scap else None
            model.plan.forward_loss_grad(t, sidx, soff, cfg, grads, grad_scale=grad_scale, loss_terms=sterms,
                                         batch_sums_reduce=ctx.allreduce_sums, slot_exchange=sx, _rows_checked=True)
        else:
            prep = _lib.PTYX_PREP_GRAD_STORE if self._store_from else 0
            if sel is not None:
                model.plan.set_select(*sel)
                prep |= _lib.PTYX_PREP_SELECT
            # one rank, the step counts already advanced, one HIP Adam launch for the whole step: the
            # call takes the optimizer step itself (PTYX_PREP_FUSED_ADAM; the k_fused3 engine's small
            # calls fold it into their last launch), the loss-term store included
            fargs = optimizer.fused_step_args() if (self.FUSE_ADAM and not extra and sp is not None and
                                                    hasattr(optimizer, "fused_step_args")) else None
            if fargs is not None:
                model.plan.set_adam(fargs, (_ptr(sterms), int(G), _ptr(rstart), _ptr(cnt), _ptr(terms_all)))
                prep |= _lib.PTYX_PREP_FUSED_ADAM
            model.plan.forward_loss_grad(t, sidx, soff, cfg, grads, grad_scale=grad_scale, loss_terms=sterms,
                                         max_batch=max(key[0]), _rows_checked=True, prep=prep)
            if sel is not None and done is not None:
                done[0] = True
            if fargs is not None:
                return
        if extra:
            terms = ctx.terms_tail(flat_grad, extra, G)
            if mine_t is not None:
                terms.index_copy_(0, mine_t, sterms)
            # (with the slot exchange the object / position gradients are already whole)
            ctx.allreduce(flat_grad[ar_skip:] if (split and scap) else flat_grad)
            if sx is not None and sx.defer:
                model.plan.set_adam(fargs, (_ptr(terms), int(G), _ptr(rstart), _ptr(cnt), _ptr(terms_all)))
                sx.finish(adam=True)
                return
        if sp is not None:
            optimizer._external_step_inc = True
        # the loss terms into the iteration's table, then the counter advances: inside the HIP
        # Adam's first launch when it runs one, else a launch of its own
        store = (_ptr(terms), int(G), _ptr(rstart), _ptr(cnt), _ptr(terms_all))
        fold = hasattr(optimizer, "_step_store")
        if fold:
            optimizer._step_store, optimizer._step_store_done = store, False
        try:
            optimizer.step()
            done = fold and optimizer._step_store_done
        finally:
            optimizer._external_step_inc = False
            if fold:
                optimizer._step_store, optimizer._step_store_done = None, False
        if not done:
            _lib.check(lib.ptyx_step_store(st, *store))

    def run(self, model, optimizer, loss_fn, batches, ga, live, flat_grad, ctx=None, extra=0, slots=False,
            ar_skip=0):
        """All optimizer steps of one recon_step iteration; returns the (n_batches, 5) loss terms.
        ``live``: the parameters whose ``.grad`` are views of ``flat_grad`` (DistContext.grad_views);
        ``extra``: the floats after them that carry a step's loss terms through the all-reduce;
        ``slots``: split steps exchange object-gradient slots (reconstruction.SlotExchange) and
        all-reduce only ``flat_grad[ar_skip:]``."""
        dev = model.opt_obja.device
        ga = max(1, int(ga))
        steps = _local_steps(ctx, batches, ga)
        idx_all, istart, rstart = self._tables(steps, ga, dev)
        # every position must be held (checked once per iteration on the host, as fused_into does)
        flat_np = np.concatenate([p for st in steps for p in st[0]] or [np.zeros(0, np.int64)])
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
        # the object gradients at the head of the flat buffer (live order): a whole-batch step's
        # call overwrites them, so its select launch zeroes only what follows
        self._store_from = 0
        for p in (live if self.STORE else ()):
            if p is model.opt_obja or p is model.opt_objp:
                self._store_from += p.numel()
            else:
                break
        if model.shift_probes and any(model.opt_probe_pos_shifts is q for q in live):
            grads["shifts"] = model.opt_probe_pos_shifts.grad
        base = model._base()
        # the graph bakes in every pointer the step reads or writes (H is a fixed buffer here)
        ptrs = tuple(int(v.data_ptr()) for v in (model.opt_obja, model.opt_objp, model.opt_probe,
                                                  model.opt_probe_pos_shifts, flat_grad, cnt,
                                                  idx_all, istart, rstart, terms_all)) + \
            tuple(int(v.data_ptr()) for v in base.values() if isinstance(v, torch.Tensor))
        # every value a capture bakes in besides pointers: the groups' hyperparameters (lr, betas,
        # eps, weight_decay, maximize, ...), the loss configuration and the engine-variant tuning
        def _hv(v):
            return tuple(_hv(x) for x in v) if isinstance(v, (tuple, list)) else \
                (float(v) if isinstance(v, (int, float, bool)) or torch.is_tensor(v) else repr(v))
        hyper = tuple(tuple(sorted((k, _hv(v)) for k, v in g.items() if k not in ("params", "capturable")))
                      for g in optimizer.param_groups)
        lcfg = astuple(LossConfig.from_loss_params(loss_fn.loss_params))
        tuning = tuple(_lib.get_tuning(k) for k in _lib.TUNING_KEYS)
        live_ids = tuple(id(p) for p in live)
        saved = [g.get("capturable", False) for g in optimizer.param_groups]
        for g in optimizer.param_groups:
            g["capturable"] = True            # fused Adam keeps its step counts on the device already
        def state_ptrs():   # the optimizer state a captured step reads and writes (replaced by a load)
            return tuple(int(v.data_ptr()) for p in live for v in optimizer.state.get(p, {}).values()
                         if isinstance(v, torch.Tensor))

        # consecutive steps of one shape: a run of CHUNK of them replays as ONE graph of CHUNK step
        # bodies (the device counter picks each body's mini-batch), so the replay boundary's idle
        # gap (≈ 8 µs at c2, more than a launch inside a graph) is paid once per CHUNK steps
        shapes = [(tuple(len(p) for p in st[0]),) + tuple(st[1:]) for st in steps]
        run_left = [0] * len(steps)
        for i in range(len(steps) - 1, -1, -1):
            run_left[i] = 1 + (run_left[i + 1] if i + 1 < len(steps) and shapes[i + 1] == shapes[i] else 0)
        K = max(1, int(self.CHUNK))
        try:
            i = 0
            while i < len(steps):
                pieces, G, split, mine, scap = steps[i]
                scap = scap if (split and slots) else 0
                sizes = tuple(len(p) for p in pieces)
                key = (sizes, G, split, mine, scap, live_ids, hyper, lcfg, tuning, ptrs, id(optimizer), state_ptrs(),
                       (self.STORE, self.FUSE_ADAM, self.SELECT))
                if key not in self.static:
                    n, nb = sum(sizes), len(sizes)
                    self.static[key] = (torch.zeros(n, dtype=torch.int32, device=dev),
                                        torch.as_tensor(batch_offsets([np.zeros(s) for s in sizes])).to(dev),
                                        torch.zeros((nb, 5), dtype=torch.float32, device=dev),
                                        torch.as_tensor(mine, dtype=torch.long).to(dev) if (extra and mine) else None)
                args = (model, optimizer, loss_fn, flat_grad, grads, key, 1.0 / ga, cnt, idx_all, istart, rstart,
                        terms_all, ctx, extra, G, split, scap, ar_skip)
                n_body = K if (K > 1 and key in self._seen and run_left[i] >= K) else 1
                gkey = key if n_body == 1 else ("chunk", n_body, key)
                gr = self.graphs.get(gkey)
                if gr is not None:
                    gr.replay()
                elif key in self._seen:
                    # second step of this shape (the optimizer state exists by now): capture it, or a
                    # chunk of n_body of them
                    gr = torch.cuda.CUDAGraph()
                    if self.pool is None:
                        self.pool = torch.cuda.graph_pool_handle()
                    sts = optimizer._step_tensors() if hasattr(optimizer, "_step_tensors") else []
                    if 0 < len(sts) <= 256:   # the step-count pointer array exists before the capture
                        self._step_ptrs(key, sts, dev)
                    torch.cuda.synchronize(dev)
                    with torch.cuda.graph(gr, pool=self.pool):
                        for _ in range(n_body):
                            self._body(*args)
                    self.graphs[gkey] = gr
                    self.captures += 1
                    while len(self.graphs) > self.MAX_GRAPHS:   # oldest first (e.g. a learning-rate schedule)
                        self._evict(next(iter(self.graphs)))
                    gr.replay()
                else:
                    self._body(*args)
                    self.eager += 1
                    self._seen.add(key)
                    i += 1
                    continue
                self.replays += n_body
                i += n_body
        finally:
            for g, c in zip(optimizer.param_groups, saved):
                g["capturable"] = c
        return terms_all.clone()
