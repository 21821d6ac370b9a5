"""Reconstruction loop on the HIP engine: PtyRAD's recon_step contract + RCCL data parallelism.

Mirrors ``src/ptyrad/reconstruction.py``:
  select_scan_indices :441-477, make_batches :479-587 ('random', 'compact' and 'sparse'),
  recon_step :658-781 (Adam / SGD branch), toggle_grad_requires :783-790, loss_logger :808-832.

Hot loop: every optimizer step's group of ``grad_accumulation`` mini-batches is ONE engine call
(``CombinedLoss.fused_into``: each batch keeps its own NRMSE normalisation, and the engine
accumulates Σ_m ∂loss_m/∂θ / grad_accumulation straight into ``.grad`` — the reference's
accumulated gradient, reconstruction.py:741-760, without autograd temporaries).

Multi-GPU (replaces the accelerate/DDP wrapper, utils/common.py:58-90): ``DistContext``.
* A group with at least as many mini-batches as ranks is dealt round-robin, whole mini-batches
  per rank.  A group with fewer (the reference default grad_accumulation = 1) is SPLIT: every rank
  takes a contiguous part of every mini-batch (the reference's split_batches=True,
  utils/common.py:63), the engine's per-batch loss sums are all-reduced between its forward and
  its adjoint (ptyx_forward_loss_grad_begin / _end), and each loss keeps the single-device
  normalisation of its WHOLE mini-batch — exact, unlike DDP's average of per-rank losses.
* Batches are fixed for the run (recon_loop never regroups, reconstruction.py:634-636), so
  ``DistContext.local_indices`` tells each rank, before loading anything, which scan positions'
  DPs it needs: the rank keeps only those (PtychoHIP ``measurements_index``), unlike DDP which
  holds and broadcasts the whole stack.
* The ``.grad`` of every parameter the loss reaches and that is trainable this iteration
  (``toggle_grad_requires``) is a view into ONE flat buffer; the engine accumulates into the
  views, ONE all-reduce(sum) of the buffer gives every rank the exact single-device accumulated
  gradient (up to fp32 summation order), with no pack / unpack copies.  Frozen or unreached
  parameters keep ``.grad = None`` (Adam skips them, as on one device).
* Every rank then takes the same optimizer step, so replicas stay identical.  No per-forward
  buffer broadcast, no loss averaging.
"""
from __future__ import annotations

import hashlib
import time
import zlib

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


def make_batches(indices, pos, batch_size, mode="random", verbose=True, rng=None, random_state=None):
    """Mini-batches of ~batch_size indices (reference :479-587).

    'random'  = shuffled array_split;
    'compact' = MiniBatchKMeans clusters of the positions;
    'sparse'  = one seed per compact cluster (the position closest to its centroid), then every
                other index, in index order, joins the group whose nearest member is FARTHEST
                from it (reference :548-587).  Same greedy rule; the per-group minimum distances
                are kept as a running (groups × positions) array instead of the reference's full
                pairwise-distance matrix, so memory is O(groups · positions), not O(positions²).
    """
    indices = np.asarray(indices)
    if pos is not None and len(indices) and indices.max() >= len(pos):
        raise ValueError(f"Maximum index '{indices.max()}' is larger than total number of probe positions ({len(pos)})")
    num_batch = max(1, len(indices) // batch_size)
    if mode == "random":
        rng = rng if rng is not None else np.random.default_rng()
        return np.array_split(rng.permutation(indices), num_batch)
    if mode not in ("compact", "sparse"):
        raise ValueError(f"GROUP_MODE '{mode}' must be 'random', 'compact' or 'sparse'")
    from sklearn.cluster import MiniBatchKMeans
    pos = np.asarray(pos)
    pos_s = pos[indices]
    km = MiniBatchKMeans(init="k-means++", n_init=10, n_clusters=num_batch, max_iter=10, batch_size=3072,
                         random_state=random_state)
    km.fit(pos_s)
    compact = [indices[np.where(km.labels_ == b)[0]] for b in range(num_batch)]
    if mode == "compact":
        return compact
    return sparse_groups(indices, pos, compact)


def sparse_groups(indices, pos, compact):
    """The 'sparse' grouping of make_batches (reference :548-587) from its compact clusters."""
    from scipy.spatial.distance import cdist
    indices = np.asarray(indices)
    pos = np.asarray(pos)
    pos_s = pos[indices]
    groups, used = [], []
    for cb in compact:
        centroid = np.mean(pos[cb], axis=0)
        j = int(np.argmin(np.linalg.norm(pos_s - centroid, axis=1)))
        groups.append([int(indices[j])])
        used.append(j)
    # dmin[g, s] = min over members m of group g of |pos[m] - pos[s]| (cdist, as the reference)
    dmin = np.stack([cdist(pos[[g[0]]], pos)[0] for g in groups])
    for idx in np.delete(indices.copy(), used):
        g = int(np.argmax(dmin[:, idx]))
        groups[g].append(int(idx))
        np.minimum(dmin[g], cdist(pos[[idx]], pos)[0], out=dmin[g])
    flat = np.sort(np.concatenate(groups))
    if not np.array_equal(flat, np.sort(indices)):
        raise AssertionError("sparse grouping lost or duplicated an index")
    return [np.array(g) for g in groups]


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

    def __init__(self, group=None, split_batches=None, always_reduce=False, band_exchange=False,
                 slot_exchange=True):
        """split_batches: None = split a group's mini-batches over the ranks only when the group has
        fewer mini-batches than ranks; True = always (accelerate's split_batches=True,
        utils/common.py:63); False = never (whole mini-batches round-robin).
        always_reduce: run the collectives even with one rank (tests that exercise RCCL on one GPU).
        band_exchange: object gradients by row band (ObjectBands): each rank sends only the rows
        its windows touched to their owners, owners run the optimizer on their band (ZeRO-1),
        then send the updated rows back to the ranks that read them; the rest of the gradient is
        all-reduced.  False (default): one flat all-reduce; True: always by band; "auto": by band
        when the ranks' touched rows line up by rank within a window of their bands (a row-sharded
        scan), else the flat all-reduce.  The band exchange is opt-in because it changes what the
        caller's optimizer holds: the object moments live in the band optimizer
        (``ObjectBands.opt``), so ``optimizer.state_dict()`` lacks them (a resumed run restarts
        them), and its steps are not graph-replayed.  With the band exchange, call
        ``sync_object(model)`` on every rank before reading the object outside recon_step.
        slot_exchange: in a SPLIT optimizer step (every mini-batch split over the ranks), the
        object gradient is formed on every rank from all ranks' per-pattern object-gradient slots
        (one all-gather of 32/W slots a rank at the default cadence, then the deterministic gather
        over all of them: bitwise the same on every rank) and the step's position-gradient rows are
        exchanged with them, so only the probe gradient and the loss terms are all-reduced — instead
        of an all-reduce of the whole object (SlotExchange).  Used when the engine keeps slots
        (CombinedLoss.slot_exchange_ok); False: the flat all-reduce."""
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.split_batches = split_batches
        self.always_reduce = bool(always_reduce) and dist.is_initialized()
        if band_exchange is None:
            band_exchange = False
        if band_exchange != "auto":
            band_exchange = bool(band_exchange)
        self.band_exchange = band_exchange
        self.slot_exchange = bool(slot_exchange)
        self._slot_bufs = {}
        self.bands = None
        self.block_split = None   # the split decision local_indices built a measurement block for

    def _collective(self) -> bool:
        return self.world > 1 or self.always_reduce

    def my_batches(self, group_batches):
        """Round-robin deal of a group's mini-batches to ranks (positions of batch b on rank b % world)."""
        return [i for i in range(len(group_batches)) if i % self.world == self.rank]

    def splits(self, group_batches) -> bool:
        """A group with fewer mini-batches than ranks is split within its mini-batches (same
        decision on every rank: it depends only on the group size, the world size and the
        split_batches setting)."""
        if self.split_batches is not None:
            return bool(self.split_batches)
        return 1 < self.world and len(group_batches) < self.world

    def split_ranges(self, group, cap):
        """Consecutive mini-batch ranges [a, b) of a split group whose parts fit one engine call of
        ``cap`` patterns on EVERY rank: decided from the whole mini-batches' sizes (rank 0's part,
        ⌈len / world⌉, is the largest), so all ranks cut the group alike and each range is one
        all-reduce of its loss sums on every rank.  Exact: every mini-batch keeps its own
        normalisation.  A single part larger than ``cap`` raises on every rank alike."""
        sizes = [-(-len(np.asarray(b).reshape(-1)) // self.world) for b in group]
        if cap is None or cap <= 0:
            return [(0, len(group))]
        if max(sizes, default=0) > cap:
            raise ValueError(f"a mini-batch part of {max(sizes)} positions exceeds the engine's call capacity {cap}")
        out, a, n = [], 0, 0
        for i, s in enumerate(sizes):
            if i > a and n + s > cap:
                out.append((a, i))
                a, n = i, 0
            n += s
        out.append((a, len(group)))
        return out

    def my_part(self, batch):
        """This rank's contiguous share of one mini-batch (np.array_split over the ranks; rank 0's
        share is never empty for a non-empty mini-batch)."""
        return np.array_split(np.asarray(batch).reshape(-1), self.world)[self.rank]

    def local_batches(self, batches, grad_accumulation=1, split=True):
        """The mini-batches (or parts of them) this rank processes over one iteration of recon_step.
        split=False: the loss cannot be split (CombinedLoss.supports_batch_split), whole batches."""
        ga = max(1, int(grad_accumulation))
        split = bool(split)
        out = []
        for g0 in range(0, len(batches), ga):
            group = batches[g0:g0 + ga]
            if split and self.splits(group):
                out += [p for p in (self.my_part(b) for b in group) if p.size]
            else:
                out += [group[i] for i in self.my_batches(group)]
        return out

    def allreduce_sums(self, t):
        """Sum of the engine's per-mini-batch loss sums over the ranks (in place; float64)."""
        if self._collective():
            dist.all_reduce(t, group=self.group)

    def local_indices(self, batches, grad_accumulation=1, split=None, loss_fn=None, model_params=None,
                      init_variables=None):
        """Sorted scan indices whose DPs this rank needs: its ``measurements_index`` block.

        split: whether groups with fewer mini-batches than ranks are split within the mini-batches.
        None = the decision recon_step makes, ``loss_fn.supports_batch_split`` on the model these
        ``model_params`` / ``init_variables`` build (True without a loss_fn).  The decision is
        recorded; recon_step refuses (on every rank, before any collective) to run a split that
        disagrees with it, since the block would then lack DPs the rank is given."""
        if split is None:
            split = loss_fn.supports_batch_split(model_params=model_params, init_variables=init_variables) \
                if loss_fn is not None else True
        self.block_split = bool(split)
        mine = self.local_batches(batches, grad_accumulation, split)
        if not mine:
            return np.zeros(0, np.int64)
        return np.unique(np.concatenate([np.asarray(b).reshape(-1) for b in mine]))

    def grad_views(self, params, extra=0, device=None):
        """Give each param a zeroed ``.grad`` that is a view into ONE flat f32 buffer; returns it.
        ``params`` must be the same list, in the same order, on every rank.  The buffer is reused
        from step to step (zeroed on the device) while the list stays the same.  ``extra`` floats
        follow the parameters' views: the step's (G, 5) loss terms ride in the same all-reduce
        (``terms_tail``), so a step needs no separate collective for them."""
        n = sum(p.numel() for p in params) + int(extra)
        dev = params[0].device if params else (device or torch.device("cpu"))
        key = (tuple(id(p) for p in params), int(extra))
        cached = getattr(self, "_flat", None)
        if cached is not None and cached[0] == key and cached[1].numel() == n and cached[1].device == dev:
            flat = cached[1]
            flat.zero_()
        else:
            flat = torch.zeros(n, dtype=torch.float32, device=dev)
            self._flat = (key, flat)
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return flat

    def sync_object(self, model):
        """Make the whole object current on every rank.  Call it on EVERY rank (it is a
        collective) before reading the object outside recon_step — a checkpoint, a plot — when the
        band exchange is in use: it leaves rows a rank neither owns nor reads out of date."""
        if self.bands is not None and self.bands.stale:
            self.bands.sync([model.opt_obja, model.opt_objp])
        model._stale_object = False

    def agree(self, *items, device=None):
        """For each ``items`` tuple (plain values): whether every rank holds the same one.  ONE
        all-reduce(MAX) of (h, -h) per tuple, h a 62-bit hash of its repr; every rank gets the
        same answers, so every rank takes the same branch afterwards."""
        if not self._collective():
            return [True] * len(items)
        hs = [int.from_bytes(hashlib.blake2b(repr(it).encode(), digest_size=8).digest(), "little") >> 2
              for it in items]
        on_dev = dist.get_backend(self.group) == "nccl" and device is not None
        t = torch.tensor([v for h in hs for v in (h, -h)], dtype=torch.int64,
                         device=device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        t = t.cpu().tolist()
        return [t[2 * i] == h and -t[2 * i + 1] == h for i, h in enumerate(hs)]

    def step_plan(self, batches, ga, split_ok, band, n_flat, cap):
        """What this iteration's collectives depend on, as plain values: the mini-batches (sizes
        and a CRC of their indices: every rank must iterate the same global batching), the
        grad_accumulation, the split decision of every optimizer step and its engine-call ranges
        (one loss-sum all-reduce each), the exchange and the flat gradient size.  Ranks that
        disagree on any of these would pair mismatched RCCL collectives (a hang)."""
        crc, sizes = 0, []
        for b in batches:
            a = np.ascontiguousarray(np.asarray(b).reshape(-1), dtype=np.int64)
            crc = zlib.crc32(a.tobytes(), crc)
            sizes.append(int(a.size))
        steps = []
        for g0 in range(0, len(batches), ga):
            group = batches[g0:g0 + ga]
            sp = bool(split_ok) and self.splits(group)
            steps.append((sp, len(group), tuple(self.split_ranges(group, cap)) if sp else None))
        return (self.world, int(ga), bool(split_ok), bool(band), int(n_flat), tuple(sizes), crc, tuple(steps))

    def allreduce(self, flat):
        """ONE all-reduce(sum) of the gradient buffer (in place)."""
        if self._collective() and flat is not None and flat.numel():
            dist.all_reduce(flat, group=self.group)

    def all_gather_into(self, out, inp):
        """out (W·k, ...) = every rank's inp (k, ...), rank by rank (one all-gather)."""
        if not self._collective():
            out.copy_(inp)
        elif dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, inp, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world)), inp, group=self.group)

    def slot_cap(self, group):
        """Patterns per rank of a split engine call over ``group``'s mini-batches, padded to the
        largest rank's share (rank 0's: Σ ⌈|b| / W⌉), the same on every rank."""
        return sum(-(-len(np.asarray(b).reshape(-1)) // self.world) for b in group)

    def slot_buffers(self, device, block):
        """Persistent (this rank's block, all ranks' blocks) buffers of the slot exchange (a
        captured step holds their addresses)."""
        key = (str(device), int(block))
        b = self._slot_bufs.get(key)
        if b is None:
            b = (torch.zeros(block, dtype=torch.float32, device=device),
                 torch.zeros(self.world * block, dtype=torch.float32, device=device))
            self._slot_bufs[key] = b
        return b

    @staticmethod
    def terms_tail(flat, extra, G):
        """The (G, 5) loss-term rows at the start of the ``extra`` floats grad_views appended."""
        n0 = flat.numel() - int(extra)
        return flat[n0:n0 + 5 * G].view(G, 5)

    def put_terms(self, tail, terms_local, idx_local):
        """Rows of the group's loss terms this rank owns, into the (zeroed) tail of the flat
        buffer: after the gradient all-reduce every rank holds the whole group's terms."""
        if len(idx_local):
            if list(idx_local) == list(range(tail.shape[0])):
                tail.copy_(terms_local)
            else:
                tail[torch.as_tensor(idx_local, device=tail.device)] = terms_local.to(tail.device)


class SlotExchange:
    """The object-gradient exchange of one split engine call (DistContext.slot_exchange; replaces
    the object part of DDP's gradient all-reduce, reconstruction.py:753, at the default cadence).

    Every rank runs its parts of the step's mini-batches with the object gather deferred
    (ptyx_forward_loss_grad_begin / _end with PTYX_PREP_DEFER_GATHER), exports its patterns'
    unit-coefficient object-gradient slots and table rows (window origin, mini-batch coefficients,
    scan index and position-gradient row) padded to ``cap`` patterns as ONE block, all-gathers the
    blocks (one collective), and runs the deterministic slot gather over all W·cap rows: the
    object gradient of the whole step, identical on every rank, and the other ranks'
    position-gradient rows added to its own.  Bytes a rank sends: its cap slots (128 KiB each at
    N = 128) and rows, against 2·(W−1)/W of the object and position gradients for the all-reduce."""

    def __init__(self, ctx, cap, defer=False):
        self.ctx, self.cap = ctx, int(cap)
        # defer: the call only exports and all-gathers; finish() runs the gather later (after the
        # caller's all-reduce of the other gradients, so the optimizer step can ride in it)
        self.defer, self._pending = bool(defer), None

    def _block(self, plan):
        """(this rank's block, all blocks): with RCCL the rank's block IS its slice of the
        all-gather output (in place: the engine writes its slots there, nothing is copied)."""
        ctx = self.ctx
        bf = plan.slot_block_floats(self.cap)
        send, recv = ctx.slot_buffers(plan.device, bf)
        inplace = ctx._collective() and dist.get_backend(ctx.group) == "nccl"
        return (recv[ctx.rank * bf:(ctx.rank + 1) * bf] if inplace else send), recv

    def target(self, plan):
        """(block, cap) for ptyx_plan_slot_target before the engine call."""
        return self._block(plan)[0], self.cap

    def __call__(self, plan, t, grads, cfg, used=True):
        ctx, cap = self.ctx, self.cap
        mine, recv = self._block(plan)
        plan.export_slots(cap, mine, grads.get("shifts"), use_last=used)
        ctx.all_gather_into(recv, mine)
        self._pending = (plan, recv, t, grads, cfg.sparse_n if cfg.sparse_on else 1)
        if not self.defer:
            self.finish()

    def finish(self, adam=False):
        """The deferred gather over every rank's slots; ``adam``: with the optimizer step the plan has
        registered (ptyx_obj_gather_slots_adam: the other gradients must be final by now)."""
        plan, recv, t, grads, sn = self._pending
        self._pending = None
        plan.gather_slots(recv, self.ctx.world, self.cap, self.ctx.rank, t, grads, sn, adam=adam)

    def dense(self, tensors):
        """The same exchange for a loss without slots (the CPU test doubles): each tensor holds
        this rank's contribution and becomes, on every rank, the sum of all ranks' contributions
        in rank order (one all-gather each)."""
        W = self.ctx.world
        for x in tensors:
            buf = torch.empty((W,) + tuple(x.shape), dtype=x.dtype, device=x.device)
            self.ctx.all_gather_into(buf.view((W * x.shape[0],) + tuple(x.shape[1:])) if x.dim() else buf, x)
            acc = buf[0].clone()
            for r in range(1, W):
                acc = acc + buf[r]
            x.copy_(acc)

class ObjectBands:
    """Row-band ownership of the object for the band-sized gradient exchange (the
    ZeRO-1 option; replaces the object part of DDP's bucketed all-reduce, reconstruction.py:753).

    Rank j owns rows [e_j, e_{j+1}) of every (O, Nz, Ny, Nx) object tensor.  The edges follow the
    ranks' touched rows (a row-sharded scan: each edge is the middle of two neighbours' overlap,
    so a band is the rank's own rows less half a window at each inner edge), or are uniform when
    the touched ranges do not line up by rank.  A rank's windows touch rows [lo, hi) only, so its
    object gradient is zero elsewhere.  Per optimizer step:
      reduce   each rank sends the rows of [lo, hi) that other ranks own to their owners (P2P); an
               owner adds what it receives to its own rows, in rank order;
      step     the caller's optimizer class, with the same hyperparameters, steps views of the
               owned rows (optimizer state for 1/W of the object per rank);
      halo     each owner sends its updated rows that other ranks touch back to them (P2P): every
               rank again holds current values of the rows its windows read.
    Bytes per rank and step: twice the touched rows outside the own band (the halo of a
    row-sharded scan), instead of a full-object all-reduce (2·(W−1)/W of the object).  Rows a rank
    neither owns nor touches go stale; ``sync`` (one all-gather of the bands) refreshes the whole
    object when a consumer needs it: a constraint with a global footprint (recon_step checks
    CombinedConstraint.object_footprint), a checkpoint or a plot (``DistContext.sync_object``).
    A pixel that at most two ranks touch gets the same sum as the all-reduce bit for bit (a + b);
    with more contributors only the fp32 summation order differs.

    Optimizer state: the objects' moments live in this rank's band optimizer (``ObjectBands.opt``),
    not in the caller's optimizer, so ``optimizer.state_dict()`` (save.py:110's optim_state_dict)
    does not hold them: a run resumed from such a checkpoint restarts the object moments.  The
    band optimizer's hyperparameters (lr, betas, …) are copied from the caller's groups every step."""

    def __init__(self, ctx, Ny, device, ranges=None):
        self.ctx, self.Ny, self.device = ctx, int(Ny), device
        W = ctx.world
        self.ranges = list(ranges) if ranges is not None else [(0, self.Ny)] * W
        self.edges = self.band_edges(self.ranges, self.Ny, W)
        self.b0, self.b1 = self.edges[ctx.rank], self.edges[ctx.rank + 1]
        self.stale = False        # rows outside [b0, b1) ∪ [lo, hi) may be out of date
        self.opt = None
        self._src_groups = []   # the caller's param group behind each band-optimizer group
        self.views = {}

    @staticmethod
    def band_edges(ranges, Ny, W):
        """W + 1 edges: the middles of neighbouring ranks' touched ranges when those are ordered by
        rank (lo and hi increasing), else the uniform split ⌈Ny / W⌉."""
        lo = [r[0] for r in ranges]
        hi = [r[1] for r in ranges]
        if W > 1 and all(lo[j] < lo[j + 1] and hi[j] < hi[j + 1] for j in range(W - 1)) and \
                all(h > l for l, h in ranges):
            e = [0]
            for j in range(1, W):
                e.append(min(Ny, max(e[-1], (hi[j - 1] + lo[j]) // 2)))
            return e + [Ny]
        R = -(-Ny // W)
        return [min(Ny, j * R) for j in range(W)] + [Ny]

    @classmethod
    def disjoint(cls, ranges, Ny, W, halo):
        """The ranks' touched rows line up by rank and each reaches at most ``halo`` rows past its
        band: the band exchange then moves halos instead of whole objects (the auto default)."""
        e = cls.band_edges(ranges, Ny, W)
        ordered = all(ranges[j][0] < ranges[j + 1][0] and ranges[j][1] < ranges[j + 1][1] for j in range(W - 1))
        return W > 1 and ordered and all(h > l and l >= e[j] - halo and h <= e[j + 1] + halo
                                         for j, (l, h) in enumerate(ranges))

    def set_rows(self, lo, hi):
        """Every rank's touched rows [lo, hi), exchanged (one small all-gather; every rank calls it)."""
        self.ranges = exchange_ranges(self.ctx, lo, hi, self.device)

    def band(self, j):
        return self.edges[j], self.edges[j + 1]

    def _peer(self, r):
        return dist.get_global_rank(self.ctx.group, r) if self.ctx.group is not None else r

    def sent_rows(self):
        """Rows this rank sends in reduce() — and receives back in halo() (the all-reduce would
        move 2·(W−1)/W of Ny)."""
        lo, hi = self.ranges[self.ctx.rank]
        return sum(max(0, min(hi, self.band(j)[1]) - max(lo, self.band(j)[0]))
                   for j in range(self.ctx.world) if j != self.ctx.rank)

    def halo_rows(self):
        """Rows of this rank's band that other ranks touch (sent in halo())."""
        return sum(max(0, min(h, self.b1) - max(l, self.b0))
                   for i, (l, h) in enumerate(self.ranges) if i != self.ctx.rank)

    def _exchange(self, t, sends, recvs):
        """One batched P2P group: sends [(peer, a, b)] rows of t, receives [(peer, a, b)] rows into
        fresh buffers; returns [(a, b, buf)] in peer order."""
        ops, bufs = [], []
        for j, a, b in sends:
            ops.append(dist.P2POp(dist.isend, t[:, :, a:b].contiguous(), self._peer(j), self.ctx.group))
        for i, a, b in recvs:
            buf = torch.empty(t[:, :, a:b].shape, dtype=t.dtype, device=t.device)
            ops.append(dist.P2POp(dist.irecv, buf, self._peer(i), self.ctx.group))
            bufs.append((a, b, buf))
        # one batched group: RCCL pairs every send with its receive without ordering deadlocks
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        return bufs

    def _pairs(self, mine_rows):
        """(peer, a, b) row blocks: mine_rows=True → my touched rows in peer j's band (reduce
        sends, halo receives); False → peer i's touched rows in my band (reduce receives, halo
        sends)."""
        me, W = self.ctx.rank, self.ctx.world
        out = []
        for j in range(W):
            if j == me:
                continue
            if mine_rows:
                a, b = max(self.ranges[me][0], self.band(j)[0]), min(self.ranges[me][1], self.band(j)[1])
            else:
                a, b = max(self.ranges[j][0], self.b0), min(self.ranges[j][1], self.b1)
            if a < b:
                out.append((j, a, b))
        return out

    def reduce(self, grads):
        """grads: (O, Nz, Ny, Nx) object-gradient tensors, in place: the owner's rows get the sum."""
        for g in grads:
            for a, b, buf in self._exchange(g, self._pairs(True), self._pairs(False)):   # in rank order
                g[:, :, a:b] += buf

    def halo(self, params):
        """The owners' current rows back to every rank whose windows read them."""
        for p in params:
            for a, b, buf in self._exchange(p.data, self._pairs(False), self._pairs(True)):
                p.data[:, :, a:b] = buf
        self.stale = self.ctx.world > 1

    def step(self, optimizer, params, candidates=None):
        """Step `optimizer`'s class on the owned rows of the object params (their .grad holds the
        reduced gradient there).  The band optimizer holds a view for every object tensor of
        `optimizer` (`candidates`), so a tensor frozen when it was built still gets its band later;
        a view whose tensor has no .grad this step is skipped, as Adam skips a frozen tensor."""
        if self.opt is None:
            cand = candidates if candidates is not None else params
            groups = []
            for gr in optimizer.param_groups:
                mine = [p for p in gr["params"] if any(p is q for q in cand)]
                if mine:
                    views = []
                    for p in mine:
                        v = torch.nn.Parameter(p.data[:, :, self.b0:self.b1])   # shares p's storage
                        self.views[id(p)] = (p, v)
                        views.append(v)
                    groups.append({**{k: v for k, v in gr.items() if k != "params"}, "params": views})
                    self._src_groups.append(gr)
            self.opt = type(optimizer)(groups, **optimizer.defaults) if groups else None
        if self.opt is not None:   # hyperparameters follow the caller's optimizer (lr schedules, edits)
            for bg, gr in zip(self.opt.param_groups, self._src_groups):
                for k, v in gr.items():
                    if k != "params":
                        bg[k] = v
        for p, v in self.views.values():
            v.grad = None
            band = p.data[:, :, self.b0:self.b1]
            if v.data.data_ptr() != band.data_ptr():   # a constraint replaced the tensor's storage
                v.data = band
        for p in params:
            pv = self.views.get(id(p))
            if pv is not None:
                pv[1].grad = p.grad[:, :, self.b0:self.b1] if p.grad is not None else None
        if self.opt is not None:
            self.opt.step()
            for _, v in self.views.values():
                v.grad = None

    def sync(self, params):
        """Every rank receives every owner's rows: the whole object is current again."""
        W = self.ctx.world
        Rm = max(self.edges[j + 1] - self.edges[j] for j in range(W))
        for p in params:
            O, Nz, _, Nx = p.shape
            mine = torch.zeros((O, Nz, Rm, Nx), dtype=p.dtype, device=p.device)
            mine[:, :, :self.b1 - self.b0] = p.data[:, :, self.b0:self.b1]
            out = torch.empty(W * mine.numel(), dtype=p.dtype, device=p.device)
            if W > 1:
                dist.all_gather_into_tensor(out, mine.reshape(-1), group=self.ctx.group)
            else:
                out.copy_(mine.reshape(-1))
            out = out.view((W,) + tuple(mine.shape))
            for j in range(W):
                a, b = self.band(j)
                if a < b and j != self.ctx.rank:
                    p.data[:, :, a:b] = out[j, :, :, :b - a]
        self.stale = False

    gather = sync


def exchange_ranges(ctx, lo, hi, device):
    """Every rank's (lo, hi) (one small all-gather; every rank calls it)."""
    W = ctx.world
    rng_ = torch.tensor([int(lo), int(hi)], dtype=torch.int64,
                        device=device if dist.is_initialized() and dist.get_backend(ctx.group) == "nccl" else "cpu")
    allr = [torch.zeros_like(rng_) for _ in range(W)]
    if W > 1:
        dist.all_gather(allr, rng_, group=ctx.group)
    else:
        allr = [rng_]
    return [(int(r[0]), int(r[1])) for r in allr]


def touched_rows(model, batches, N):
    """Object rows [lo, hi) the windows of these mini-batches reach (crop_pos y + N)."""
    idx = np.concatenate([np.asarray(b).reshape(-1) for b in batches]) if len(batches) else np.zeros(0, int)
    if not idx.size:
        return 0, 0
    cp = getattr(model, "crop_pos", None)
    if cp is None:
        cp = model.crop_pos_np
    cp = cp.cpu().numpy() if isinstance(cp, torch.Tensor) else np.asarray(cp)
    cy = cp[idx, 0]
    return int(cy.min()), int(cy.max()) + int(N)


# ------------------------------------------------------------------ the reference step
GRAPH_MIN_STEPS = 4   # graph replay pays for its capture from this many optimizer steps per iteration


def recon_step(batches, grad_accumulation, model, optimizer, loss_fn, constraint_fn, niter, verbose=True,
               acc=None, dist_ctx=None, graphs=None):
    """One iteration over ``batches`` (reconstruction.py:658-781, non-LBFGS branch).

    Optimizer steps happen every ``grad_accumulation`` batches and after the last one; each step's
    group of batches runs as one fused engine call (sharded over ranks when ``dist_ctx`` is given).

    graphs: replay the optimizer steps from hipGraphs (``ptyrad_amd.stepgraph``; bitwise the same
    trajectory).  None = when eligible and the iteration has ≥ GRAPH_MIN_STEPS steps; False = never;
    True = required (raises with the reason when not eligible).
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
    optimizer.zero_grad(set_to_none=True)
    ga = max(1, int(grad_accumulation))
    dev = model.opt_obja.device
    # parameters whose .grad this iteration's steps fill: trainable now and reached by the loss
    reached = {id(model.optimizable_tensors[k]) for k in model.engine_grad_names()}
    live = [p for p in params if p.requires_grad and id(p) in reached]
    split_ok = hasattr(loss_fn, "supports_batch_split") and loss_fn.supports_batch_split(model)
    if ctx.block_split is not None and ctx.block_split != split_ok and any(
            ctx.splits(batches[g0:g0 + ga]) for g0 in range(0, len(batches), ga)):
        # (the same on every rank: no rank enters a collective this iteration)
        raise ValueError(f"the rank's measurement block was built for split_batches={ctx.block_split} "
                         f"(DistContext.local_indices) but this loss / model {'can' if split_ok else 'cannot'} "
                         "split mini-batches: build it with local_indices(..., loss_fn=loss_fn, model_params=..., "
                         "init_variables=...)")
    objs = [p for p in (model.opt_obja, model.opt_objp) if any(p is q for q in live)]
    band = False
    obj_all = [p for p in (model.opt_obja, model.opt_objp) if any(p is q for q in params)]
    # "auto" remembers a batching it found not row-sharded (every rank iterates the same global
    # batches, so every rank skips alike): no touched-rows pass or range all-gather for it again
    auto_key = None
    if ctx.band_exchange == "auto" and ctx.bands is None and ctx._collective() and objs:
        crc = zlib.crc32(np.ascontiguousarray(np.concatenate([np.asarray(b).reshape(-1) for b in batches]),
                                              dtype=np.int64).tobytes()) if len(batches) else 0
        auto_key = (crc, len(batches), ga, bool(split_ok))
    if ctx.band_exchange is not False and ctx._collective() and objs and \
            not (auto_key is not None and getattr(ctx, "_not_banded", None) == auto_key):
        # the rows each rank's windows reach this iteration (recomputed: the batches may change);
        # band_exchange "auto": by band when the ranks' rows line up (a row-sharded scan)
        N = int(model.opt_probe.shape[1])
        lo, hi = touched_rows(model, ctx.local_batches(batches, grad_accumulation, split_ok), N)
        ranges = exchange_ranges(ctx, lo, hi, dev)
        Ny = int(model.opt_obja.shape[2])
        if ctx.bands is None and (ctx.band_exchange is True or ObjectBands.disjoint(ranges, Ny, ctx.world, N)):
            ctx.bands = ObjectBands(ctx, Ny, dev, ranges)
        elif ctx.bands is None:
            ctx._not_banded = auto_key
        if ctx.bands is not None:
            band = True
            ctx.bands.ranges = ranges
            if ctx.bands.stale:
                ctx.bands.halo(obj_all)      # rows this iteration reads, current from their owners
            live = objs + [p for p in live if not any(p is q for q in objs)]   # objects first in the flat buffer
    # slot exchange (split steps): the object gradient from every rank's per-pattern slots, the
    # position-gradient rows with them; only the rest of the flat buffer is all-reduced
    slots = False
    if ctx.slot_exchange and ctx._collective() and split_ok and not band and objs and \
            getattr(loss_fn, "slot_exchange_ok", None) is not None and loss_fn.slot_exchange_ok(model):
        plan_ = getattr(model, "plan", None)
        cap_ = plan_.call_capacity if plan_ is not None else None
        maxp = int(plan_.dims.max_patterns) if plan_ is not None else None
        sgroups = [batches[g0:g0 + ga] for g0 in range(0, len(batches), ga) if ctx.splits(batches[g0:g0 + ga])]
        slots = bool(sgroups) and (maxp is None or all(
            ctx.world * ctx.slot_cap(g[a:b]) <= maxp for g in sgroups for a, b in ctx.split_ranges(g, cap_)))
    ar_skip = 0
    if slots:
        sp_ = model.opt_probe_pos_shifts
        sh = [p for p in live if p is sp_]
        live = objs + sh + [p for p in live if not any(p is q for q in objs) and p is not sp_]
        ar_skip = sum(p.numel() for p in objs + sh)
    rows = []
    use_graphs = False
    if graphs is not False and not band:
        from .stepgraph import StepGraphs, ineligible_reason
        why = ineligible_reason(model, optimizer, loss_fn, ctx, batches, ga)
        if graphs and why:
            raise RuntimeError(f"recon_step(graphs=True): {why}")
        use_graphs = why is None and (graphs or -(-len(batches) // ga) >= GRAPH_MIN_STEPS) and bool(live)
    # with collectives, the step's loss terms ride in the gradient all-reduce (5·ga extra floats)
    extra = 5 * ga if ctx._collective() else 0
    if ctx._collective():
        # before any step collective: every rank must plan the same collective sequence (else
        # refuse on every rank instead of hanging in RCCL), and take the same graph decision
        # (else every rank runs the eager steps)
        cap = model.plan.call_capacity if hasattr(model, "plan") else None
        plan_fp = ctx.step_plan(batches, ga, split_ok, band, sum(p.numel() for p in live) + extra, cap) + \
            (("slots", bool(slots), int(ar_skip)),)
        same_plan, same_mode = ctx.agree(plan_fp, ("graphs", bool(use_graphs)), device=dev)
        if not same_plan:
            raise RuntimeError(f"recon_step iteration {niter} (rank {ctx.rank}): the ranks disagree on the "
                               "iteration's mini-batches, grad_accumulation, split decision or parameter set, so "
                               "their collectives would not pair up; every rank must pass the same global batches")
        if not same_mode:
            if not getattr(ctx, "_warned_graphs", False):
                print(f"[ptyrad_amd] rank {ctx.rank}: ranks disagree on graph-replay eligibility "
                      f"(this rank: {'eligible' if use_graphs else 'not eligible'}); every rank runs eager steps",
                      flush=True)
                ctx._warned_graphs = True
            use_graphs = False
    if use_graphs:
        sg = getattr(model, "_step_graphs", None)
        if sg is None:
            sg = model._step_graphs = StepGraphs()
        flat = ctx.grad_views(live, extra, dev)
        rows.append(sg.run(model, optimizer, loss_fn, batches, ga, live, flat, ctx=ctx, extra=extra,
                           slots=slots, ar_skip=ar_skip))
        optimizer.zero_grad(set_to_none=True)
        model.clear_cache()
    for g0 in (range(0, len(batches), ga) if not use_graphs else ()):
        group = batches[g0:g0 + ga]
        flat = ctx.grad_views(live, extra, dev)
        if ctx.splits(group) and split_ok:
            # every rank holds a part of every mini-batch; the loss sums are all-reduced inside the
            # engine call, so each mini-batch keeps its whole-batch normalisation.  Rank 0's part of
            # every mini-batch is non-empty: its terms are the group's.
            cap = model.plan.call_capacity if hasattr(model, "plan") else None
            terms = torch.cat([loss_fn.fused_into(model, [ctx.my_part(b) for b in group[a:b]], grad_scale=1.0 / ga,
                                                  batch_sums_reduce=ctx.allreduce_sums,
                                                  **({"slot_exchange": SlotExchange(ctx, ctx.slot_cap(group[a:b]))}
                                                     if slots else {}))
                               for a, b in ctx.split_ranges(group, cap)])
            mine = list(range(len(group))) if ctx.rank == 0 else []
            if ctx.rank:
                terms = terms[:0]
        else:
            if ctx.splits(group) and not getattr(ctx, "_warned_idle", False):
                print(f"[ptyrad_amd] warning: {len(group)} mini-batch(es) per optimizer step on {ctx.world} ranks and "
                      "a loss that cannot be split (pacbed / simlar / blur stages): ranks without a mini-batch idle",
                      flush=True)
                ctx._warned_idle = True
            mine = ctx.my_batches(group)
            if mine:
                terms = loss_fn.fused_into(model, [group[i] for i in mine], grad_scale=1.0 / ga)
            else:
                terms = torch.zeros((0, 5), device=dev)
        if extra:
            tail = ctx.terms_tail(flat, extra, len(group))
            ctx.put_terms(tail, terms, mine)
        if band:
            n_obj = sum(p.numel() for p in objs)
            ctx.allreduce(flat[n_obj:])                # probe, positions, propagator, loss terms:
            ctx.bands.reduce([p.grad for p in objs])   # small (a collective first: RCCL's communicator)
            saved = [p.grad for p in objs]
            for p in objs:
                p.grad = None                          # the caller's optimizer skips the objects
            optimizer.step()
            for p, g in zip(objs, saved):
                p.grad = g
            ctx.bands.step(optimizer, objs, obj_all)
            ctx.bands.halo(objs)                       # updated rows back to the ranks that read them
        else:
            # (a split step's object and position gradients came with the slot exchange)
            ctx.allreduce(flat[ar_skip:] if slots and ctx.splits(group) else flat)
            optimizer.step()
        optimizer.zero_grad(set_to_none=True)
        # the loss terms stay on the device until the iteration ends (no host sync per step)
        rows.append(tail.clone() if extra else terms)
        model.clear_cache()
    for row in (torch.cat(rows).cpu().numpy() if rows else ()):   # one sync per iteration
        for name, v in zip(LOSS_TERM_NAMES, row):
            if name in batch_losses:
                batch_losses[name].append(v)
    check_plans(model, niter)
    if constraint_fn is not None:
        if band and ctx.bands.stale and object_footprint(constraint_fn, niter) == "global":
            ctx.bands.sync(obj_all)              # (a Fourier filter / blur / global min reads every row)
        constraint_fn(model, niter)
    model._stale_object = bool(band and ctx.bands.stale)
    iter_t = time_sync() - t0
    model.loss_iters.append((niter, loss_logger(batch_losses, niter, iter_t, verbose=verbose)))
    model.iter_times.append(iter_t)
    model.dz_iters.append((niter, model.opt_slice_thickness.detach().cpu().numpy()))
    model.avg_tilt_iters.append((niter, model.opt_obj_tilts.detach().mean(0).cpu().numpy()))
    return batch_losses


def object_footprint(constraint_fn, niter):
    """What the constraints of this iteration read of the object: 'none', 'pointwise' (every pixel
    from its own value: a rank's current rows stay exact) or 'global' (anything else, and any
    constraint function that does not say)."""
    f = getattr(constraint_fn, "object_footprint", None)
    return f(niter) if f is not None else "global"


def check_plans(model, niter):
    """Raise the input errors (scan index, window, measurement row out of range) that the device
    flagged during this iteration's engine calls, right after the iteration's one host sync.
    Graph-replayed steps never pass through Plan's per-call check, so without this a bad index
    would surface only at some later eager call (ptyx_plan_check: a host read, no sync)."""
    plans = [getattr(model, "_plan", None)] + list(getattr(model, "_stack_plans", {}).values())
    for pl in plans:
        if pl is None:
            continue
        try:
            pl._prev_errors()
        except IndexError as e:
            raise IndexError(f"recon_step iteration {niter}: {e}") from None


def recon_loop(model, optimizer, loss_fn, constraint_fn, batches, NITER, grad_accumulation=1, verbose=True,
               dist_ctx=None):
    """Minimal recon_loop (reconstruction.py:589-656) without saving/plotting; the whole object is
    current on every rank when it returns."""
    for niter in range(1, NITER + 1):
        recon_step(batches, grad_accumulation, model, optimizer, loss_fn, constraint_fn, niter, verbose=verbose,
                   dist_ctx=dist_ctx)
    if dist_ctx is not None:
        dist_ctx.sync_object(model)
    return model.loss_iters


def create_optimizer(optimizer_params, optimizable_params, verbose=True):
    """torch.optim.<name>(param groups with per-tensor lr, **configs) (reconstruction.py:285-368).

    One deliberate difference: Adam / AdamW on device parameters, with no ``fused`` / ``foreach``
    choice in the configs, are ``ptyrad_amd.optim.Adam`` / ``AdamW``: torch.optim.Adam / AdamW
    themselves (same param groups, state and state_dict) whose update runs as one grid-filling
    HIP launch.  torch's default (foreach) path issues about ten kernels per parameter group from
    Python and its fused path one latency-bound kernel per group, and at the reference's default
    cadence (grad_accumulation = 1, one step per 32-pattern mini-batch) either costs more than the
    engine call (tools/recon_overhead.py, tools/trace_gaps.py)."""
    name = optimizer_params.get("name", "Adam")
    cls = getattr(torch.optim, name, None)
    if cls is None:
        raise ValueError(f"Optimizer '{name}' is not supported.")
    configs = dict(optimizer_params.get("configs") or {})
    params = [p for g in optimizable_params for p in (g["params"] if isinstance(g, dict) else [g])]
    if (name in ("Adam", "AdamW") and "fused" not in configs and "foreach" not in configs and params and
            all(p.is_cuda and p.dtype == torch.float32 for p in params)):
        from . import optim
        cls = getattr(optim, name)
    return cls(optimizable_params, **configs)
