"""Torch-tensor front end of the C ABI (include/ptyx.h): plans, argument marshalling, streams.

All tensors passed here must already live on the plan's device (HBM-resident inputs); the
engine never copies data between host and device and never synchronises the stream.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

LOSS_TERM_NAMES = ("loss_single", "loss_poissn", "loss_pacbed", "loss_sparse", "loss_simlar")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _need(t, dtype, name, device):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


@dataclass
class LossConfig:
    """Hot-path subset of PtyRAD's loss_params (src/ptyrad/params/loss_params.py)."""
    single_on: bool = True
    single_w: float = 1.0
    single_q: float = 0.5
    poissn_on: bool = False
    poissn_w: float = 1.0
    poissn_q: float = 1.0
    poissn_eps: float = 1e-6
    sparse_on: bool = True
    sparse_w: float = 0.1
    sparse_n: int = 1
    pacbed_on: bool = False     # ptyx_loss_pacbed on the fused call's dp, then ptyx_adjoint_dldi
    pacbed_w: float = 0.5
    pacbed_q: float = 0.2

    @classmethod
    def from_loss_params(cls, lp: dict) -> "LossConfig":
        if lp.get("loss_simlar", {}).get("state", False):
            raise NotImplementedError("loss_simlar is not on the fused HIP path; use the generic "
                                      "(autograd) path of ptyrad_amd.losses.CombinedLoss")
        s, p, sp = lp["loss_single"], lp["loss_poissn"], lp["loss_sparse"]
        pb = lp.get("loss_pacbed", {"state": False})
        return cls(bool(s["state"]), float(s.get("weight", 1.0)), float(s.get("dp_pow", 0.5)),
                   bool(p["state"]), float(p.get("weight", 1.0)), float(p.get("dp_pow", 1.0)),
                   float(p.get("eps", 1e-6)),
                   bool(sp["state"]), float(sp.get("weight", 0.1)), int(sp.get("ln_order", 1)),
                   bool(pb["state"]), float(pb.get("weight", 0.5)), float(pb.get("dp_pow", 0.2)))

    def to_c(self, grad_scale: float, max_batch: int = 0, prep: int = 0) -> _lib.LossCfg:
        if self.pacbed_on and not (self.single_on or self.poissn_on):
            # the engine needs one data term: a zero-weight loss_single (adds nothing)
            return _lib.LossCfg(1, 0.0, self.single_q, 0, self.poissn_w, self.poissn_q, self.poissn_eps,
                                int(self.sparse_on), self.sparse_w, int(self.sparse_n), float(grad_scale),
                                int(max_batch), int(prep))
        return _lib.LossCfg(int(self.single_on), self.single_w, self.single_q,
                            int(self.poissn_on), self.poissn_w, self.poissn_q, self.poissn_eps,
                            int(self.sparse_on), self.sparse_w, int(self.sparse_n), float(grad_scale),
                            int(max_batch), int(prep))


class Plan:
    """One ptyx_plan: fixed device and geometry (N, P, O, Nz, object extent, n_scans)."""

    def __init__(self, N, P, O, Nz, Ny, Nx, n_scans, max_patterns, shift_probes=True,
                 meas_f16=False, device=None, prop_grad=False):
        self.lib = _lib.load()
        device = torch.device(device if device is not None else "cuda")
        if device.type != "cuda":
            raise ValueError("ptyx plans need a HIP device (torch 'cuda' device on ROCm)")
        self.device = torch.device("cuda", device.index if device.index is not None
                                   else torch.cuda.current_device())
        flags = ((_lib.PTYX_SHIFT_PROBES if shift_probes else 0) | (_lib.PTYX_MEAS_F16 if meas_f16 else 0) |
                 (_lib.PTYX_PROP_GRAD if prop_grad else 0))
        self.dims = _lib.Dims(int(N), int(P), int(O), int(Nz), int(Ny), int(Nx), int(n_scans),
                              int(max_patterns), flags)
        self.shift_probes = bool(shift_probes)
        self.meas_f16 = bool(meas_f16)
        h = ctypes.c_void_p()
        _lib.check(self.lib.ptyx_plan_create(ctypes.byref(h), ctypes.byref(self.dims), self.device.index))
        self._h = h

    @property
    def workspace_bytes(self) -> int:
        return int(self.lib.ptyx_plan_workspace_bytes(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self.lib.ptyx_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ marshalling
    def _inputs(self, obja, objp, probe_rv, shifts, H, occu, crop_pos, meas, tilts=None, kvec=None, dz=0.0,
                meas_rows=None):
        d, dev = self.dims, self.device
        _need(obja, torch.float32, "obja", dev)
        _need(objp, torch.float32, "objp", dev)
        _need(probe_rv, torch.float32, "probe", dev)
        _need(shifts, torch.float32, "shifts", dev)
        _need(occu, torch.float32, "omode_occu", dev)
        _need(crop_pos, torch.int32, "crop_pos", dev)
        if tuple(obja.shape) != (d.O, d.Nz, d.Ny, d.Nx) or obja.shape != objp.shape:
            raise ValueError(f"object shape {tuple(obja.shape)} != {(d.O, d.Nz, d.Ny, d.Nx)}")
        if tuple(probe_rv.shape) != (d.P, d.N, d.N, 2):
            raise ValueError(f"probe shape {tuple(probe_rv.shape)} != {(d.P, d.N, d.N, 2)}")
        if tuple(shifts.shape) != (d.n_scans, 2) or tuple(crop_pos.shape) != (d.n_scans, 2):
            raise ValueError("shifts / crop_pos must be (n_scans, 2)")
        if H is not None:
            if H.dtype == torch.complex64:
                H = torch.view_as_real(H)
            _need(H, torch.float32, "H", dev)
            if tuple(H.shape) != (d.N, d.N, 2):
                raise ValueError("H must be (N, N) complex64")
        if meas is not None:
            _need(meas, torch.float16 if self.meas_f16 else torch.float32, "meas", dev)
            rows = d.n_scans if meas_rows is None else meas.shape[0]
            if tuple(meas.shape) != (rows, d.N, d.N):
                raise ValueError(f"meas shape {tuple(meas.shape)} != {(rows, d.N, d.N)}")
        if meas_rows is not None:   # rank-local measurement block (scan index -> row)
            _need(meas_rows, torch.int32, "meas_rows", dev)
            if tuple(meas_rows.shape) != (d.n_scans,):
                raise ValueError("meas_rows must be (n_scans,) int32")
        if tilts is not None:
            _need(tilts, torch.float32, "obj_tilts", dev)
            _need(kvec, torch.float32, "kvec", dev)
            if tuple(tilts.shape) != (d.n_scans, 2) or tuple(kvec.shape) != (d.N,):
                raise ValueError("per-position obj_tilts must be (n_scans, 2) and kvec (N,)")
        rows_n = int(meas.shape[0]) if (meas is not None and meas_rows is not None) else 0
        inp = _lib.Inputs(_ptr(obja), _ptr(objp), _ptr(probe_rv), _ptr(shifts), _ptr(H), _ptr(occu),
                          _ptr(crop_pos), _ptr(meas), _ptr(tilts), _ptr(kvec if tilts is not None else None),
                          float(dz), _ptr(meas_rows), rows_n)
        return inp, H

    def _idx(self, idx):
        if isinstance(idx, torch.Tensor) and idx.device == self.device and idx.dtype == torch.int32:
            return idx.contiguous()
        return torch.as_tensor(np.asarray(idx.cpu() if isinstance(idx, torch.Tensor) else idx),
                               dtype=torch.int32).to(self.device, non_blocking=True)

    def _grads(self, grads: dict | None):
        grads = grads or {}
        d, dev = self.dims, self.device
        for k, shape in (("obja", (d.O, d.Nz, d.Ny, d.Nx)), ("objp", (d.O, d.Nz, d.Ny, d.Nx)),
                         ("probe", (d.P, d.N, d.N, 2)), ("shifts", (d.n_scans, 2)), ("H", (d.N, d.N, 2)),
                         ("tilts", (d.n_scans, 2)), ("dz", ())):
            g = grads.get(k)
            if g is not None:
                _need(g, torch.float32, f"grad {k}", dev)
                if tuple(g.shape) != shape:
                    raise ValueError(f"grad {k} shape {tuple(g.shape)} != {shape}")
        return _lib.Grads(_ptr(grads.get("obja")), _ptr(grads.get("objp")), _ptr(grads.get("probe")),
                          _ptr(grads.get("shifts")), _ptr(grads.get("H")), _ptr(grads.get("tilts")),
                          _ptr(grads.get("dz")))

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ per-kernel timing
    def profile_begin(self):
        _lib.check(self.lib.ptyx_profile_begin(self._h))

    def profile_end(self) -> dict:
        """{kernel name: (launches, total_ms)} from HIP events recorded on the launch stream."""
        cap = 32
        arr = (_lib.KernelStat * cap)()
        n = ctypes.c_int32(0)
        _lib.check(self.lib.ptyx_profile_end(self._h, arr, cap, ctypes.byref(n)))
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].total_ms))
                for i in range(min(n.value, cap))}

    # ------------------------------------------------------------------ entry points
    def forward(self, t: dict, idx, dp_out=None):
        """ptyx_forward: dp (n, N, N) f32 = PtychoAD.forward(idx); calls larger than the plan's
        max_patterns run in pieces (patterns are independent in the forward model)."""
        self._prev_errors()
        idx_t = self._idx(idx)
        n = int(idx_t.numel())
        if dp_out is None:
            dp_out = torch.empty((n, self.dims.N, self.dims.N), dtype=torch.float32, device=self.device)
        inp, _keep = self._inputs(t["obja"], t["objp"], t["probe"], t["shifts"], t.get("H"), t["occu"],
                                  t["crop_pos"], None, t.get("tilts"), t.get("kvec"), t.get("dz", 0.0))
        step = max(1, int(self.dims.max_patterns))
        for a in range(0, n, step):
            b = min(n, a + step)
            _lib.check(self.lib.ptyx_forward(self._h, self._stream(), ctypes.byref(inp), _ptr(idx_t[a:b]), b - a,
                                             _ptr(dp_out[a:b])))
        return dp_out

    def _prev_errors(self):
        """Input errors the device flagged in an earlier call on this plan (include/ptyx.h:
        ptyx_plan_check; a host read, no synchronisation), raised as IndexError — what the
        reference's advanced indexing raises (models.py:261-264)."""
        rc = self.lib.ptyx_plan_check(self._h)
        if rc == _lib.PTYX_EINVAL:
            raise IndexError(self.lib.ptyx_last_error().decode())
        _lib.check(rc)

    def check(self):
        """Synchronise the plan's stream and raise IndexError if any call so far had a scan index,
        window or meas_rows entry out of range (the device checks every pattern as it reads it)."""
        torch.cuda.current_stream(self.device).synchronize()
        self._prev_errors()

    def forward_loss_grad(self, t: dict, idx, batch_offsets, loss_cfg: LossConfig, grads: dict,
                          grad_scale: float = 1.0, loss_terms=None, dp_out=None, max_batch=None, prep=0,
                          batch_sums_reduce=None, slot_exchange=None, _rows_checked=False):
        """ptyx_forward_loss_grad over consecutive mini-batches; returns loss_terms (n_batches, 5).

        batch_offsets on the host (numpy / list / CPU tensor) let calls larger than the plan's
        capacity (max_patterns, or the register engines' slot capacity) be split at mini-batch
        boundaries; device offsets must fit in one call.

        batch_sums_reduce: the mini-batches are this rank's PARTS of mini-batches split over ranks
        (ptyx_forward_loss_grad_begin / _end).  It is called with the (n_batches, PTYX_BATCH_SUMS) float64
        device tensor of the parts' additive loss sums and must sum it over the ranks in place
        (one all-reduce); the loss terms and gradient coefficients then belong to the whole
        mini-batches.  Such a call is never split, so it must fit the plan's capacity.

        slot_exchange (with batch_sums_reduce; plans with ``slot_floats`` > 0): the call leaves the
        object gradient to ``slot_exchange(plan, t, grads, loss_cfg)``, which exports this rank's
        per-pattern slots, all-gathers them and runs ``gather_slots`` over every rank's patterns
        (reconstruction.SlotExchange).
        """
        self._prev_errors()   # (_rows_checked: kept for callers; the device checks every call)
        if batch_sums_reduce is not None:
            return self._split_call(t, idx, batch_offsets, loss_cfg, grads, grad_scale, loss_terms, dp_out,
                                    batch_sums_reduce, slot_exchange)
        if slot_exchange is not None:
            raise ValueError("slot_exchange is for split-batch calls (batch_sums_reduce)")
        host_off = not (isinstance(batch_offsets, torch.Tensor) and batch_offsets.device.type != "cpu")
        if max_batch is None:
            if not host_off:
                max_batch = 0
            else:
                off = np.asarray(batch_offsets)
                max_batch = int(np.max(np.diff(off))) if off.size > 1 else 0
        cap = self.register_capacity
        cap = min(cap, int(self.dims.max_patterns)) if cap > 0 else int(self.dims.max_patterns)
        if host_off:
            off = np.asarray(batch_offsets.cpu() if isinstance(batch_offsets, torch.Tensor) else batch_offsets,
                             dtype=np.int64)
            if off[-1] - off[0] > cap and np.max(np.diff(off)) <= cap:
                if prep & (_lib.PTYX_PREP_FUSED_ADAM | _lib.PTYX_PREP_SELECT):
                    raise ValueError("PTYX_PREP_FUSED_ADAM / PTYX_PREP_SELECT on a call larger than one engine call")
                return self._chunked(t, idx, off, cap, loss_cfg, grads, grad_scale, loss_terms, dp_out, max_batch,
                                     store=bool(prep & _lib.PTYX_PREP_GRAD_STORE))
        idx_t = self._idx(idx)
        off_t = self._idx(batch_offsets)
        n, nb = int(idx_t.numel()), int(off_t.numel()) - 1
        if loss_terms is None:
            loss_terms = torch.empty((nb, 5), dtype=torch.float32, device=self.device)
        inp, _keep = self._inputs(t["obja"], t["objp"], t["probe"], t["shifts"], t.get("H"), t["occu"],
                                  t["crop_pos"], t["meas"], t.get("tilts"), t.get("kvec"), t.get("dz", 0.0),
                                  t.get("meas_rows"))
        cfg = loss_cfg.to_c(grad_scale, max_batch, prep)
        g = self._grads(grads)
        _lib.check(self.lib.ptyx_forward_loss_grad(self._h, self._stream(), ctypes.byref(inp), _ptr(idx_t),
                                                   _ptr(off_t), nb, n, ctypes.byref(cfg), _ptr(loss_terms),
                                                   _ptr(dp_out), ctypes.byref(g)))
        return loss_terms

    def set_select(self, idx_all, istart, cnt, grad, grad_n, steps, n_steps):
        """ptyx_plan_set_select: the step selection (ptyx_step_select's arguments, device pointers)
        the next forward_loss_grad call with PTYX_PREP_SELECT begins with; the call's idx is then
        the output buffer its indices are picked into."""
        _lib.check(self.lib.ptyx_plan_set_select(self._h, idx_all, istart, cnt, grad, int(grad_n), steps,
                                                 int(n_steps)))

    def set_adam(self, args, store=None):
        """ptyx_plan_set_adam: the optimizer step the next forward_loss_grad call with
        PTYX_PREP_FUSED_ADAM takes.  ``args``: ptyrad_amd.optim's ``fused_step_args()``; ``store``:
        (terms, nb, rstart, cnt, terms_all) device pointers of the step's ptyx_step_store, or None."""
        st = store if store is not None else (None, 0, None, None, None)
        _lib.check(self.lib.ptyx_plan_set_adam(self._h, *args, *st))

    def loss_pacbed(self, t: dict, idx, batch_offsets, dp, loss_cfg: LossConfig, loss_terms, grad_scale=1.0,
                    want_dldi=True):
        """ptyx_loss_pacbed: writes loss_terms[:, 2] and returns dL/d(dp) (or None)."""
        idx_t = self._idx(idx)
        off_t = self._idx(batch_offsets)
        n, nb = int(idx_t.numel()), int(off_t.numel()) - 1
        _need(dp, torch.float32, "dp", self.device)
        meas = t["meas"]
        if t.get("meas_rows") is not None:   # pacbed addresses meas through idx only: map it to rows
            idx_t = t["meas_rows"][idx_t.long()].contiguous()
        _need(meas, torch.float16 if self.meas_f16 else torch.float32, "meas", self.device)
        ws = torch.empty(int(self.lib.ptyx_pacbed_ws_bytes(self.dims.N, nb)) // 8 + 1, dtype=torch.float64,
                         device=self.device)
        dLdI = torch.empty_like(dp) if want_dldi else None
        _lib.check(self.lib.ptyx_loss_pacbed(self._stream(), _ptr(dp), _ptr(meas), int(self.meas_f16), _ptr(idx_t),
                                             _ptr(off_t), nb, n, self.dims.N, float(loss_cfg.pacbed_w),
                                             float(loss_cfg.pacbed_q), float(grad_scale), _ptr(loss_terms),
                                             _ptr(dLdI), _ptr(ws)))
        return dLdI

    @property
    def call_capacity(self) -> int:
        """Patterns one ptyx_forward_loss_grad call takes without being split: the register
        engines' capacity, within max_patterns (what a split-batch call must fit)."""
        cap = self.register_capacity
        return min(cap, int(self.dims.max_patterns)) if cap > 0 else int(self.dims.max_patterns)

    @property
    def register_capacity(self) -> int:
        """Patterns per call the register-resident engines take (0: none for this geometry)."""
        return int(self.lib.ptyx_plan_register_capacity(self._h))

    def _chunked(self, t, idx, off, cap, loss_cfg, grads, grad_scale, loss_terms, dp_out, max_batch, store=False):
        """Split a call at mini-batch boundaries into groups of <= cap patterns (each batch keeps
        its own normalisation; gradients accumulate across the group calls; with ``store`` the
        first piece overwrites the object gradient, PTYX_PREP_GRAD_STORE)."""
        nb = off.size - 1
        if loss_terms is None:
            loss_terms = torch.empty((nb, 5), dtype=torch.float32, device=self.device)
        idx_t = self._idx(idx)
        pieces, b0 = [], 0
        while b0 < nb:
            b1 = b0 + 1
            while b1 < nb and off[b1 + 1] - off[b0] <= cap:
                b1 += 1
            pieces.append((b0, b1))
            b0 = b1
        for i, (b0, b1) in enumerate(pieces):
            # the object / probe are prepared once for all the pieces; every piece but the last may
            # leave its probe-gradient reduction to the next (PTYX_PREP_DEFER_PROBE)
            prep = _lib.PTYX_PREP_FULL if i == 0 else _lib.PTYX_PREP_REUSE
            if i < len(pieces) - 1:
                prep |= _lib.PTYX_PREP_DEFER_PROBE
            if i == 0 and store:
                prep |= _lib.PTYX_PREP_GRAD_STORE
            sub_off = (off[b0:b1 + 1] - off[b0]).astype(np.int32)
            sub_idx = idx_t[int(off[b0]):int(off[b1])]
            sub_dp = None if dp_out is None else dp_out[int(off[b0]):int(off[b1])]
            self.forward_loss_grad(t, sub_idx, sub_off, loss_cfg, grads, grad_scale=grad_scale,
                                   loss_terms=loss_terms[b0:b1], dp_out=sub_dp, max_batch=max_batch, prep=prep,
                                   _rows_checked=True)
        return loss_terms

    def _split_call(self, t, idx, batch_offsets, loss_cfg, grads, grad_scale, loss_terms, dp_out, reduce,
                    slot_exchange=None):
        """ptyx_forward_loss_grad_begin → reduce(batch sums) → ptyx_forward_loss_grad_end
        (→ slot_exchange: the object gradient over every rank's patterns)."""
        idx_t = self._idx(idx)
        off_t = self._idx(batch_offsets)
        n, nb = int(idx_t.numel()), int(off_t.numel()) - 1
        cap = self.call_capacity
        if n > cap:   # (recon_step cuts split groups by DistContext.split_ranges, the same on every rank)
            raise ValueError(f"a split-batch call of {n} patterns exceeds the plan's capacity {cap}")
        if loss_terms is None:
            loss_terms = torch.empty((nb, 5), dtype=torch.float32, device=self.device)
        sums = torch.empty((nb, _lib.PTYX_BATCH_SUMS), dtype=torch.float64, device=self.device)
        inp, _keep = self._inputs(t["obja"], t["objp"], t["probe"], t["shifts"], t.get("H"), t["occu"],
                                  t["crop_pos"], t["meas"], t.get("tilts"), t.get("kvec"), t.get("dz", 0.0),
                                  t.get("meas_rows"))
        cfg = loss_cfg.to_c(grad_scale, 0, _lib.PTYX_PREP_CALL |
                            (_lib.PTYX_PREP_DEFER_GATHER if slot_exchange is not None else 0))
        g = self._grads(grads)
        if slot_exchange is not None:   # the slots go straight into this rank's exchange block
            self.set_slot_target(*slot_exchange.target(self))
        _lib.check(self.lib.ptyx_forward_loss_grad_begin(self._h, self._stream(), ctypes.byref(inp), _ptr(idx_t),
                                                         _ptr(off_t), nb, n, ctypes.byref(cfg), _ptr(dp_out),
                                                         ctypes.byref(g), _ptr(sums)))
        try:
            reduce(sums)
        finally:   # always close the call (the plan refuses other work while one is open)
            _lib.check(self.lib.ptyx_forward_loss_grad_end(self._h, self._stream(), _ptr(sums), _ptr(loss_terms)))
        if slot_exchange is not None:
            slot_exchange(self, t, grads, loss_cfg)
        return loss_terms

    # ------------------------------------------------------------------ slot exchange (ABI 208)
    @property
    def slot_floats(self) -> int:
        """Floats per pattern of the object-gradient slots this plan's split calls can export
        (ptyx_plan_slot_floats; 0: no slot exchange for this geometry)."""
        return int(self.lib.ptyx_plan_slot_floats(self._h))

    def slot_block_floats(self, cap: int) -> int:
        """Floats of one rank's slot-exchange block of ``cap`` patterns (slots, then table rows)."""
        return int(self.lib.ptyx_slot_block_floats(self._h, int(cap)))

    def set_slot_target(self, block, cap: int):
        """ptyx_plan_slot_target: the next deferring split call writes its slots into ``block``."""
        if block is not None:
            _need(block, torch.float32, "block", self.device)
            if block.numel() != self.slot_block_floats(cap):
                raise ValueError(f"block must hold slot_block_floats({cap}) floats")
        _lib.check(self.lib.ptyx_plan_slot_target(self._h, _ptr(block), int(cap)))

    def export_slots(self, cap: int, block, d_shifts=None, use_last=True):
        """ptyx_slots_export: this rank's block (slot_block_floats(cap) floats) from the last
        deferred split call; use_last False: padding rows only."""
        _need(block, torch.float32, "block", self.device)
        if block.numel() != self.slot_block_floats(cap):
            raise ValueError(f"block must hold slot_block_floats({cap}) floats")
        if d_shifts is not None:
            _need(d_shifts, torch.float32, "d_shifts", self.device)
        _lib.check(self.lib.ptyx_slots_export(self._h, self._stream(), int(bool(use_last)), int(cap), _ptr(block),
                                              _ptr(d_shifts)))

    def gather_slots(self, blocks, n_ranks: int, cap: int, rank: int, t: dict, grads: dict, sparse_n: int,
                     adam=False):
        """ptyx_obj_gather_slots: object gradient of every rank block's patterns (the all-gathered
        ``blocks``) into grads['obja'] / ['objp'], and the other ranks' position-gradient rows
        into grads['shifts'].  ``adam``: then the optimizer step set_adam registered
        (ptyx_obj_gather_slots_adam; every other gradient must be final)."""
        _need(blocks, torch.float32, "blocks", self.device)
        if blocks.numel() != n_ranks * self.slot_block_floats(cap):
            raise ValueError("blocks must hold n_ranks x slot_block_floats(cap) floats")
        g = {k: grads.get(k) for k in ("obja", "objp", "shifts")}
        for k, v in g.items():
            if v is not None:
                _need(v, torch.float32, f"grad {k}", self.device)
        fn = self.lib.ptyx_obj_gather_slots_adam if adam else self.lib.ptyx_obj_gather_slots
        _lib.check(fn(self._h, self._stream(), _ptr(blocks), int(n_ranks), int(cap), int(rank), _ptr(t["obja"]),
                      _ptr(t["objp"]), _ptr(g["obja"]), _ptr(g["objp"]), int(sparse_n), _ptr(g["shifts"])))

    def adjoint_dldi(self, t: dict, idx, dLdI, grads: dict, grad_scale: float = 1.0):
        """ptyx_adjoint_dldi: accumulate gradients for an external dL/d(dp)."""
        self._prev_errors()
        idx_t = self._idx(idx)
        n = int(idx_t.numel())
        _need(dLdI, torch.float32, "dLdI", self.device)
        inp, _keep = self._inputs(t["obja"], t["objp"], t["probe"], t["shifts"], t.get("H"), t["occu"],
                                  t["crop_pos"], None, t.get("tilts"), t.get("kvec"), t.get("dz", 0.0))
        g = self._grads(grads)
        step = max(1, int(self.dims.max_patterns))
        for a in range(0, n, step):   # pieces of max_patterns: the external-loss adjoint is per pattern
            b = min(n, a + step)
            _lib.check(self.lib.ptyx_adjoint_dldi(self._h, self._stream(), ctypes.byref(inp), _ptr(idx_t[a:b]),
                                                  b - a, _ptr(dLdI[a:b]), float(grad_scale), ctypes.byref(g)))


def batch_offsets(batches) -> np.ndarray:
    """[0, len(b0), len(b0)+len(b1), ...] for a list of index arrays (reference make_batches output)."""
    sizes = [len(b) for b in batches]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
