"""CombinedLoss — drop-in for PtyRAD's ``CombinedLoss`` (src/ptyrad/losses.py:17-155).

``forward(model_DP, measured_DP, object_patches, omode_occu) -> (total, [5 terms])`` keeps the
reference signature and runs in torch on the engine's dp (generic path; the dp's backward runs
the HIP adjoint).  ``fused(model, batches)`` is the hot path: one ptyx_forward_loss_grad call
computes dp, the loss terms of every mini-batch and all gradients on the GPU, and returns a
loss tensor whose backward hands those gradients to autograd.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .engine import LOSS_TERM_NAMES, LossConfig, batch_offsets


def _engine_terms(plan, t, idx_t, off, cfg, grads, grad_scale, shift_probes, rows_checked=False):
    """One ptyx_forward_loss_grad call (plus the pacbed loss and its adjoint when on); gradients
    are accumulated (+=) into ``grads``, scaled by ``grad_scale``.  ``off``: host batch offsets
    (the Plan splits calls beyond its capacity at mini-batch boundaries).  rows_checked: the caller
    verified on the host that every position's DP is in the rank-local block (no device check)."""
    if cfg.pacbed_on:   # loss_pacbed (losses.py:77-89): HIP loss on the call's dp, then the HIP adjoint
        N = t["probe"].shape[1]
        dp = torch.empty((int(idx_t.numel()), N, N), dtype=torch.float32, device=t["obja"].device)
        terms = plan.forward_loss_grad(t, idx_t, off, cfg, grads, grad_scale=grad_scale, dp_out=dp,
                                       _rows_checked=rows_checked)
        dLdI = plan.loss_pacbed(t, idx_t, off, dp, cfg, terms, grad_scale=grad_scale, want_dldi=bool(grads))
        if grads:
            plan.adjoint_dldi(t, idx_t, dLdI, {k: v for k, v in grads.items() if k != "shifts" or shift_probes})
        return terms
    return plan.forward_loss_grad(t, idx_t, off, cfg, grads, grad_scale=grad_scale, _rows_checked=rows_checked)


class _FusedLoss(torch.autograd.Function):
    """Σ_m loss_m over mini-batches; backward = cached engine gradients × grad_output.

    ``plan`` / ``base`` name the geometry (the model's plan, or a pre-blur patch-stack plan)."""

    @staticmethod
    def forward(ctx, obja, objp, probe_rv, shifts, H_rv, tilts, dz_t, plan, base, idx_t, off_t, cfg, shift_probes):
        want = {"obja": obja.requires_grad, "objp": objp.requires_grad, "probe": probe_rv.requires_grad,
                "shifts": shifts.requires_grad and shift_probes, "H": H_rv.requires_grad,
                "tilts": tilts is not None and tilts.requires_grad, "dz": dz_t is not None and dz_t.requires_grad}
        grads = {}
        for k, p in (("obja", obja), ("objp", objp), ("probe", probe_rv), ("shifts", shifts), ("H", H_rv),
                     ("tilts", tilts), ("dz", dz_t)):
            if want[k]:
                grads[k] = torch.zeros_like(p)
        t = {"obja": obja.detach(), "objp": objp.detach(), "probe": probe_rv.detach(), "shifts": shifts.detach(),
             "H": H_rv.detach(), "tilts": None if tilts is None else tilts.detach().contiguous()}
        t.update(base)
        terms = _engine_terms(plan, t, idx_t, off_t, cfg, grads, 1.0, shift_probes)
        ctx.grads = grads
        total = terms.sum()
        ctx.mark_non_differentiable(terms)
        return total, terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        out = []
        for k in ("obja", "objp", "probe", "shifts", "H", "tilts", "dz"):
            g = ctx.grads.get(k)
            out.append(None if g is None else g * g_total)
        ctx.grads = None
        return (*out, None, None, None, None, None, None)


def model_stages(model_params=None, init_variables=None) -> bool:
    """Whether a PtychoHIP built from these constructor inputs runs an autograd stage (detector blur,
    object pre-blur, on-the-fly measurement padding / resampling: models.py:375-412) — the model
    attributes CombinedLoss._special reads, decided from the inputs alone."""
    mp = model_params or {}
    iv = init_variables or {}
    blur = any(mp.get(k) not in (None, 0) for k in ("detector_blur_std", "obj_preblur_std"))
    sf = iv.get("on_the_fly_meas_scale_factors")
    otf = iv.get("on_the_fly_meas_padded") is not None or (
        sf is not None and any(float(f) != 1 for f in np.asarray(sf).reshape(-1)))
    return bool(blur or otf)


class CombinedLoss(torch.nn.Module):
    """Same loss_params dict and call signature as the reference CombinedLoss."""

    def __init__(self, loss_params, device="cuda"):
        super().__init__()
        self.device = device
        self.loss_params = loss_params

    # ---------------------------------------------------------------- generic (torch) path
    def get_loss_single(self, model_DP, measured_DP):           # losses.py:36-50
        p = self.loss_params["loss_single"]
        if not p["state"]:
            return torch.tensor(0.0, device=model_DP.device)
        q = p.get("dp_pow", 0.5)
        mq = measured_DP.pow(q)
        return p["weight"] * torch.sqrt(torch.mean((model_DP.pow(q) - mq) ** 2)) / mq.mean()

    def get_loss_poissn(self, model_DP, measured_DP):           # losses.py:52-75
        p = self.loss_params["loss_poissn"]
        if not p["state"]:
            return torch.tensor(0.0, device=model_DP.device)
        q, eps = p.get("dp_pow", 1.0), p.get("eps", 1e-6)
        mq, iq = measured_DP.pow(q), model_DP.pow(q)
        return -p["weight"] * torch.mean(mq * torch.log(iq + eps) - iq) / mq.mean()

    def get_loss_pacbed(self, model_DP, measured_DP):           # losses.py:77-89
        p = self.loss_params["loss_pacbed"]
        if not p["state"]:
            return torch.tensor(0.0, device=model_DP.device)
        q = p.get("dp_pow", 0.2)
        d = model_DP.mean(0).pow(q) - measured_DP.mean(0).pow(q)
        return p["weight"] * torch.sqrt(torch.mean(d * d)) / measured_DP.pow(q).mean()

    def get_loss_sparse(self, objp_patches, omode_occu):        # losses.py:91-104
        p = self.loss_params["loss_sparse"]
        if not p["state"]:
            return torch.tensor(0.0, device=objp_patches.device)
        n = p["ln_order"]
        m = torch.mean(objp_patches.abs().pow(n), dim=(0, 2, 3, 4))
        return p["weight"] * (m.pow(1.0 / n) * omode_occu).sum()

    def get_loss_simlar(self, object_patches, omode_occu):      # losses.py:106-141
        """Std over object modes of the (blurred / resampled) patches; the blur is the HIP
        gaussian_blur of ptyrad_amd.stages (torchvision's kernel, reflect padding)."""
        p = self.loss_params.get("loss_simlar", {"state": False})
        if not p["state"]:
            return torch.tensor(0.0, device=object_patches.device)
        from .stages import GaussianBlur
        std, sf = p.get("blur_std"), p.get("scale_factor")
        total = torch.tensor(0.0, device=object_patches.device)
        for c, kinds in ((0, ("amplitude", "both")), (1, ("phase", "both"))):
            if p.get("obj_type", "both") not in kinds:
                continue
            x = object_patches[..., c]
            if std is not None and std != 0:
                x = GaussianBlur.apply(x.contiguous(), float(std))
            if sf is not None and any(f != 1 for f in sf):
                x = torch.nn.functional.interpolate(x, scale_factor=sf, mode="area")
            total = total + (x * omode_occu[:, None, None, None]).std(1).mean()
        return p["weight"] * total

    def forward(self, model_DP, measured_DP, object_patches, omode_occu):
        losses = [self.get_loss_single(model_DP, measured_DP),
                  self.get_loss_poissn(model_DP, measured_DP),
                  self.get_loss_pacbed(model_DP, measured_DP),
                  self.get_loss_sparse(object_patches[..., 1], omode_occu),
                  self.get_loss_simlar(object_patches, omode_occu)]
        return sum(losses), losses

    # ---------------------------------------------------------------- fused HIP path
    def fused(self, model, batches):
        """Forward + loss + adjoint of every mini-batch in ``batches`` in one engine call.

        Returns (Σ_m total_m as a differentiable scalar, terms (n_batches, 5) tensor).
        ``(loss / grad_accumulation).backward()`` then leaves exactly the reference's accumulated
        gradients (reconstruction.py:741-760) in ``.grad``.

        Optional stages (ptyrad_amd/stages.py): with ``obj_preblur_std`` the engine runs on the
        pre-blurred patch stack (groups of ≤ PREBLUR_GROUP patterns, split at mini-batch
        boundaries); with ``detector_blur_std`` the loss sees the blurred dp, so each mini-batch
        runs HIP forward → HIP blur → this module's loss terms → HIP adjoints.
        """
        flat = np.concatenate([np.asarray(b).reshape(-1) for b in batches])
        model._check_indices(flat)
        dev = model.opt_obja.device
        if getattr(model, "detector_blur", False) or (self._simlar_on() and self.simlar_per_batch):
            # the loss sees blurred intensities: HIP forward → HIP blur → loss terms of this module
            # → HIP adjoints, per mini-batch
            return self._per_batch(model, batches)
        if self._simlar_on():   # data terms on the engine (one call), loss_simlar beside it
            total, terms = self._data_loss().fused(model, batches)
            s_total, s_terms = self._simlar_terms(model, batches)
            terms = terms.clone()
            terms[:, 4] = s_terms
            return total + s_total, terms
        cfg = LossConfig.from_loss_params(self.loss_params)
        if getattr(model, "preblur", False):
            return self._preblur_fused(model, batches, cfg)
        if getattr(model, "otf_meas", False):
            return self._local_fused(model, batches, cfg)
        self._check_held(model, flat)
        idx_t = torch.as_tensor(flat, dtype=torch.int32).to(dev, non_blocking=True)
        off = batch_offsets(batches)   # host offsets: the Plan splits at mini-batch boundaries
        total, terms = _FusedLoss.apply(model.opt_obja, model.opt_objp, model.opt_probe,
                                        model.opt_probe_pos_shifts, model._H_rv(), model._tilts(), model._dz_t(),
                                        model.plan, model._base(), idx_t, off, cfg, model.shift_probes)
        return total, terms

    @staticmethod
    def _check_held(model, flat):
        held = getattr(model, "holds_measurements", None)
        if held is not None and not held(flat):
            raise IndexError("mini-batch positions outside this rank's measurement block (measurements_index)")

    def _special(self, model):
        return (getattr(model, "detector_blur", False) or getattr(model, "preblur", False) or
                getattr(model, "otf_meas", False) or self._simlar_on())

    def _simlar_on(self):
        return bool(self.loss_params.get("loss_simlar", {}).get("state", False))

    simlar_per_batch = False   # A/B: loss_simlar through the per-mini-batch generic path instead

    def _data_loss(self):
        """This loss without loss_simlar (the engine's terms; loss_simlar runs beside the call)."""
        lp = dict(self.loss_params)
        lp["loss_simlar"] = dict(lp.get("loss_simlar", {}), state=False)
        return CombinedLoss(lp, device=self.device)

    SIMLAR_PATCH_BYTES = 1 << 30   # patch-stack bytes per loss_simlar chunk (one type)

    def _simlar_terms(self, model, batches):
        """loss_simlar (losses.py:106-141) of every mini-batch of a call, vectorised over the call:
        the object patches of up to SIMLAR_PATCH_BYTES at a time by the HIP patch gather (and the
        HIP gaussian_blur, kernel 5, reflect padding; pre-blurred first when obj_preblur_std is on),
        torch's 'area' interpolation when scale_factor ≠ 1, the occupancy-weighted std over the
        object modes, each pattern's sum of it.  Mini-batch m's term is w·Σ_type Σ_{j∈m} S_j /
        (B_m·count) — the reference's mean over (B, Nz, Ny, Nx) of mini-batch m alone.  Returns
        (Σ_m term_m, differentiable — its backward is the blur adjoint and the HIP patch
        scatter-add into the object gradients —, the (n_batches,) detached terms)."""
        from .stages import MAX_PLANES, BlurredPatches, GaussianBlur, SimlarStd
        p = self.loss_params["loss_simlar"]
        dev = model.opt_obja.device
        O, Nz = int(model.opt_obja.shape[0]), int(model.opt_obja.shape[1])
        N = int(model.opt_probe.shape[1])
        sigma = p.get("blur_std")
        sigma = float(sigma) if sigma not in (None, 0) else None
        sf = p.get("scale_factor")
        resample = sf is not None and any(f != 1 for f in sf)
        types = [c for c, kinds in ((0, ("amplitude", "both")), (1, ("phase", "both")))
                 if p.get("obj_type", "both") in kinds]
        occ = model.omode_occu.to(dev, torch.float32)
        sizes = [len(np.asarray(b).reshape(-1)) for b in batches]
        bid = np.repeat(np.arange(len(batches)), sizes)
        flat = np.concatenate([np.asarray(b).reshape(-1) for b in batches]) if batches else np.zeros(0, np.int64)
        cap = max(1, min(MAX_PLANES, self.SIMLAR_PATCH_BYTES // (4 * O * Nz * N * N)))
        terms = torch.zeros(len(batches), dtype=torch.float64, device=dev)
        total = torch.zeros((), dtype=torch.float32, device=dev)
        for j0 in range(0, len(flat), cap):
            idx_t = torch.as_tensor(flat[j0:j0 + cap], dtype=torch.int32, device=dev)
            b_t = torch.as_tensor(bid[j0:j0 + cap], dtype=torch.long, device=dev)
            if getattr(model, "preblur", False):
                pre = model._blurred_patches(idx_t)
            for c in types:
                if getattr(model, "preblur", False):
                    x = pre[c]
                    if sigma:
                        x = GaussianBlur.apply(x.contiguous(), sigma)
                else:
                    obj = model.opt_obja if c == 0 else model.opt_objp
                    x = BlurredPatches.apply(obj, model.crop_pos, idx_t, N, sigma)   # (O, Nz, B, N, N)
                if resample:   # torch 'area' on (B, O, Nz, N, N), back to modes first
                    x = torch.nn.functional.interpolate(x.permute(2, 0, 1, 3, 4), scale_factor=list(sf), mode="area")
                    x = x.permute(1, 2, 0, 3, 4)
                nzr, B = int(x.shape[1]), int(x.shape[2])
                count = nzr * int(x.shape[3]) * int(x.shape[4])
                # the std over modes per pixel, summed per (slice, pattern) plane, on the device
                S = SimlarStd.apply(x.reshape(O, nzr * B, -1), occ).reshape(nzr, B).sum(0)   # per pattern
                w = torch.as_tensor(float(p["weight"]) / (np.asarray(sizes, np.float64)[bid[j0:j0 + cap]] * count),
                                    dtype=torch.float32, device=dev)
                total = total + (S * w).sum()
                terms.index_add_(0, b_t, (S.detach() * w).double())
        return total, terms.float()

    def supports_batch_split(self, model=None, *, model_params=None, init_variables=None) -> bool:
        """Whether ``fused_into(..., batch_sums_reduce=...)`` can take mini-batches split over ranks:
        every loss term must be a function of per-pattern additive sums (not loss_pacbed, whose
        mean pattern is a per-batch N² sum, nor the autograd stages).

        Before the model exists (a rank choosing which DPs to load, DistContext.local_indices) the
        stages are read from the constructor's ``model_params`` / ``init_variables`` instead, by
        the rules PtychoHIP applies, so the block and recon_step make the same decision."""
        if self.loss_params.get("loss_pacbed", {}).get("state", False):
            return False
        if model is not None:
            return not self._special(model)
        return not (self.loss_params.get("loss_simlar", {}).get("state", False) or
                    model_stages(model_params, init_variables))

    def fused_into(self, model, batches, grad_scale=1.0, batch_sums_reduce=None, slot_exchange=None):
        """The hot path without autograd: gradients of (Σ_m loss_m)·grad_scale are ACCUMULATED
        straight into the ``.grad`` tensors of the optimisable parameters the loss reaches
        (created, zeroed, when missing) — the engine writes them in place, no temporaries.
        Equivalent to ``(fused(model, batches)[0] * grad_scale).backward()``.  Returns the
        (n_batches, 5) loss terms.  Stages that need torch autograd (detector blur, pre-blur,
        on-the-fly measurements, loss_simlar) run exactly that way, into the same ``.grad``.

        batch_sums_reduce (data-parallel split of mini-batches, DistContext): ``batches[m]`` is this
        rank's part (possibly empty) of mini-batch m, the same number of parts on every rank;
        ``batch_sums_reduce(t)`` sums a float64 device tensor over the ranks in place.  The engine
        normalises every loss by its WHOLE mini-batch (ptyx_forward_loss_grad_begin / _end), so the
        ranks' gradients sum to the single-device gradient.  Rows of parts this rank does not hold
        are zero in the returned terms.

        slot_exchange (with batch_sums_reduce; reconstruction.SlotExchange): the object gradient of
        the split mini-batches is formed on every rank from every rank's per-pattern slots
        (all-gathered), and the position-gradient rows are exchanged likewise, instead of being
        left for an all-reduce of the whole object."""
        names = model.engine_grad_names()
        for k in names:
            p = model.optimizable_tensors[k]
            if p.requires_grad and p.grad is None:
                p.grad = torch.zeros_like(p)
        special = self._special(model)
        if batch_sums_reduce is not None:
            if not self.supports_batch_split(model):
                raise NotImplementedError("mini-batches split over ranks need additive loss terms "
                                          "(no loss_pacbed / loss_simlar / blur / on-the-fly stages)")
            return self._split_into(model, batches, grad_scale, batch_sums_reduce, slot_exchange)
        if slot_exchange is not None:
            raise ValueError("slot_exchange needs split mini-batches (batch_sums_reduce)")
        if special and self._simlar_on() and not getattr(model, "detector_blur", False) and not self.simlar_per_batch:
            # the data terms as without loss_simlar (one engine call), loss_simlar beside it
            terms = self._data_loss().fused_into(model, batches, grad_scale)
            s_total, s_terms = self._simlar_terms(model, batches)
            if s_total.requires_grad:
                torch.autograd.backward(s_total * grad_scale)
            terms[:, 4] = s_terms
            return terms
        if special:
            total, terms = self.fused(model, batches)
            if total.requires_grad:
                torch.autograd.backward(total * grad_scale)
            return terms
        flat = np.concatenate([np.asarray(b).reshape(-1) for b in batches])
        model._check_indices(flat)
        self._check_held(model, flat)
        cfg = LossConfig.from_loss_params(self.loss_params)
        dev = model.opt_obja.device
        idx_t = torch.as_tensor(flat, dtype=torch.int32).to(dev, non_blocking=True)
        H_rv = model._H_rv()
        tilts, dz_t = model._tilts(), model._dz_t()
        t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
             "shifts": model.opt_probe_pos_shifts.detach(), "H": H_rv.detach(),
             "tilts": None if tilts is None else tilts.detach().contiguous()}
        t.update(model._base())
        live = lambda p: p is not None and p.requires_grad and p.grad is not None  # noqa: E731
        grads = {}
        for k, p in (("obja", model.opt_obja), ("objp", model.opt_objp), ("probe", model.opt_probe),
                     ("tilts", tilts), ("dz", dz_t)):
            if live(p):
                grads[k] = p.grad
        if model.shift_probes and live(model.opt_probe_pos_shifts):
            grads["shifts"] = model.opt_probe_pos_shifts.grad
        if H_rv.requires_grad:          # optimised dz / tilts: dL/dH, then autograd through H(dz, tilts)
            grads["H"] = torch.zeros_like(H_rv)
        terms = _engine_terms(model.plan, t, idx_t, batch_offsets(batches), cfg, grads, float(grad_scale),
                              model.shift_probes, rows_checked=True)    # _check_held above
        if "H" in grads:
            torch.autograd.backward(H_rv, grads["H"])
        return terms

    def slot_exchange_ok(self, model):
        """Whether a split step of this loss on this model can exchange per-pattern object-gradient
        slots (reconstruction.SlotExchange): the register engines keep them (ptyx_plan_slot_floats)
        and the call is the plain fused one (no autograd stage, no optimised propagator, no
        per-position tilts)."""
        plan = getattr(model, "plan", None)
        return (plan is not None and plan.slot_floats > 0 and not self._special(model) and
                not getattr(model, "prop_opt", False) and model._dz_t() is None and model._tilts() is None and
                self.supports_batch_split(model))

    def _split_into(self, model, parts, grad_scale, reduce, slot_exchange=None):
        """fused_into for this rank's parts of mini-batches split over ranks."""
        from .engine import LossConfig as _LC
        dev = model.opt_obja.device
        G = len(parts)
        parts = [np.asarray(b).reshape(-1) for b in parts]
        held = [m for m, b in enumerate(parts) if b.size]
        terms = torch.zeros((G, 5), dtype=torch.float32, device=dev)
        H_rv = model._H_rv()
        if model._tilts() is not None:
            raise NotImplementedError("split mini-batches with per-position tilts are not supported")
        t = {"obja": model.opt_obja.detach(), "objp": model.opt_objp.detach(), "probe": model.opt_probe.detach(),
             "shifts": model.opt_probe_pos_shifts.detach(), "H": H_rv.detach(), "tilts": None}
        t.update(model._base())
        live = lambda p: p is not None and p.requires_grad and p.grad is not None  # noqa: E731
        grads = {k: p.grad for k, p in (("obja", model.opt_obja), ("objp", model.opt_objp),
                                         ("probe", model.opt_probe)) if live(p)}
        if model.shift_probes and live(model.opt_probe_pos_shifts):
            grads["shifts"] = model.opt_probe_pos_shifts.grad
        cfg = _LC.from_loss_params(self.loss_params)
        if not held:   # nothing here: still join the reduction of the group's sums (and the slot exchange)
            reduce(torch.zeros((G, _lib.PTYX_BATCH_SUMS), dtype=torch.float64, device=dev))
            if slot_exchange is not None:
                slot_exchange(model.plan, t, grads, cfg, used=False)
            return terms
        local = [parts[m] for m in held]
        flat = np.concatenate(local)
        model._check_indices(flat)
        self._check_held(model, flat)
        sel = torch.as_tensor(held, dtype=torch.long, device=dev)

        def group_reduce(sums):          # local rows -> the group's (G, PTYX_BATCH_SUMS) rows -> sum over ranks
            full = torch.zeros((G, sums.shape[1]), dtype=torch.float64, device=dev)
            full.index_copy_(0, sel, sums)
            reduce(full)
            sums.copy_(full.index_select(0, sel))

        idx_t = torch.as_tensor(flat, dtype=torch.int32).to(dev, non_blocking=True)
        if H_rv.requires_grad:          # optimised dz / tilts: this rank's share of dL/dH, then autograd
            grads["H"] = torch.zeros_like(H_rv)
        local_terms = model.plan.forward_loss_grad(t, idx_t, batch_offsets(local), cfg,
                                                   grads, grad_scale=float(grad_scale), batch_sums_reduce=group_reduce,
                                                   slot_exchange=slot_exchange, _rows_checked=True)   # _check_held above
        if "H" in grads:
            torch.autograd.backward(H_rv, grads["H"])
        terms.index_copy_(0, sel, local_terms)
        return terms

    PREBLUR_GROUP = 8192

    def _grouped(self, model, batches, cap, run, strict=False):
        """Split ``batches`` at mini-batch boundaries into groups of ≤ cap patterns (a larger
        mini-batch forms a group of its own unless ``strict``); ``run(group)`` returns
        (total, terms) of one engine call.  Gradients accumulate across the calls."""
        totals, rows, group, n = [], [], [], 0
        for b in batches:
            nb = len(np.asarray(b).reshape(-1))
            if strict and nb > cap:
                raise ValueError(f"a mini-batch of {nb} positions exceeds the call capacity {cap}")
            if group and n + nb > cap:
                t, r = run(group)
                totals.append(t)
                rows.append(r)
                group, n = [], 0
            group.append(b)
            n += nb
        if group:
            t, r = run(group)
            totals.append(t)
            rows.append(r)
        return sum(totals), torch.cat(rows)

    def _preblur_fused(self, model, batches, cfg):
        dev = model.opt_obja.device

        def run(group):
            flat = np.concatenate([np.asarray(b).reshape(-1) for b in group])
            idx_t = torch.as_tensor(flat, dtype=torch.int32).to(dev)
            off_t = torch.as_tensor(batch_offsets(group)).to(dev, non_blocking=True)
            A, Ph, sh, tl, plan, base, ar, _ = model._stack_inputs(idx_t, with_meas=True)
            return _FusedLoss.apply(A, Ph, model.opt_probe, sh, model._H_rv(), tl, model._dz_t(), plan, base, ar,
                                    off_t, cfg, model.shift_probes)

        return self._grouped(model, batches, self.PREBLUR_GROUP, run)

    def _local_fused(self, model, batches, cfg):
        """On-the-fly measurements: call-local positions / shifts / gathered DPs (models.py:384-412)."""
        dev = model.opt_obja.device

        def run(group):
            flat = np.concatenate([np.asarray(b).reshape(-1) for b in group])
            idx_t = torch.as_tensor(flat, dtype=torch.int32).to(dev)
            off_t = torch.as_tensor(batch_offsets(group)).to(dev, non_blocking=True)
            sh, tl, base, ar = model._local_inputs(idx_t, with_meas=True)
            return _FusedLoss.apply(model.opt_obja, model.opt_objp, model.opt_probe, sh, model._H_rv(), tl,
                                    model._dz_t(), model.plan, base, ar, off_t, cfg, model.shift_probes)

        return self._grouped(model, batches, int(model.plan.dims.n_scans), run, strict=True)

    def _per_batch(self, model, batches):
        totals, rows = [], []
        for b in batches:
            dp = model(b)
            total, terms = self.forward(dp, model.get_measurements(b), model._current_object_patches,
                                        model.omode_occu)
            totals.append(total)
            rows.append(torch.stack([torch.as_tensor(x, device=dp.device, dtype=torch.float32).detach().reshape(())
                                     for x in terms]))
        return sum(totals), torch.stack(rows)


__all__ = ["CombinedLoss", "LOSS_TERM_NAMES"]
