"""PtychoHIP — drop-in for PtyRAD's ``PtychoAD`` (src/ptyrad/models.py:30-436) on the HIP engine.

Same constructor (``init_variables``, ``model_params``, ``device``, ``verbose``), same
optimisable parameters (``opt_obja``, ``opt_objp``, ``opt_probe`` as a real view,
``opt_probe_pos_shifts``, ``opt_obj_tilts``, ``opt_slice_thickness``), buffers and bookkeeping
lists, so ``recon_step``, ``CombinedConstraint``, ``make_save_dict`` and the plotting code that
read a PtychoAD find what they expect.  The forward model and its gradients run in
``libptyx.so`` (include/ptyx.h); there is no torch fallback for them.

Two ways to get gradients:
* generic   — ``dp = model(indices)`` is differentiable: its backward runs ptyx_adjoint_dldi with
              whatever dL/d(dp) a downstream torch loss produced (any loss, incl. pacbed/simlar);
* fused     — ``ptyrad_amd.losses.CombinedLoss.fused(model, batches)`` runs forward + loss +
              adjoint in one engine call (ptyx_forward_loss_grad), the hot path.

Optional stages (ptyrad_amd/stages.py): detector blur (models.py:379-380) and
object pre-blur (:275-284) run as HIP kernels around the engine; pre-blurred patches are handed to
the engine as a patch-stack object (one (N, N) window per position, crop_pos (b·N, 0)).

Propagators (models.py:300-360): fixed H (case 4), fixed global tilt (2B), and optimised global
tilts / slice thickness (1, 2A, 3): H is rebuilt from the parameters on every call and the engine
returns dL/dH (PTYX_PROP_GRAD), which torch autograd carries to dz / tilts (an (N, N) expression).

On-the-fly measurement padding / resampling (models.py:384-412) runs as ptyx_meas_gather; engine
calls then take call-local positions / shifts / DPs (rows 0..n-1 of plan-sized arrays).

Per-position tilts (tilt_type 'each', models.py:330-356), fixed or optimised, also with an optimised slice thickness,
run in the engine (per-pattern separable ramps, d_tilts, d_dz).

Rank-local measurements (the data-parallel driver): ``init_variables["measurements"]``
may hold only the DPs of the scan positions listed in ``init_variables["measurements_index"]``
(``DistContext.local_indices(batches, grad_accumulation, loss_fn=..., model_params=...,
init_variables=...)``, which makes recon_step's split decision for this loss and model); the engine
reads them through a
scan-index → row map (ptyx_inputs.meas_rows), and any call on a position outside the block raises.
The reference registers the full stack on every rank (models.py:109).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from .engine import Plan
from .stages import BlurredPatches, GaussianBlur, stack_crop_pos

_PARAM_NAMES = ("obja", "objp", "obj_tilts", "slice_thickness", "probe", "probe_pos_shifts")


class _EngineForward(torch.autograd.Function):
    """dp = PtychoAD.forward(idx); backward = ptyx_adjoint_dldi (autograd of models.py:422-436).

    ``plan`` / ``base`` (occu, crop_pos, tilt grid) name the geometry: the model's own plan, or a
    patch-stack / call-local plan.  ``H_rv`` is the propagator (N,N,2) and ``tilts`` the
    per-position tilts (or None); their gradients come from the engine's d_H / d_tilts."""

    @staticmethod
    def forward(ctx, obja, objp, probe_rv, shifts, H_rv, tilts, dz_t, plan, base, idx_t, shift_probes):
        ctx.plan, ctx.base, ctx.shift_probes = plan, base, shift_probes
        ctx.save_for_backward(obja, objp, probe_rv, shifts, H_rv, tilts, dz_t, idx_t)
        with torch.no_grad():
            return plan.forward(_tensors(obja, objp, probe_rv, shifts, H_rv, tilts, base), idx_t)

    @staticmethod
    def backward(ctx, grad_dp):
        obja, objp, probe_rv, shifts, H_rv, tilts, dz_t, idx_t = ctx.saved_tensors
        want = ctx.needs_input_grad
        grads = {}
        outs = [None] * 7
        for i, (k, p) in enumerate((("obja", obja), ("objp", objp), ("probe", probe_rv), ("shifts", shifts),
                                    ("H", H_rv), ("tilts", tilts), ("dz", dz_t))):
            if want[i]:
                outs[i] = torch.zeros_like(p)
                grads[k] = outs[i]
        if not ctx.shift_probes:
            grads.pop("shifts", None)
        if grads:
            ctx.plan.adjoint_dldi(_tensors(obja, objp, probe_rv, shifts, H_rv, tilts, ctx.base), idx_t,
                                  grad_dp.contiguous().float(), grads)
        return (*outs, None, None, None, None)


def _tensors(obja, objp, probe_rv, shifts, H_rv, tilts, base):
    t = {"obja": obja.detach(), "objp": objp.detach(), "probe": probe_rv.detach(), "shifts": shifts.detach(),
         "H": H_rv.detach(), "tilts": None if tilts is None else tilts.detach().contiguous()}
    t.update(base)
    return t


class PtychoHIP(nn.Module):
    """Optimisable ptychography model whose forward/adjoint run on the MI355X engine."""

    def __init__(self, init_variables, model_params, device="cuda", verbose=True, max_patterns=None):
        super().__init__()
        with torch.no_grad():
            self.device = device
            self.verbose = verbose
            self.detector_blur_std = model_params.get("detector_blur_std")
            self.obj_preblur_std = model_params.get("obj_preblur_std")
            for k in ("detector_blur_std", "obj_preblur_std"):
                v = getattr(self, k)
                if v not in (None, 0) and not float(v) > 0:
                    raise ValueError(f"{k} must be None, 0 or > 0")
            self._stack_plans = {}
            # on-the-fly measurement padding / resampling (models.py:81-86, :384-412)
            pad = init_variables.get("on_the_fly_meas_padded")
            if pad is not None and not torch.is_tensor(pad):     # numpy (reference init) or a device
                pad = torch.tensor(np.asarray(pad))              # tensor (ptyrad_amd.ingest)
            self.meas_padded = None if pad is None else pad.to(device=device, dtype=torch.float32).contiguous()
            self.meas_padded_idx = None if pad is None else \
                torch.tensor(np.asarray(init_variables["on_the_fly_meas_padded_idx"]), dtype=torch.int32)
            sf = init_variables.get("on_the_fly_meas_scale_factors")
            self.meas_scale_factors = None if sf is None else [float(f) for f in np.asarray(sf).reshape(-1)]
            start_iter, lrs = {}, {}
            for k, p in model_params["update_params"].items():
                start_iter[k] = p["start_iter"]
                lrs[k] = p["lr"]
            self.optimizer_params = model_params.get("optimizer_params", {"name": "Adam", "configs": {}})
            self.start_iter = start_iter
            self.lr_params = lrs

            obj = np.asarray(init_variables["obj"])
            if "obja" in init_variables:          # exact amplitude / phase (fixtures, resume)
                obja = np.asarray(init_variables["obja"], np.float32)
                objp = np.asarray(init_variables["objp"], np.float32)
            else:                                  # models.py:99-100 (abs / angle of complex64)
                o = torch.tensor(obj.astype(np.complex64))
                obja, objp = o.abs().numpy(), o.angle().numpy()
            self.opt_obja = nn.Parameter(torch.tensor(obja, dtype=torch.float32, device=device))
            self.opt_objp = nn.Parameter(torch.tensor(objp, dtype=torch.float32, device=device))
            self.opt_obj_tilts = nn.Parameter(torch.tensor(np.asarray(init_variables.get("obj_tilts", [[0.0, 0.0]])),
                                                           dtype=torch.float32, device=device))
            self.opt_slice_thickness = nn.Parameter(torch.tensor(init_variables.get("slice_thickness", 1.0),
                                                                 dtype=torch.float32, device=device))
            probe = torch.tensor(np.asarray(init_variables["probe"]).astype(np.complex64), device=device)
            self.opt_probe = nn.Parameter(torch.view_as_real(probe).contiguous())
            self.opt_probe_pos_shifts = nn.Parameter(torch.tensor(np.asarray(init_variables["probe_pos_shifts"]),
                                                                  dtype=torch.float32, device=device))
            self.register_buffer("omode_occu", torch.tensor(np.asarray(init_variables["omode_occu"]),
                                                            dtype=torch.float32, device=device))
            self.register_buffer("H", torch.tensor(np.asarray(init_variables["H"]).astype(np.complex64), device=device))
            meas = init_variables.get("measurements")
            if isinstance(meas, torch.Tensor):   # e.g. ptyrad_amd.ingest output, already on the device
                meas_dtype = torch.float16 if meas.dtype == torch.float16 else torch.float32
                meas_t = meas.to(device=device, dtype=meas_dtype).contiguous()
            else:
                meas_dtype = torch.float16 if (meas is not None and np.asarray(meas).dtype == np.float16) \
                    else torch.float32
                meas_t = None if meas is None else torch.as_tensor(np.asarray(meas)).to(device=device,
                                                                                        dtype=meas_dtype)
            self.register_buffer("measurements", meas_t)
            for k, dt in (("N_scan_slow", torch.int32), ("N_scan_fast", torch.int32)):
                self.register_buffer(k, torch.tensor(init_variables.get(k, 0), dtype=dt, device=device))
            self.register_buffer("crop_pos", torch.tensor(np.asarray(init_variables["crop_pos"]), dtype=torch.int32,
                                                          device=device))
            # rank-local measurement block: row r of `measurements` is scan position meas_index[r]
            mi = init_variables.get("measurements_index")
            self.meas_index = None if mi is None else np.asarray(mi, dtype=np.int64).reshape(-1)
            self.meas_rows = None
            self._meas_rows_np = None
            if self.meas_index is not None:
                n_sc = int(self.crop_pos.shape[0])
                if meas_t is None or meas_t.shape[0] != self.meas_index.size:
                    raise ValueError("measurements_index must list one scan index per measurement row")
                if self.meas_index.size and (self.meas_index.min() < 0 or self.meas_index.max() >= n_sc or
                                             np.unique(self.meas_index).size != self.meas_index.size):
                    raise ValueError("measurements_index must hold distinct scan indices in [0, N_scans)")
                rows = np.full(n_sc, -1, np.int32)
                rows[self.meas_index] = np.arange(self.meas_index.size, dtype=np.int32)
                self._meas_rows_np = rows
                self.meas_rows = torch.tensor(rows, device=device)
            for k in ("slice_thickness", "dx", "dk", "lambd"):
                self.register_buffer(k, torch.tensor(float(init_variables.get(k, 0.0)), dtype=torch.float32,
                                                     device=device))
            self.scan_affine = init_variables.get("scan_affine")
            self.tilt_obj = bool(self.lr_params.get("obj_tilts", 0) != 0 or torch.any(self.opt_obj_tilts))
            self.shift_probes = bool(self.lr_params.get("probe_pos_shifts", 0) != 0)   # models.py:120
            self.change_thickness = bool(self.lr_params.get("slice_thickness", 0) != 0)
            self.change_tilt = bool(self.lr_params.get("obj_tilts", 0) != 0)
            # per-position tilts (tilt_type 'each', models.py:330-356): the engine applies each
            # position's separable ramp exp(i dz (Ky tan θy + Kx tan θx)) to H itself
            self.pos_tilts = bool(self.tilt_obj and self.opt_obj_tilts.shape[0] != 1)
            # models.py:210-219 / :346-349 (case 2B, global): a fixed tilt only changes the one
            # propagator every position uses, so the engine takes the tilted H as its H
            self.register_buffer("H_eff", self._tilted_H() if (self.tilt_obj and not self.pos_tilts) else self.H)
            # cases 1 / 2A / 3 (models.py:339-356): H is rebuilt from the optimised dz / tilts on
            # every call and the engine returns dL/dH (PTYX_PROP_GRAD), which autograd carries on
            self.prop_opt = self.change_thickness or (self.tilt_obj and self.change_tilt)
            self._init_propagator_grid()
            self._dz = float(self.opt_slice_thickness.detach().cpu())
            self.probe_int_sum = self.get_complex_probe_view().abs().pow(2).sum()
            self.loss_iters, self.iter_times, self.dz_iters, self.avg_tilt_iters = [], [], [], []
            self._current_object_patches = None
            self.optimizable_tensors = {
                "obja": self.opt_obja, "objp": self.opt_objp, "obj_tilts": self.opt_obj_tilts,
                "slice_thickness": self.opt_slice_thickness, "probe": self.opt_probe,
                "probe_pos_shifts": self.opt_probe_pos_shifts}
            self.create_optimizable_params_dict(self.lr_params, verbose)
            self._validate_geometry()
            if self.pos_tilts and self.opt_obj_tilts.shape != (self.crop_pos.shape[0], 2):
                raise ValueError("per-position obj_tilts must be (N_scans, 2)")
            O, Nz, Ny, Nx = self.opt_obja.shape
            P, N = self.opt_probe.shape[0], self.opt_probe.shape[1]
            n_scans = self.crop_pos.shape[0]
            # plan workspace scales with the largest call (per-pattern intensities of mixed-state
            # calls are N² f32 each); larger calls are split at mini-batch boundaries by Plan
            self.meas_f16 = meas_dtype == torch.float16
            cap = max_patterns or min(n_scans, 65536)
            # with on-the-fly measurements every engine call is call-local: positions, shifts and
            # the gathered DPs of the call sit in rows 0..n-1 of (cap)-row arrays
            self.otf_meas = self.meas_padded is not None or (
                self.meas_scale_factors is not None and any(f != 1 for f in self.meas_scale_factors))
            if self.otf_meas:
                cap = min(cap, 65535)
                self._meas_buf = torch.zeros((cap, N, N), dtype=torch.float32, device=device)
            # the main plan (its workspace sized for `cap` patterns per call) is created on first use:
            # pre-blur models run on patch-stack plans only
            self._plan = None
            self._plan_args = (N, P, O, Nz, Ny, Nx, cap if self.otf_meas else n_scans, cap)

    @property
    def plan(self):
        if self._plan is None:
            self._plan = Plan(*self._plan_args, shift_probes=self.shift_probes,
                              meas_f16=self.meas_f16 and not self.otf_meas, device=self.opt_obja.device,
                              prop_grad=self.prop_opt)
        return self._plan

    # ------------------------------------------------------------------ reference API
    def get_complex_probe_view(self):
        return torch.view_as_complex(self.opt_probe)

    def create_optimizable_params_dict(self, lr_params, verbose=True):
        """models.py:187-208: requires_grad from lr, Adam param groups with per-tensor lr."""
        self.lr_params = lr_params
        self.optimizable_params = []
        for name, lr in lr_params.items():
            if name not in self.optimizable_tensors:
                raise ValueError(f"'{name}' is not a valid parameter name; choose from {list(_PARAM_NAMES)}")
            self.optimizable_tensors[name].requires_grad = (lr != 0)
            if lr != 0:
                self.optimizable_params.append({"params": [self.optimizable_tensors[name]], "lr": lr})

    def _validate_geometry(self):
        N = self.opt_probe.shape[1]
        Ny, Nx = self.opt_obja.shape[-2:]
        cp = self.crop_pos.detach().cpu().numpy()
        if cp.size and (cp.min() < 0 or cp[:, 0].max() > Ny - N or cp[:, 1].max() > Nx - N):
            raise ValueError("crop_pos places a probe window outside the object")

    def _check_indices(self, indices):
        idx = np.asarray(indices.cpu() if isinstance(indices, torch.Tensor) else indices).reshape(-1)
        if idx.size and (idx.min() < 0 or idx.max() >= self.crop_pos.shape[0]):
            raise IndexError("scan index out of range")
        return idx

    def holds_measurements(self, indices) -> bool:
        """True when this model's measurement block has the DPs of every scan index given."""
        idx = self._check_indices(indices)
        return self._meas_rows_np is None or bool(np.all(self._meas_rows_np[idx] >= 0))

    def _meas_row_index(self, idx_t):
        """Rows of `measurements` for scan indices idx_t (device int32); raises outside the block."""
        if self.meas_rows is None:
            return idx_t
        if not self.holds_measurements(idx_t):
            raise IndexError("a scan index outside this rank's measurement block (measurements_index)")
        return self.meas_rows[idx_t.long()].contiguous()

    def engine_grad_names(self):
        """Optimisable tensors the loss reaches (the reference's autograd leaves .grad None for the
        rest, e.g. slice_thickness with one slice: H is then unused, forward.py:60-63)."""
        Nz = int(self.opt_obja.shape[1])
        names = ["obja", "objp", "probe"]
        if self.shift_probes:
            names.append("probe_pos_shifts")
        if self.change_thickness and Nz > 1:
            names.append("slice_thickness")
        if self.tilt_obj and self.change_tilt and Nz > 1:
            names.append("obj_tilts")
        return names

    def _init_propagator_grid(self):
        """create_grids (models.py:163-171) + init_propagator_vars (:221-223): Ky, Kx on the
        half-bin-shifted, ifftshifted grid; Kz = sqrt(k² - Kx² - Ky²), k = 2π/λ (f32)."""
        N = self.opt_probe.shape[1]
        dev = self.H.device
        g = (torch.arange(-N // 2, N // 2, device=dev) + 0.5) / N
        k1 = torch.fft.ifftshift(2 * torch.pi * g / self.dx)
        Ky, Kx = torch.meshgrid(k1, k1, indexing="ij")
        self.register_buffer("propagator_grid", torch.stack([Ky, Kx], dim=0))
        k = 2 * torch.pi / self.lambd
        self.register_buffer("Kz", torch.sqrt(k ** 2 - Kx ** 2 - Ky ** 2))
        # Kz − k without the cancellation, fp64 from the f32 grid: the dz gradient's kernel (_dz_phase)
        q2, k64 = Kx.double() ** 2 + Ky.double() ** 2, float(k)
        self.register_buffer("Kz0", (-q2 / (k64 + torch.sqrt(k64 ** 2 - q2))).float())

    def _dz_phase(self, H, dz, extra=None):
        """H — the reference's value, exp(i dz Kz) (× the tilt ramps) in f32 — with the gradient in dz
        taken as Re Σ conj(g_H) i (Kz − k + extra) H instead of through exp(i dz Kz).  The constant
        part k of the phase is a global phase of every propagation, so the loss does not depend on
        it and its term Re Σ conj(g_H) i k H is exactly 0 — but in f32 (k ≈ 150 Å⁻¹, dz·k ≈ 300 rad)
        its rounding is ≈ 1e-3 of the gradient (the reference's own floor, tests/test_oracle_golden.py);
        dropping it leaves the same exact-arithmetic gradient without that noise (pinned to the fp64
        oracle in tests/test_gpu_propagator.py).  The value is H bit for bit (× exp(0) = 1)."""
        kern = self.Kz0 if extra is None else self.Kz0 + extra.detach()
        return H.detach() * torch.exp(1j * (dz - dz.detach()) * kern)

    def _propagator(self):
        """get_propagators (models.py:300-360) for a global tilt: the (N, N) complex64 H every
        position uses, differentiable in opt_slice_thickness / opt_obj_tilts when they are optimised."""
        if self.pos_tilts:   # the engine applies the per-position ramps; H is exp(i dz Kz) or the fixed H
            if not self.change_thickness:
                return self.H_eff
            dz = self.opt_slice_thickness
            return self._dz_phase(torch.exp(1j * dz.detach() * self.Kz), dz)
        if not self.prop_opt:
            return self.H_eff
        Ky, Kx = self.propagator_grid
        dz = self.opt_slice_thickness
        ty = self.opt_obj_tilts[:, 0, None, None] / 1e3
        tx = self.opt_obj_tilts[:, 1, None, None] / 1e3
        if self.tilt_obj and self.change_thickness:                       # case 1
            ramp = Ky * torch.tan(ty) + Kx * torch.tan(tx)
            d0 = dz.detach()
            H = torch.exp(1j * d0 * self.Kz) * torch.exp(1j * d0 * ramp)   # (the tilts' gradient: through ramp)
            H = self._dz_phase(H, dz, ramp) * torch.exp(1j * d0 * (ramp - ramp.detach()))
        elif self.tilt_obj:                                                # case 2A
            H = self.H * torch.exp(1j * dz * (Ky * torch.tan(ty) + Kx * torch.tan(tx)))
        else:                                                              # case 3
            H = self._dz_phase(torch.exp(1j * dz.detach() * self.Kz), dz)[None]
        return H[0]

    def _H_rv(self):
        return torch.view_as_real(self._propagator().contiguous())

    def _tilted_H(self):
        """H · exp(i dz (Ky tan θy + Kx tan θx)) on the half-bin-shifted, ifftshifted k grid
        (models.py:163-171 create_grids, :215-219 init_propagator_vars)."""
        N = self.opt_probe.shape[1]
        dev = self.H.device
        g = (torch.arange(-N // 2, N // 2, device=dev) + 0.5) / N
        k = torch.fft.ifftshift(2 * torch.pi * g / self.dx)
        Ky, Kx = torch.meshgrid(k, k, indexing="ij")
        dz = self.opt_slice_thickness.detach()
        ty = self.opt_obj_tilts[:, 0, None, None] / 1e3
        tx = self.opt_obj_tilts[:, 1, None, None] / 1e3
        return (self.H * torch.exp(1j * dz * (Ky * torch.tan(ty) + Kx * torch.tan(tx))))[0].contiguous()

    def _engine_tensors(self):
        return _tensors(self.opt_obja, self.opt_objp, self.opt_probe, self.opt_probe_pos_shifts, self._H_rv(),
                        self._tilts(), self._base())

    def _base(self, crop_pos=None, meas=None, stack=False):
        b = {"occu": self.omode_occu, "crop_pos": self.crop_pos if crop_pos is None else crop_pos,
             "meas": self.measurements if (meas is None and not stack) else meas}
        if self.meas_rows is not None and meas is None and not stack:
            b["meas_rows"] = self.meas_rows
        if self.pos_tilts:   # the ramps use the current dz (a host value: one sync per call if optimised)
            dz = float(self.opt_slice_thickness.detach()) if self.change_thickness else self._dz
            b.update(kvec=self.propagator_grid[0][:, 0].contiguous(), dz=dz)
        return b

    def _dz_t(self):
        """opt_slice_thickness as an engine input when its gradient runs through the tilt ramps."""
        return self.opt_slice_thickness if (self.pos_tilts and self.change_thickness) else None

    def _tilts(self, il=None, pad_to=None):
        """Per-position tilts for an engine call: all positions, or rows ``il`` (call-local /
        patch-stack calls, zero-padded to ``pad_to`` rows); None without per-position tilts."""
        if not self.pos_tilts:
            return None
        if il is None:
            return self.opt_obj_tilts
        t = self.opt_obj_tilts[il]
        if pad_to is not None and pad_to > t.shape[0]:
            t = torch.cat([t, t.new_zeros((pad_to - t.shape[0], 2))])
        return t

    # ------------------------------------------------------------------ object pre-blur (stages.py)
    @property
    def preblur(self):
        return self.obj_preblur_std not in (None, 0)

    @property
    def detector_blur(self):
        return self.detector_blur_std not in (None, 0)

    @staticmethod
    def _stack_capacity(B):
        """Patch-stack plans come in power-of-two capacities (≥ 32), so the k / k+1 mini-batch
        sizes of array_split, grad_accumulation groups and the last group share one plan."""
        return max(32, 1 << (int(B) - 1).bit_length())

    def _stack_plan(self, C):
        """Plan for a (O, Nz, C·N, N) patch-stack object (pre-blurred patches, capacity C)."""
        plan = self._stack_plans.get(C)
        if plan is None:
            if len(self._stack_plans) >= 4:
                # drop the oldest; an autograd graph that still holds it keeps it alive (Plan.__del__)
                self._stack_plans.pop(next(iter(self._stack_plans)))
            O, Nz = self.opt_obja.shape[:2]
            P, N = self.opt_probe.shape[:2]
            plan = Plan(N, P, O, Nz, C * N, N, C, C, shift_probes=self.shift_probes,
                        meas_f16=self.meas_f16 and not self.otf_meas, device=self.opt_obja.device,
                        prop_grad=self.prop_opt)
            self._stack_plans[C] = plan
        return plan

    def _blurred_patches(self, idx_t):
        """(O,Nz,B,N,N) pre-blurred amplitude and phase patches (models.py:267-284), differentiable."""
        N = self.opt_probe.shape[1]
        std = float(self.obj_preblur_std)
        return (BlurredPatches.apply(self.opt_obja, self.crop_pos, idx_t, N, std),
                BlurredPatches.apply(self.opt_objp, self.crop_pos, idx_t, N, std))

    def _stack_inputs(self, idx_t, with_meas=False):
        """Engine inputs on the patch stack: (obja, objp, shifts, plan, base, idx, patches).

        The stack is zero-padded to the plan capacity C; the engine runs on patterns 0..B-1 only."""
        B = int(idx_t.numel())
        C = self._stack_capacity(B)
        N = self.opt_probe.shape[1]
        A, Ph = self._blurred_patches(idx_t)
        O, Nz = A.shape[:2]
        il = idx_t.long()
        pad = C - B
        sh = self.opt_probe_pos_shifts[il]
        if pad:
            sh = torch.cat([sh, sh.new_zeros((pad, 2))])
            Ap = torch.nn.functional.pad(A, (0, 0, 0, 0, 0, pad))
            Php = torch.nn.functional.pad(Ph, (0, 0, 0, 0, 0, pad))
        else:
            Ap, Php = A, Ph
        meas = None
        if with_meas:
            meas = self._gather_meas(idx_t) if self.otf_meas else \
                self.measurements[self._meas_row_index(idx_t).long()].contiguous()
            if pad:
                meas = torch.cat([meas, meas.new_zeros((pad, N, N))])
        base = self._base(stack_crop_pos(C, N, idx_t.device), meas, stack=True)
        ar = torch.arange(B, dtype=torch.int32, device=idx_t.device)
        return (Ap.reshape(O, Nz, C * N, N), Php.reshape(O, Nz, C * N, N), sh, self._tilts(il, C),
                self._stack_plan(C), base, ar, (A, Ph))

    def get_obj_patches(self, indices):
        """models.py:251-284: (B,O,Nz,N,N,2) amplitude/phase patches (pre-blurred when enabled)."""
        idx = self._check_indices(indices)
        if self.preblur:
            idx_t = torch.as_tensor(idx, dtype=torch.int32).to(self.opt_obja.device)
            A, Ph = self._blurred_patches(idx_t)
            return torch.stack([A, Ph], dim=-1).permute(2, 0, 1, 3, 4, 5)
        idx = torch.as_tensor(idx, device=self.opt_obja.device, dtype=torch.long)
        N = self.opt_probe.shape[1]
        r = torch.arange(N, device=self.opt_obja.device)
        cp = self.crop_pos[idx].long()
        gy = (cp[:, 0, None, None] + r[None, :, None]).expand(-1, N, N)
        gx = (cp[:, 1, None, None] + r[None, None, :]).expand(-1, N, N)
        a = self.opt_obja[:, :, gy, gx].permute(2, 0, 1, 3, 4)
        p = self.opt_objp[:, :, gy, gx].permute(2, 0, 1, 3, 4)
        return torch.stack([a, p], dim=-1)

    def get_probes(self, indices):
        """models.py:286-298 (torch restatement; not on the hot path)."""
        probe = self.get_complex_probe_view()
        idx = self._check_indices(indices)
        if not self.shift_probes:
            return torch.broadcast_to(probe, (len(idx), *probe.shape))
        N = probe.shape[-1]
        g = torch.remainder(torch.arange(N, device=probe.device) + N // 2, N).float() / N
        s = self.opt_probe_pos_shifts[torch.as_tensor(idx, device=probe.device)]
        w = torch.exp(-2j * torch.pi * (s[:, 0, None, None] * g[None, :, None] + s[:, 1, None, None] * g[None, None, :]))
        return torch.fft.ifft2(torch.fft.fft2(probe)[None] * w[:, None])

    def get_propagators(self, indices):
        """models.py:300-360: (1,N,N), or (B,N,N) with per-position tilts."""
        if self.pos_tilts:
            Ky, Kx = self.propagator_grid
            t = self.opt_obj_tilts[torch.as_tensor(self._check_indices(indices), device=Ky.device)] / 1e3
            ramp_arg = Ky * torch.tan(t[:, 0, None, None]) + Kx * torch.tan(t[:, 1, None, None])
            if self.change_thickness:            # case 1 (models.py:339-342): the current dz
                dz = self.opt_slice_thickness
                d0 = dz.detach()
                H = torch.exp(1j * d0 * self.Kz) * torch.exp(1j * d0 * ramp_arg)
                return self._dz_phase(H, dz, ramp_arg) * torch.exp(1j * d0 * (ramp_arg - ramp_arg.detach()))
            return self.H * torch.exp(1j * self._dz * ramp_arg)
        return self._propagator()[None,]

    def get_propagated_probe(self, index):
        probe = self.get_probes(index)[0].detach()
        H = self.get_propagators(index)[[0]].detach()
        n_slices = self.opt_objp.shape[1]
        out = torch.zeros((n_slices, *probe.shape), dtype=probe.dtype, device=probe.device)
        psi = probe
        for n in range(n_slices):
            out[n] = psi
            psi = torch.fft.ifft2(H[None] * torch.fft.fft2(psi))
        return out

    def _gather_meas(self, idx_t, out=None):
        """ptyx_meas_gather: the call's DPs with the on-the-fly padding / resampling applied."""
        from . import _lib
        n = int(idx_t.numel())
        Hm, Wm = self.measurements.shape[-2:]
        N = self.opt_probe.shape[1]
        if out is None:
            out = torch.empty((n, N, N), dtype=torch.float32, device=self.measurements.device)
        if self.meas_padded is not None:
            Hp, Wp = self.meas_padded.shape[-2:]
            h1, _, w1, _ = (int(v) for v in self.meas_padded_idx)
            canvas = ctypes.c_void_p(self.meas_padded.data_ptr())
        else:
            Hp, Wp, h1, w1, canvas = Hm, Wm, 0, 0, ctypes.c_void_p(0)
        sy, sx = self.meas_scale_factors if self.meas_scale_factors is not None else (1.0, 1.0)
        lib = _lib.load()
        idx_t = self._meas_row_index(idx_t)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.measurements.device).cuda_stream)
        _lib.check(lib.ptyx_meas_gather(st, ctypes.c_void_p(self.measurements.data_ptr()),
                                        int(self.measurements.dtype == torch.float16), Hm, Wm,
                                        ctypes.c_void_p(idx_t.data_ptr()), n, canvas, Hp, Wp, h1, w1, sy, sx, N, N,
                                        ctypes.c_void_p(out.data_ptr())))
        return out

    def _local_inputs(self, idx_t, with_meas=False):
        """Call-local engine inputs (on-the-fly measurements): shifts / crop_pos / DPs of the call's
        positions in rows 0..n-1 of plan-sized arrays; the engine then runs on idx = 0..n-1."""
        n, cap = int(idx_t.numel()), int(self.plan.dims.n_scans)
        if n > cap:
            raise ValueError(f"calls with on-the-fly measurements take at most {cap} positions")
        il = idx_t.long()
        sh, cp = self.opt_probe_pos_shifts[il], self.crop_pos[il]
        if n < cap:
            sh = torch.cat([sh, sh.new_zeros((cap - n, 2))])
            cp = torch.cat([cp, cp.new_zeros((cap - n, 2))])
        meas = None
        if with_meas:
            self._gather_meas(idx_t, self._meas_buf[:n])
            meas = self._meas_buf
        base = self._base(cp.contiguous(), meas, stack=True)
        return sh, self._tilts(il, cap), base, torch.arange(n, dtype=torch.int32, device=idx_t.device)

    def get_measurements(self, indices=None):
        """models.py:384-416, including the on-the-fly padding / resampling (HIP gather)."""
        if indices is None:
            return self.measurements
        idx = self._check_indices(indices)
        if self.otf_meas:
            return self._gather_meas(torch.as_tensor(idx, dtype=torch.int32).to(self.measurements.device))
        idx = torch.as_tensor(idx, device=self.measurements.device, dtype=torch.int32)
        return self.measurements[self._meas_row_index(idx).long()].float()

    def clear_cache(self):
        self._current_object_patches = None

    def forward(self, indices):
        """models.py:422-436: dp_fwd (B,N,N) f32 from the HIP engine, differentiable."""
        idx = self._check_indices(indices)
        idx_t = torch.as_tensor(idx, dtype=torch.int32).to(self.opt_obja.device, non_blocking=True)
        if self.preblur:
            A, Ph, sh, tl, plan, base, ar, (pa, pp) = self._stack_inputs(idx_t)
            dp = _EngineForward.apply(A, Ph, self.opt_probe, sh, self._H_rv(), tl, self._dz_t(), plan, base, ar,
                                      self.shift_probes)
            self._current_object_patches = torch.stack([pa, pp], dim=-1).permute(2, 0, 1, 3, 4, 5)
        elif self.otf_meas:
            sh, tl, base, ar = self._local_inputs(idx_t)
            dp = _EngineForward.apply(self.opt_obja, self.opt_objp, self.opt_probe, sh, self._H_rv(), tl,
                                      self._dz_t(), self.plan, base, ar, self.shift_probes)
            self._current_object_patches = self.get_obj_patches(idx)
        else:
            dp = _EngineForward.apply(self.opt_obja, self.opt_objp, self.opt_probe, self.opt_probe_pos_shifts,
                                      self._H_rv(), self._tilts(), self._dz_t(), self.plan,
                                      self._base(meas=None, stack=True), idx_t, self.shift_probes)
            # object patches for losses that use them (loss_sparse / loss_simlar, losses.py:152-153)
            self._current_object_patches = self.get_obj_patches(idx)
        if self.detector_blur:                      # get_forward_meas, models.py:375-382
            dp = GaussianBlur.apply(dp, float(self.detector_blur_std))
        return dp


PtychoAD = PtychoHIP   # name the reference's callers import
