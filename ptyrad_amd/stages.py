"""Optional forward stages on the HIP path, as autograd-aware torch ops.

* detector blur  — ``PtychoAD.get_forward_meas`` (src/ptyrad/models.py:375-382):
                   ``dp = gaussian_blur(dp, kernel_size=5, sigma=detector_blur_std)``.
* object pre-blur — ``PtychoAD.get_obj_patches`` (src/ptyrad/models.py:267-284): every amplitude
                   and phase plane of every object patch is blurred on its own (reflect padding at
                   the PATCH edge, not the object edge), so the blurred patches are position-
                   specific and cannot be produced by blurring the object once.

``gaussian_blur`` is torchvision.transforms.functional.gaussian_blur (absent from this image): a
normalised 1-D kernel exp(-x²/2σ²) on linspace(-(k-1)/2, (k-1)/2, k) in f32, applied as the
outer-product 2-D kernel with reflect padding of k//2.  Forward: ``ptyx_obj_rblur``; backward:
``ptyx_blur_adjoint`` (its exact transpose).  Patches: ``ptyx_patch_gather`` /
``ptyx_patch_scatter_add``.  Everything runs in libptyx.so; there is no torch fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

KERNEL_SIZE = 5          # models.py:281, :380
MAX_PLANES = 65535       # grid limit of the blur / patch kernels per call


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _check_f32(t, name):
    if t.dtype != torch.float32 or t.device.type != "cuda" or not t.is_contiguous():
        raise TypeError(f"{name}: expected a contiguous float32 HIP tensor")


def blur_planes(x: torch.Tensor, sigma: float, kernel_size: int = KERNEL_SIZE, adjoint: bool = False):
    """gaussian_blur over the last two axes of ``x`` (or its transpose when ``adjoint``)."""
    _check_f32(x, "blur input")
    lib = _lib.load()
    Ny, Nx = x.shape[-2:]
    flat = x.reshape(-1, Ny, Nx)
    out = torch.empty_like(flat)
    fn = lib.ptyx_blur_adjoint if adjoint else lib.ptyx_obj_rblur
    st = _stream(x.device)
    for a in range(0, flat.shape[0], MAX_PLANES):
        b = min(flat.shape[0], a + MAX_PLANES)
        _lib.check(fn(st, _ptr(flat[a:b]), _ptr(out[a:b]), b - a, Ny, Nx, int(kernel_size), float(sigma)))
    return out.reshape(x.shape)


class GaussianBlur(torch.autograd.Function):
    """dp ↦ gaussian_blur(dp, 5, σ) (models.py:379-380); backward = the exact transpose."""

    @staticmethod
    def forward(ctx, x, sigma):
        ctx.sigma = sigma
        return blur_planes(x.contiguous(), sigma)

    @staticmethod
    def backward(ctx, g):
        return blur_planes(g.contiguous().float(), ctx.sigma, adjoint=True), None


def _patch_call(fn, a, O, Nz, Ny, Nx, crop_pos, idx_t, N, out):
    lib = _lib.load()
    st = _stream(a.device)
    n = int(idx_t.numel())
    _lib.check(getattr(lib, fn)(st, _ptr(a), O, Nz, Ny, Nx, _ptr(crop_pos), _ptr(idx_t), n, N, _ptr(out)))


def patch_gather(obj: torch.Tensor, crop_pos: torch.Tensor, idx_t: torch.Tensor, N: int) -> torch.Tensor:
    """(O,Nz,Ny,Nx) → (O,Nz,B,N,N) patches at crop_pos[idx] (get_obj_ROI, models.py:251-265)."""
    _check_f32(obj, "object")
    O, Nz, Ny, Nx = obj.shape
    B = int(idx_t.numel())
    if B > MAX_PLANES:
        raise ValueError(f"patch_gather: at most {MAX_PLANES} patches per call")
    out = torch.empty((O, Nz, B, N, N), dtype=torch.float32, device=obj.device)
    if B:
        _patch_call("ptyx_patch_gather", obj, O, Nz, Ny, Nx, crop_pos, idx_t, N, out)
    return out


def patch_scatter_add(gpatch: torch.Tensor, crop_pos: torch.Tensor, idx_t: torch.Tensor, gobj: torch.Tensor):
    """gobj += transpose of patch_gather (f32 atomics)."""
    _check_f32(gpatch, "patch gradient")
    _check_f32(gobj, "object gradient")
    O, Nz, Ny, Nx = gobj.shape
    N = gpatch.shape[-1]
    if int(idx_t.numel()):
        _patch_call("ptyx_patch_scatter_add", gpatch, O, Nz, Ny, Nx, crop_pos, idx_t, N, gobj)
    return gobj


class BlurredPatches(torch.autograd.Function):
    """get_obj_patches for one of obja / objp: gather + per-patch gaussian_blur (models.py:267-284).

    Returns (O, Nz, B, N, N) — the patch stack that the engine takes as an (O, Nz, B·N, N) object
    with crop_pos (b·N, 0).  ``sigma`` None / 0 gives the plain gather.
    """

    @staticmethod
    def forward(ctx, obj, crop_pos, idx_t, N, sigma):
        ctx.save_for_backward(crop_pos, idx_t)
        ctx.sigma, ctx.obj_shape = sigma, obj.shape
        p = patch_gather(obj.detach().contiguous(), crop_pos, idx_t, N)
        return blur_planes(p, sigma) if sigma else p

    @staticmethod
    def backward(ctx, g):
        crop_pos, idx_t = ctx.saved_tensors
        g = g.contiguous().float()
        if ctx.sigma:
            g = blur_planes(g, ctx.sigma, adjoint=True)
        gobj = torch.zeros(ctx.obj_shape, dtype=torch.float32, device=g.device)
        patch_scatter_add(g, crop_pos, idx_t, gobj)
        return gobj, None, None, None, None


class SimlarStd(torch.autograd.Function):
    """loss_simlar's core (losses.py:106-141): x (O, Q, …) one type's patches (modes first), occ
    (O) → (Q,) per-plane sums of torch.std(occ·x, dim=0) (unbiased) by ptyx_simlar_std; backward
    ptyx_simlar_std_grad."""

    @staticmethod
    def forward(ctx, x, occ):
        x = x.contiguous()
        _check_f32(x, "simlar patches")
        occ = occ.detach().to(x.device, torch.float32).contiguous()
        O, Q = int(x.shape[0]), int(x.shape[1])
        P = int(x[0, 0].numel()) if Q else 0
        sums = torch.empty(Q, dtype=torch.float32, device=x.device)
        _lib.check(_lib.load().ptyx_simlar_std(_stream(x.device), _ptr(x), O, Q, P, _ptr(occ), _ptr(sums)))
        ctx.save_for_backward(x, occ)
        return sums

    @staticmethod
    def backward(ctx, g):
        x, occ = ctx.saved_tensors
        O, Q = int(x.shape[0]), int(x.shape[1])
        P = int(x[0, 0].numel()) if Q else 0
        g = g.contiguous().float()
        gx = torch.empty_like(x)
        _lib.check(_lib.load().ptyx_simlar_std_grad(_stream(x.device), _ptr(x), O, Q, P, _ptr(occ), _ptr(g), _ptr(gx)))
        return gx, None


def stack_crop_pos(B: int, N: int, device) -> torch.Tensor:
    """crop_pos of a (.., B·N, N) patch-stack object: patch b starts at row b·N."""
    cp = torch.zeros((B, 2), dtype=torch.int32, device=device)
    cp[:, 0] = torch.arange(B, dtype=torch.int32, device=device) * N
    return cp


__all__ = ["GaussianBlur", "BlurredPatches", "SimlarStd", "blur_planes", "patch_gather", "patch_scatter_add",
           "stack_crop_pos", "KERNEL_SIZE"]
