"""Import the read-only PtyRAD reference (/root/reference/src) for fixture generation.

Used ONLY by tests/golden/make_golden.py, in the build container (the reference
does not exist on the GPU box).  Four optional packages that the reference
imports at module top level are absent from this image (torchvision, h5py,
tifffile, optuna); none of them is called on the hot path with blur options
off and no file I/O, so they are replaced by inert stubs that
raise if anything actually calls into them.
"""
import os
import sys
import types

REF_SRC = "/root/reference/src"


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def _raiser(what):
    def f(*a, **k):
        raise RuntimeError(f"{what} is stubbed out for fixture generation")
    return f


def tv_gaussian_blur(img, kernel_size, sigma):
    """torchvision.transforms.functional.gaussian_blur restated from its published algorithm
    (torchvision is absent here): f32 1-D kernel exp(-x²/2σ²) on linspace(-(k-1)/2, (k-1)/2, k),
    normalised; 2-D kernel = outer product; reflect padding k//2; per-plane conv2d.  Installed
    into ptyrad.models only for the blur fixtures (make_golden.py --blur-only)."""
    import torch
    import torch.nn.functional as F
    ks = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
    s = float(sigma if not isinstance(sigma, (list, tuple)) else sigma[0])
    half = (ks - 1) * 0.5
    x = torch.linspace(-half, half, ks, dtype=img.dtype, device=img.device)
    pdf = torch.exp(-0.5 * (x / s).pow(2))
    k1 = pdf / pdf.sum()
    k2 = torch.mm(k1[:, None], k1[None, :])
    shape = img.shape
    y = F.pad(img.reshape(-1, 1, shape[-2], shape[-1]), [ks // 2] * 4, mode="reflect")
    return F.conv2d(y, k2[None, None]).reshape(shape)


def import_reference():
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    if "torchvision" not in sys.modules:
        tv = _stub("torchvision")
        tr = _stub("torchvision.transforms")
        fn = _stub("torchvision.transforms.functional", gaussian_blur=_raiser("gaussian_blur"))
        tv.transforms = tr
        tr.functional = fn
    if "h5py" not in sys.modules:
        class _Placeholder:  # noqa: D401 - inert placeholder type
            def __init__(self, *a, **k):
                raise RuntimeError("h5py is stubbed out for fixture generation")
        _stub("h5py", File=_Placeholder, Group=_Placeholder, Dataset=_Placeholder)
    if "tifffile" not in sys.modules:
        _stub("tifffile", imread=None, imwrite=None)
    if "optuna" not in sys.modules:
        op = _stub("optuna")
        op.samplers = _stub("optuna.samplers")
        op.pruners = _stub("optuna.pruners")
        op.trial = _stub("optuna.trial", Trial=object)
        op.Trial = object
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    import ptyrad.models as models
    import ptyrad.losses as losses
    import ptyrad.reconstruction as reconstruction
    return models, losses, reconstruction
