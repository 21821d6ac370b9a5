"""Checkpoint / resume with PtyRAD's own key layout.

* ``make_save_dict`` mirrors ``save.py:85-137``. It has the same top-level keys,
  ``optimizable_tensors`` with the probe as a complex tensor, and the same
  ``model_attributes`` fields, and it works on a ``PtychoHIP`` or any object with the
  ``PtychoAD`` attribute contract.
* ``save_ptyrad(path, d)`` writes a ``.pt`` file. That is the container the reference's
  ``load_ptyrad`` (``load.py:495``) reads through ``load_pt`` (``:479``). numpy arrays become
  tensors, so this module can read the file back with ``torch.load(weights_only=True)``.
  The reference's preferred container, ``.hdf5`` (``save_dict_to_hdf5``, ``save.py:140-213``),
  needs h5py, which this image lacks. Asking for it raises ``NotImplementedError``.
* ``load_ptyrad(path)`` reads the file with ``weights_only=True``. ``resume(model, optimizer,
  ckpt)`` restores the optimizable tensors and, when saved, the optimizer state. A resumed
  reconstruction then continues as if it had never stopped.
"""
from __future__ import annotations

import os

import numpy as np
import torch

PTYRAD_FORMAT_VERSION = "0.1.0b9"   # the reference release whose layout this follows

MODEL_ATTRIBUTES = ("detector_blur_std", "obj_preblur_std", "start_iter", "lr_params", "omode_occu", "H",
                    "N_scan_slow", "N_scan_fast", "crop_pos", "slice_thickness", "dx", "dk", "scan_affine",
                    "tilt_obj", "shift_probes", "probe_int_sum")


def _portable(v):
    """numpy → torch, containers recursively; leaves str / numbers / None / tensors."""
    if isinstance(v, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(v))
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().clone()
    if isinstance(v, dict):
        return {k: _portable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        out = [_portable(x) for x in v]
        return out if isinstance(v, list) else tuple(out)
    return v


def make_save_dict(output_path, model, params, optimizer, niter, indices, batch_losses):
    """save.py:85-137: the dict PtyRAD saves per checkpoint, same keys and meanings."""
    if getattr(model, "_stale_object", False):
        raise RuntimeError("the band exchange left object rows out of date on this rank: call "
                           "DistContext.sync_object(model) on every rank before saving")
    avg_losses = {name: float(np.mean(values)) for name, values in batch_losses.items() if len(values)}
    avg_iter_t = float(np.mean(model.iter_times)) if len(model.iter_times) else float("nan")
    optimizable_tensors = {}
    for name, tensor in model.optimizable_tensors.items():
        optimizable_tensors[name] = tensor.detach().clone()
        if name == "probe":     # complex view, as the reference stores it
            optimizable_tensors["probe"] = torch.view_as_complex(model.opt_probe.detach().contiguous()).clone()
    save_opt = "optim_state" in ((params or {}).get("recon_params", {}).get("save_result") or [])
    return {
        "ptyrad_version": PTYRAD_FORMAT_VERSION,
        "output_path": output_path,
        "optimizable_tensors": optimizable_tensors,
        "optim_state_dict": optimizer.state_dict() if (save_opt and optimizer is not None) else None,
        "params": params,
        "model_attributes": {k: getattr(model, k, None) for k in MODEL_ATTRIBUTES},
        "loss_iters": model.loss_iters,
        "iter_times": model.iter_times,
        "dz_iters": model.dz_iters,
        "avg_iter_t": avg_iter_t,
        "niter": niter,
        "indices": indices,
        "batch_losses": batch_losses,
        "avg_losses": avg_losses,
    }


def save_ptyrad(path, save_dict):
    ext = os.path.splitext(path)[1].lower()
    if ext in (".h5", ".hdf5"):
        raise NotImplementedError("HDF5 checkpoints need h5py, which is absent; save as .pt (load_ptyrad reads it)")
    if ext != ".pt":
        raise ValueError(f"unsupported checkpoint extension '{ext}' (use .pt)")
    torch.save(_portable(save_dict), path)
    return path


def load_ptyrad(path):
    """Read a checkpoint written by save_ptyrad (tensors and plain containers only)."""
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    ext = os.path.splitext(path)[1].lower()
    if ext != ".pt":
        raise NotImplementedError(f"'{ext}' checkpoints are not readable here (HDF5 needs h5py)")
    return torch.load(path, map_location="cpu", weights_only=True)


def resume(model, optimizer, ckpt):
    """Restore the optimizable tensors (probe back to the real view) and the optimizer state."""
    with torch.no_grad():
        for name, t in ckpt["optimizable_tensors"].items():
            dst = model.optimizable_tensors[name]
            src = torch.view_as_real(t) if name == "probe" else t
            dst.copy_(src.to(device=dst.device, dtype=dst.dtype))
    if optimizer is not None and ckpt.get("optim_state_dict") is not None:
        optimizer.load_state_dict(ckpt["optim_state_dict"])
    for k in ("loss_iters", "iter_times", "dz_iters"):
        if ckpt.get(k) is not None and hasattr(model, k):
            setattr(model, k, list(ckpt[k]))
    return int(ckpt.get("niter") or 0)


__all__ = ["make_save_dict", "save_ptyrad", "load_ptyrad", "resume", "MODEL_ATTRIBUTES"]
