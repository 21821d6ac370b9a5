"""Test doubles for the data-parallel driver on CPU (gloo): the oracle stands in for the engine.

The product path has no CPU fallback, so the multi-rank logic of ptyrad_amd.reconstruction
(round-robin deal of mini-batches, one flat all-reduce, identical optimizer steps) is exercised
with an oracle-backed ``fused`` loss and a plain torch parameter holder.
"""
import json
import os

import numpy as np
import torch

from oracle import ptyx_oracle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _OracleFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, obja, objp, probe_rv, shifts, model, batches, lp):
        probe = (probe_rv[..., 0] + 1j * probe_rv[..., 1]).detach().numpy()
        terms, _, g = orc.forward_loss_grad(
            obja.detach().numpy(), objp.detach().numpy(), probe, shifts.detach().numpy(), model.crop_pos_np,
            model.H_np, model.occu_np, model.meas_np, batches, lp, shift_probes=True)
        ctx.g = [torch.tensor(g["obja"], dtype=torch.float32), torch.tensor(g["objp"], dtype=torch.float32),
                 torch.tensor(np.stack([g["probe"].real, g["probe"].imag], -1), dtype=torch.float32),
                 torch.tensor(g["shifts"], dtype=torch.float32)]
        t = torch.tensor(terms, dtype=torch.float32)
        ctx.mark_non_differentiable(t)
        return t.sum(), t

    @staticmethod
    def backward(ctx, gt, _):
        return tuple(x * gt for x in ctx.g) + (None, None, None)


class OracleModel(torch.nn.Module):
    """Parameter holder with the PtychoAD attribute contract recon_step uses."""

    def __init__(self, z):
        super().__init__()
        self.opt_obja = torch.nn.Parameter(torch.tensor(z["init_obja"]))
        self.opt_objp = torch.nn.Parameter(torch.tensor(z["init_objp"]))
        p = z["init_probe"]
        self.opt_probe = torch.nn.Parameter(torch.tensor(np.stack([p.real, p.imag], -1).astype(np.float32)))
        self.opt_probe_pos_shifts = torch.nn.Parameter(torch.tensor(z["init_shifts"]))
        self.opt_obj_tilts = torch.nn.Parameter(torch.zeros(1, 2), requires_grad=False)
        self.opt_slice_thickness = torch.nn.Parameter(torch.tensor(1.0), requires_grad=False)
        self.crop_pos_np, self.H_np, self.occu_np, self.meas_np = z["crop_pos"], z["H"], z["occu"], z["meas"]
        lrs = json.loads(str(z["lrs"]))
        self.lr_params = lrs
        self.start_iter = {k: (1 if v else None) for k, v in lrs.items()}
        self.optimizable_tensors = {"obja": self.opt_obja, "objp": self.opt_objp, "obj_tilts": self.opt_obj_tilts,
                                    "slice_thickness": self.opt_slice_thickness, "probe": self.opt_probe,
                                    "probe_pos_shifts": self.opt_probe_pos_shifts}
        self.optimizable_params = [{"params": [self.optimizable_tensors[k]], "lr": v} for k, v in lrs.items() if v]
        self.loss_iters, self.iter_times, self.dz_iters, self.avg_tilt_iters = [], [], [], []

    def clear_cache(self):
        pass


class OracleLoss:
    def __init__(self, lp):
        self.loss_params = lp

    def fused(self, model, batches):
        return _OracleFused.apply(model.opt_obja, model.opt_objp, model.opt_probe, model.opt_probe_pos_shifts,
                                  model, batches, self.loss_params)


def run_recon(z, rank_world=None, niter=None):
    """Run the trajectory fixture through ptyrad_amd.reconstruction.recon_step; returns final params."""
    from ptyrad_amd.reconstruction import DistContext, recon_step
    model = OracleModel(z)
    lp = json.loads(str(z["loss_params"]))
    loss = OracleLoss(lp)
    opt = torch.optim.Adam(model.optimizable_params)
    sizes = z["batch_sizes"]
    batches = np.split(z["batches"], np.cumsum(sizes)[:-1])
    ctx = DistContext()
    cfn = None
    if "constraint_params" in z.files and json.loads(str(z["constraint_params"])) is not None:
        cp, pis = json.loads(str(z["constraint_params"])), float(z["probe_int_sum"])

        def cfn(m, it):   # the constraints oracle on the replica's parameters (every rank alike)
            from tests.test_oracle_golden import apply_constraint_oracle
            prm = {"obja": m.opt_obja.detach().numpy(), "objp": m.opt_objp.detach().numpy(),
                   "probe": m.opt_probe.detach().numpy()}
            apply_constraint_oracle(prm, cp, pis, it)
            with torch.no_grad():
                m.opt_obja.copy_(torch.from_numpy(prm["obja"]))
                m.opt_objp.copy_(torch.from_numpy(prm["objp"]))
                m.opt_probe.copy_(torch.from_numpy(prm["probe"]))
    for it in range(1, (niter or int(z["niter"])) + 1):
        recon_step(batches, int(z["grad_accumulation"]), model, opt, loss, cfn, it, verbose=False, dist_ctx=ctx)
    return {k: v.detach().numpy().copy() for k, v in (("obja", model.opt_obja), ("objp", model.opt_objp),
                                                       ("probe", model.opt_probe),
                                                       ("shifts", model.opt_probe_pos_shifts))}, model


def dist_worker(rank, world, port, path, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(path, allow_pickle=False)
        params, model = run_recon(z)
        if rank == 0:
            np.savez(out_path, losses=np.array([v for _, v in model.loss_iters]), **params)
        else:
            np.savez(out_path.replace(".npz", f"_r{rank}.npz"), **params)
    finally:
        torch.distributed.destroy_process_group()
