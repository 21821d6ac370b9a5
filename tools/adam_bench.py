"""Time one optimizer step of torch's fused Adam against ptyrad_amd.optim.Adam (ptyx_adam_step)
on the reconstruction's tensors at the c2 and c5 sizes (one param group per tensor, as the
reference builds them).  Prints one JSON line per (config, optimizer)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from ptyrad_amd import optim
    dev = torch.device("cuda", 0)
    sizes = {"c2": [(1, 1, 1033, 1033), (1, 1, 1033, 1033), (1, 128, 128, 2), (65536, 2)],
             "c5": [(1, 1, 14418, 14418), (1, 1, 14418, 14418), (4, 256, 256, 2), (16384, 2)]}
    lrs = [5e-4, 5e-4, 1e-4, 1e-4]
    for cfg, shapes in sizes.items():
        for name in ("torch_fused", "ptyx"):
            ps = [torch.zeros(s, device=dev) for s in shapes]
            for p in ps:
                p.grad = torch.randn_like(p)
            groups = [{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)]
            opt = torch.optim.Adam(groups, fused=True) if name == "torch_fused" else optim.Adam(groups)
            for _ in range(3):
                opt.step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                opt.step()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            n = sum(p.numel() for p in ps)
            print(json.dumps({"config": cfg, "optimizer": name, "elements": n, "ms_per_step": round(ms, 4),
                              "GBps": round(28 * n / ms / 1e6, 1)}), flush=True)
            del opt, ps
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
