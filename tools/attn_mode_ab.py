"""GPU A/B of the attention forward forms at the decision step's shapes (kbench cases): per attention mode
(0 default, 4 row-split shift forward) the per-launch time of shift / SoftDot /
candidate attention and the module chain at B = 20 and 256, and the max difference of the outputs from
mode 0's. python tools/attn_mode_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import kbench, ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    outs = {}
    for mode in (0, 4):
        ops.attn_set_mode(mode)
        for B in (20, 256):
            feat = torch.rand(B, 36, 2176, device=dev, generator=torch.Generator(device=dev).manual_seed(B))
            q = torch.rand(B, 2176, device=dev, generator=torch.Generator(device=dev).manual_seed(B + 1)) * 0.05
            z = torch.rand(B, 5, device=dev, generator=torch.Generator(device=dev).manual_seed(B + 2))
            ctx = torch.rand(B, 80, 2048, device=dev, generator=torch.Generator(device=dev).manual_seed(B + 3))
            qi = torch.rand(B, 2048, device=dev, generator=torch.Generator(device=dev).manual_seed(B + 4)) * 0.05
            mask = torch.zeros(B, 80, dtype=torch.bool, device=dev)
            mask[:, 70:] = True
            o = [t.clone() for t in ops.shift_attn_fwd(q, feat, z)] + [t.clone() for t in ops.softdot_fwd(qi, ctx, mask)]
            torch.cuda.synchronize()
            if mode == 0:
                outs[B] = o
            diff = max((a - b).abs().max().item() for a, b in zip(o, outs[B]))
            res = {}
            for name, nb, fn in kbench._cases(B, dev):
                if name in ("shift_attn", "softdot", "cand_logit", "attn_modules", "step_chain"):
                    us = kbench._time_graph(fn)
                    res[name] = round(us, 2)
            print(f"mode {mode} B={B}: {res}  max|diff| vs mode 0 {diff:.2e}", flush=True)
    ops.attn_set_mode(0)
    del g


if __name__ == "__main__":
    main()
