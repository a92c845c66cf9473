"""Phase clocks of the LDS-staged attention backward (where its ~25 us floor goes).
dasa_mha_bwd_stamps makes workgroup 0 record s_memtime (shader cycles) at the kernel's phase boundaries:
0 start, 1 dO / V / P staged (first global round trip + LDS stores), 2 dP = dO V^T, 3 row dots, 4 dS,
5 Q / K staged (second global round trip), 6 dV, 7 dQ, 8 dK stored. Median over 30 launches per shape, at the
finetune's B = 2, 12 heads, dropout 0.1, parts automatic.
    python tools/mha_bwd_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402

PHASES = ["stage dO/V/P", "dP", "rowdot", "dS", "stage Q/K", "dV", "dQ", "dK+drain"]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    buf = torch.zeros(16, dtype=torch.int64, device=dev)
    n = lib.dasa_mha_bwd_stamps(ctypes.c_void_p(buf.data_ptr()))
    B, h, scale, seed = 2, 12, 1 / 8.0, 5
    try:
        for Lq, Lk in ((80, 80), (80, 36), (36, 80), (36, 36)):
            Q, K, V, dO = (torch.randn(B, L_, 768, device=dev) for L_ in (Lq, Lk, Lk, Lq))
            m = torch.zeros(B, Lk, device=dev)
            _, probs = ops.mha(Q, K, V, m, h, scale, 0.1, seed, save_probs=True)
            recs, wall = [], []
            for _ in range(33):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.mha_bwd(Q, K, V, probs, dO, h, scale, 0.1, seed)
                e1.record()
                torch.cuda.synchronize()
                recs.append(buf[:n].cpu().numpy().astype(np.int64))
                wall.append(e0.elapsed_time(e1) * 1e3)
            r = np.array(recs[3:])
            d = np.median(np.diff(r, axis=1), axis=0)
            tot = np.median(r[:, -1] - r[:, 0])
            line = f"Lq={Lq:3d} Lk={Lk:3d}: kernel {np.median(wall[3:]):6.1f} us (events) | wg0 {tot:7.0f} cyc |"
            line += " | ".join(f"{p} {c:6.0f}" for p, c in zip(PHASES, d))
            print(line, flush=True)
    finally:
        lib.dasa_mha_bwd_stamps(None)


if __name__ == "__main__":
    main()
