"""GPU probe: the LDS-staged attention backward (dasa_mha_bwd) at the finetune's B = 2, 12 heads, split over
1-4 workgroups per (batch, head) (dasa_mha_bwd_split): us per launch (kbench._time_graph: 20 launches in
one captured graph, so host launch latency is excluded)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    B, h, scale, seed = 2, 12, 1 / 8.0, 5
    for Lq, Lk, p in ((80, 80, 0.1), (80, 36, 0.1), (36, 80, 0.1), (36, 36, 0.1)):
        Q, K, V, dO = (torch.randn(B, L_, 768, device=dev) for L_ in (Lq, Lk, Lk, Lq))
        m = torch.zeros(B, Lk, device=dev)
        _, probs = ops.mha(Q, K, V, m, h, scale, p, seed, save_probs=True)
        line = f"Lq={Lq:3d} Lk={Lk:3d}"
        for parts in (1, 2, 3, 4, 0):
            lib.dasa_mha_bwd_split(parts)
            us = _time_graph(lambda: ops.mha_bwd(Q, K, V, probs, dO, h, scale, p, seed), reps=20)
            line += f" | parts={parts or 'auto'} {us:6.1f} us"
        print(line, flush=True)
    lib.dasa_mha_bwd_split(0)


if __name__ == "__main__":
    main()
