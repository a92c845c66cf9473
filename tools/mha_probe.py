"""GPU probe: dasa_mha_fwd on the cfg2 shapes (language stack: 160 sequences x 12 heads, L = 80, with the
0.1 attention dropout; LXRT at B = 20: 80 x 80 language, 36 x 36 visual, 80 x 36 / 36 x 80 cross),
graph-replayed back to back: us per launch and GB/s of its Q, K, V reads + output write (vs 8 TB/s)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for B, Lq, Lk, p in [(160, 80, 80, 0.1), (160, 80, 80, 0.0), (20, 80, 80, 0.1), (20, 36, 36, 0.1),
                         (20, 80, 36, 0.1), (20, 36, 80, 0.1)]:
        H = 12
        qkv = torch.randn(B, Lq, 3 * 768, device=dev)
        kv = torch.randn(B, Lk, 3 * 768, device=dev)
        Q, K, V = qkv[..., :768], kv[..., 768:1536], kv[..., 1536:]
        mask = torch.zeros(B, Lk, device=dev)
        us = _time_graph(lambda: ops.mha(Q, K, V, mask, H, 0.125, drop_p=p, seed=1), reps=20)
        nbytes = 4.0 * B * (2 * Lq + 2 * Lk) * 768
        print(f"B={B:>4} Lq={Lq:>3} Lk={Lk:>3} p={p}: {us:7.2f} us  {nbytes / us / 1e3:7.1f} GB/s  "
              f"frac {nbytes / us / 1e3 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()
