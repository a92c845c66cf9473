"""GPU probe: the isolated AdaIN / attention kernels (dasa_amd.kbench, graph-replayed back to back) under
each attention mode (dasa_attn_set_mode: 0 = automatic — two-launch D-split forward and D-split
backward at small B, whole-row forward at B >= 128; 1 = row-split kernels only), one table row per
kernel: us per launch and fraction of 8 TB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import kbench, ops  # noqa: E402


def main():
    torch.cuda.set_device(0)
    bs = tuple(int(x) for x in sys.argv[1:]) or (20, 256)
    res = {}
    for mode in (0, 1):
        ops.attn_set_mode(mode)
        res[mode] = kbench.hbm_kernels(bs)
    ops.attn_set_mode(0)
    cols = [(m, f"B{b}") for b in bs for m in (0, 1)]
    print(f"{'kernel':26s}" + "".join(f" | {k} mode{m} us  frac" for m, k in cols))
    for name in res[0]:
        if name == "hbm_stream":
            continue
        line = f"{name:26s}"
        for m, k in cols:
            e = res[m][name].get(k)
            line += f" | {e['us']:9.2f} {e['frac']:.4f}" if e else " |"
        print(line)
    print("hbm_stream", res[0]["hbm_stream"])


if __name__ == "__main__":
    main()
