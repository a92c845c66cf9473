"""GPU probe: the persistent BPTT (dasa_bilstm_bwd, H = 1024) at small B with the one-row-tile form
(dasa_bilstm_bptt_one_tile(1), default at B <= 16) and the two-tile form: us per launch (HIP events,
median of 20) and whether the two agree bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    H = 1024
    torch.manual_seed(0)
    whh_f, whh_b = [(torch.rand(4 * H, H, device=dev) - 0.5) * 0.1 for _ in range(2)]
    assert lib.dasa_bilstm_set_mode(2) == 0
    for B, L in ((2, 80), (8, 80), (16, 80), (20, 80)):
        xproj = torch.randn(B, L, 2, 4 * H, device=dev)
        li = torch.full((B,), L, dtype=torch.int32, device=dev)
        _, _, _, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
        gout = torch.randn(B, L, 2 * H, device=dev)
        line, outs = f"B={B:3d} L={L}", {}
        for one in (1, 0):
            lib.dasa_bilstm_bptt_one_tile(one)
            ts = []
            for _ in range(22):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                dg = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, None, None, H)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000)
            outs[one] = dg
            ts = sorted(ts[2:])
            line += f" | one_tile={one} {ts[len(ts) // 2]:8.1f} us"
        line += f" | bitwise {torch.equal(outs[0], outs[1])}"
        print(line, flush=True)
    lib.dasa_bilstm_bptt_one_tile(1)
    lib.dasa_bilstm_set_mode(0)


if __name__ == "__main__":
    main()
