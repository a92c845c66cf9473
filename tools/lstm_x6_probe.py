"""GPU probe: the persistent bi-LSTM forward (H = 1024, L = 80) with the recurrent product as bf16x6
(dasa_bilstm_fwd_x6(1)) vs native fp32 MFMA (0): ms per launch (median of 10, HIP events) and the max
|difference| of the outputs; the B = 20 (sampled rollout, one 32-row tile) and B = 160 (teacher
rollout's 8-step language chunk, five tiles) launches of the cfg2 iteration."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    H, L = 1024, 80
    torch.manual_seed(0)
    whh_f, whh_b = [(torch.rand(4 * H, H, device=dev) - 0.5) * 0.06 for _ in range(2)]
    for B in (20, 40, 96, 160):
        xproj = torch.randn(B, L, 2, 4 * H, device=dev) * 0.5
        li = torch.full((B,), L, dtype=torch.int32, device=dev)
        line = f"B={B:>4}"
        outs = {}
        for x6 in (0, 1, 0, 1):
            lib.dasa_bilstm_fwd_x6(x6)
            ts = []
            for _ in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out, h_n, c_n, _ = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ops.check_device_errors()
            outs[x6] = out
            ts = sorted(ts[2:])
            line += f" | x6={x6} {ts[len(ts) // 2]:7.3f} ms"
        d = (outs[1] - outs[0]).abs().max().item()
        print(line + f" | max|x6 - native| {d:.2e}", flush=True)
    lib.dasa_bilstm_fwd_x6(1)


if __name__ == "__main__":
    main()
