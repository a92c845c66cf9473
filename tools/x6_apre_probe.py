"""r04 probe: bf16x6 with A pre-split into bf16 planes (forms 22 = form 20 + pre-split A, 23 = form 8 +
pre-split A) against forms 20 / 8 splitting A in the kernel. Same products, so outputs must be bitwise
equal; prints us per launch (20 back to back, best of 3) per shape.
    python tools/x6_apre_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    L = _lib.lib()
    for M, N, K in ((12800, 3072, 768), (12800, 2304, 768), (12800, 768, 3072), (1600, 3072, 768)):
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.02
        pw, pa = ops.split3_bf16(W), ops.split3_bf16(A)
        res = {}
        for form, x in ((20, A), (22, pa), (8, A), (23, pa)):
            y = torch.empty(M, N, device=dev)
            L.dasa_gemm_force_config((1 << 21) + form)
            try:
                us = timed(lambda: ops.gemm_f32x6(x, pw, y, M=M, N=N, K=K, lda=K, ldc=N))
            finally:
                L.dasa_gemm_force_config(0)
            res[form] = (us, y)
        tf = lambda us: 2.0 * M * N * K / us / 1e6
        eq = torch.equal(res[20][1], res[22][1]) and torch.equal(res[8][1], res[23][1]) and torch.equal(res[20][1], res[8][1])
        print(f"{M}x{N}x{K}: form20 {res[20][0]:.1f} us ({tf(res[20][0]):.0f} TF)  form22 {res[22][0]:.1f} us "
              f"({tf(res[22][0]):.0f} TF)  form8 {res[8][0]:.1f} us ({tf(res[8][0]):.0f} TF)  form23 {res[23][0]:.1f} us "
              f"({tf(res[23][0]):.0f} TF)  bitwise equal: {eq}", flush=True)


if __name__ == "__main__":
    main()
