"""Run one bf16x6 GEMM shape back to back (PMC / stall studies under rocprofv3):
    python tools/x6_one.py M N K [reps] [form]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    form = int(sys.argv[5]) if len(sys.argv) > 5 else -1
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    y = torch.empty(M, N, device=dev)
    planes = ops.split3_bf16(W)
    if form >= 0:
        _lib.lib().dasa_gemm_force_config((1 << 21) + form)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        ops.gemm_f32x6(A, planes, y, M=M, N=N, K=K, lda=K, ldc=N)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        ops.gemm_f32x6(A, planes, y, M=M, N=N, K=K, lda=K, ldc=N)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{M}x{N}x{K} form {form}: {us:.1f} us  {2.0 * M * N * K / us / 1e6:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
