"""GPU probe: native fp32 MFMA GEMM (dasa_gemm_f32) vs the bf16x6 GEMM (dasa_gemm_f32x6_ws, split-K form
when the shape has few tiles) on the short-K LXRT / vision shapes the plan rule (ops._emu_ok) keeps on
the native kernels, graph-replayed back to back."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(1600, 768, 768), (720, 768, 768), (1600, 1536, 768), (720, 1536, 768), (1600, 2304, 768),
          (720, 2304, 768), (160, 768, 768), (5760, 768, 768), (12800, 768, 768)]


def main():
    dev = torch.device("cuda", 0)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        y1, y2 = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
        planes = ops._x6_weight(W)
        tn = _time_graph(lambda: ops.gemm(x, W, y1, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=b), reps=20)
        tx = _time_graph(lambda: ops.gemm_f32x6(x, planes, y2, M=M, N=N, K=K, lda=K, ldc=N, bias=b), reps=20)
        fl = 2.0 * M * N * K / 1e6
        print(f"{M:>6}x{N:>5}x{K:>5}  native {tn:7.1f} us {fl / tn:6.1f} TF | x6 {tx:7.1f} us {fl / tx:6.1f} TF"
              f" | x6/native {tn / tx:5.2f}x | emu_ok {ops._emu_ok(M, N, K, K, x)}", flush=True)


if __name__ == "__main__":
    main()
