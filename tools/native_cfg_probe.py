"""GPU probe: the native fp32 GEMM's tile configurations (dasa_gemm_force_config) on the per-step LXRT
projection shapes that stay native (K = 768, 36-108 output tiles), graph-replayed back to back."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(720, 768, 768), (1600, 768, 768), (720, 1536, 768), (720, 2304, 768), (160, 768, 768)]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    ncfg = lib.dasa_gemm_force_config(-1)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        y = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * K / 1e6
        line = f"{M:>5}x{N:>5}x{K:>5} default {_time_graph(lambda: ops.gemm(x, W, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N), reps=20):6.1f}us |"
        for cfg in range(ncfg):
            for spl in (1, 2):
                lib.dasa_gemm_force_config(cfg + (64 * spl if spl > 1 else 0))
                try:
                    us = _time_graph(lambda: ops.gemm(x, W, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N), reps=20)
                    line += f" c{cfg}s{spl} {us:5.1f}"
                finally:
                    lib.dasa_gemm_force_config(-1)
        print(line, flush=True)


if __name__ == "__main__":
    main()
