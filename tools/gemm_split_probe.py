"""GPU probe: native fp32 GEMM tile configurations x split-K (dasa_gemm_force_config = cfg + 64 * split) on
the README-finetune (BASELINE configs[3], bench.py cfg4 leg) shapes: language / LXRT projections at M = 160
(B = 2 x L = 80) and M = 72 (B = 2 x 36 views), forward (NT), dX (NN) and dW (TN), graph-replayed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(160, 768, 768, 0, 1), (72, 768, 768, 0, 1), (160, 768, 768, 0, 0), (72, 768, 768, 0, 0),
          (160, 768, 3072, 0, 0), (160, 768, 3072, 0, 1), (72, 768, 3072, 0, 1), (160, 3072, 768, 0, 0),
          (72, 3072, 768, 0, 1), (160, 768, 4096, 0, 0), (768, 768, 160, 1, 0), (768, 768, 72, 1, 0)]
CFGS = [int(c) for c in os.environ.get("PROBE_CFGS", "2,3,4,5,9,10,12,18").split(",")]
SPLITS = [int(c) for c in os.environ.get("PROBE_SPLITS", "1,2,3,4,6,8").split(",")]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    for M, N, K, opA, opB in SHAPES:
        A = torch.randn(M * K, device=dev)
        W = torch.randn(N * K, device=dev) * 0.05
        y = torch.empty(M, N, device=dev)
        lda = M if opA else K
        ldb = K if opB else N

        def run():
            ops.gemm(A, W, y, M=M, N=N, K=K, opA=opA, opB=opB, lda=lda, ldb=ldb, ldc=N)
        ref = None
        line = f"{M:>5}x{N:>5}x{K:>5} op{opA}{opB} default {_time_graph(run, reps=20):6.1f}us |"
        ref = y.clone()
        best = (1e9, "")
        for cfg in CFGS:
            for spl in SPLITS:
                lib.dasa_gemm_force_config(cfg + (64 * spl if spl > 1 else 0))
                try:
                    us = _time_graph(run, reps=20)
                    err = (y - ref).abs().max().item()
                    tag = f"c{cfg}s{spl}"
                    line += f" {tag} {us:5.1f}" + ("!" if err > 1e-3 else "")
                    if us < best[0]:
                        best = (us, tag)
                finally:
                    lib.dasa_gemm_force_config(-1)
        print(line + f" | best {best[1]} {best[0]:.1f}", flush=True)


if __name__ == "__main__":
    main()
