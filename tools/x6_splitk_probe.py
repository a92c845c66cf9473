"""bf16x6 split-K shapes of the cfg2 iteration (few output tiles: the LXRT / vision FFN outputs, the AdaIN gate
GEMM, the batched BPTT's recurrent product) under the default plan and forced (form, split) pairs — form 8
(128 x 128), 4 (64 x 128), 5 (64 x 64) — graph-timed, each twice (the first timing of a shape runs slow).
    python tools/x6_splitk_probe.py [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

# (M, N, K, batch)
SHAPES = [(720, 768, 3072, 1), (720, 768, 2176, 1), (1600, 768, 3072, 1), (720, 2048, 2048, 1), (700, 1024, 4096, 2),
          (1400, 1024, 4096, 2)]
FORMS = [(8, 0), (8, 2), (8, 4), (8, 8), (4, 1), (4, 2), (4, 3), (4, 4), (4, 6), (5, 1), (5, 2), (5, 3), (5, 4)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    global SHAPES
    if len(sys.argv) > 2:   # MxNxK[xbatch],... (e.g. the 5760-row vision-token shapes of a teacher chunk)
        SHAPES = [tuple(int(v) for v in (s.split("x") + ["1"])[:4]) for s in sys.argv[2].split(",")]
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    for M, N, K, bt in SHAPES:
        A = torch.randn(bt, M, K, device=dev, generator=g)
        W = torch.randn(bt * N, K, device=dev, generator=g) * 0.03
        wp = ops.split3_bf16(W)                      # [3][bt*N][K]: batch b at row offset b*N
        y = torch.empty(bt, M, N, device=dev)
        d = ops.GemmDesc()
        d.M, d.N, d.K, d.batch, d.opA, d.opB = M, N, K, bt, 0, 1
        d.A, d.lda, d.strideA = A.data_ptr(), K, M * K
        d.B, d.ldb, d.strideB = wp.data_ptr(), K, N * K
        d.C, d.ldc, d.strideC = y.data_ptr(), N, M * N
        d.alpha, d.beta = 1.0, 0.0
        plane = bt * N * K
        fl = 2.0 * M * N * K * bt

        def run(cfg=None, split=0):
            def f():
                if cfg is not None:
                    L.dasa_gemm_force_config((1 << 21) + cfg + 32 * split)
                try:
                    need = L.dasa_gemm_f32x6_workspace(ctypes.byref(d))
                    ws, nb = ops._gemm_ws(dev, d, need) if need else (0, 0)
                    _lib.check(L.dasa_gemm_f32x6_ws(ctypes.byref(d), plane, ws, nb, st()), "x6")
                finally:
                    if cfg is not None:
                        L.dasa_gemm_force_config(-1)
            return f
        cases = [("plan", run())] + [(f"f{c}s{s}", run(c, s)) for c, s in FORMS] + [("plan2", run())]
        line = f"{M:>5}x{N:>5}x{K:>5}x{bt}"
        ref = None
        for name, fn in cases:
            us = _time_graph(fn, reps)
            fn()
            torch.cuda.synchronize()
            err = 0.0 if ref is None else (y - ref).abs().max().item()
            if ref is None:
                ref = y.clone()
            line += f" | {name} {us:6.1f}us {fl / us / 1e6:5.1f}TF" + (f" e{err:.1e}" if err > 1e-3 else "")
        print(line, flush=True)
        del A, W, wp, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
