"""bf16x6 with A pre-split (dasa_gemm_f32x6_pp, forms 3 / 2: all operands by LDS-DMA) against the default plan and
forms 8 / 20 on the language-pipe and LXRT shapes, graph-timed; bitwise check against form 8 (one launch, no
split), and the cost of splitting A separately (dasa_f32_split3_bf16) for reference.
    python tools/x6p_probe.py [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(12800, 3072, 768), (12800, 2304, 768), (12800, 768, 768), (12800, 768, 3072), (1600, 3072, 768),
          (1600, 768, 3072), (8192, 1024, 3072)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K in SHAPES:
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.03
        bias = torch.randn(N, device=dev, generator=g) * 0.1
        wp = ops.split3_bf16(W)
        ap = ops.split3_bf16(A)
        y = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * K

        def run_default():
            ops.gemm_f32x6(A, wp, y, M=M, N=N, K=K, lda=K, ldc=N, bias=bias)

        def forced(cfg):
            def f():
                L.dasa_gemm_force_config((1 << 21) + cfg + 32 * 1)
                try:
                    ops.gemm_f32x6(A, wp, y, M=M, N=N, K=K, lda=K, ldc=N, bias=bias)
                finally:
                    L.dasa_gemm_force_config(-1)
            return f

        def pp(form):
            d = ops.GemmDesc()
            d.M, d.N, d.K, d.batch, d.opA, d.opB = M, N, K, 1, 0, 1
            d.A, d.lda, d.B, d.ldb, d.C, d.ldc = ap.data_ptr(), K, wp.data_ptr(), K, y.data_ptr(), N
            d.bias, d.alpha, d.beta = bias.data_ptr(), 1.0, 0.0

            def f():
                _lib.check(L.dasa_gemm_f32x6_pp(ctypes.byref(d), N * K, M * K, form,
                                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "pp")
            return f

        line = f"{M:>5}x{N:>5}x{K:>5}"
        res = {}
        for name, fn in (("default", run_default), ("f8", forced(8)), ("f20", forced(20)), ("f7", forced(7)),
                         ("pp3", pp(3)), ("pp2", pp(2)), ("pp4", pp(4)), ("pp5", pp(5))):
            us = _time_graph(fn, reps)
            fn()
            torch.cuda.synchronize()
            res[name] = y.clone()
            line += f" | {name} {us:7.1f}us {fl / us / 1e6:5.1f}TF"
        us_split = _time_graph(lambda: ops.split3_bf16(A), reps)
        line += f" | splitA {us_split:6.1f}us"
        eq = {k: torch.equal(res[k], res["f8"]) for k in ("pp3", "pp2", "pp4", "pp5", "f20")}
        print(line + f" | bitwise==f8 {eq}", flush=True)
        del A, W, wp, ap, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
