"""bf16x6 with 64-deep K steps (dasa_gemm_f32x6_k64, forms 1-3; PROBE_SET=quarter: forms 27 / 28) against the default plan and forms 8 / 20 / 7 on
the language-pipe, LXRT and vision shapes, graph-timed; bitwise check against form 8 (one launch, no split).
    python tools/k64_probe.py [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(12800, 3072, 768), (12800, 2304, 768), (12800, 768, 768), (12800, 768, 3072), (1600, 3072, 768),
          (1600, 768, 3072), (1600, 4096, 768), (5760, 768, 3072), (11200, 768, 768), (720, 3072, 768)]


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

        def k64(form):
            d = ops.GemmDesc()
            d.M, d.N, d.K, d.batch, d.opA, d.opB = M, N, K, 1, 0, 1
            d.A, d.lda, d.B, d.ldb, d.C, d.ldc = A.data_ptr(), K, wp.data_ptr(), K, y.data_ptr(), N
            d.bias, d.alpha, d.beta = bias.data_ptr(), 1.0, 0.0

            def f():
                _lib.check(L.dasa_gemm_f32x6_k64(ctypes.byref(d), N * K, form,
                                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "k64")
            return f

        line = f"{M:>5}x{N:>5}x{K:>5}"
        res = {}
        cases = (("default", run_default), ("f8", forced(8)), ("f20", forced(20)), ("f7", forced(7)),
                 ("k64_1", k64(1)), ("k64_2", k64(2)), ("k64_3", k64(3)))
        if os.environ.get("PROBE_SET") == "quarter":   # forms 27 / 28: four workgroups per CU
            cases = (("default", run_default), ("f8", forced(8)), ("f20", forced(20)), ("f27", forced(27)),
                     ("f28", forced(28)))
        if os.environ.get("PROBE_SET") == "order":   # is the first case of a shape slower (order effect)?
            cases = (("f20", forced(20)), ("default", run_default), ("f20b", forced(20)), ("default2", run_default))
        for name, fn in cases:
            us = _time_graph(fn, reps)
            fn()
            torch.cuda.synchronize()
            res[name] = y.clone()
            line += f" | {name} {us:7.1f}us {fl / us / 1e6:5.1f}TF"
        ref = res.get("f8", res.get("f20"))
        eq = {k: torch.equal(res[k], ref) for k in res if k not in ("default", "f8")}
        print(line + f" | bitwise==f8 {eq}", flush=True)
        del A, W, wp, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
