"""TN weight-gradient GEMMs (dW = dYᵀ X) of the cfg2 iteration's backward: the native fp32 kernel (dasa_gemm_f32,
opA = 1) against the bf16x6 TN kernel (dasa_gemm_f32x6_tn) in each form / split count, graph-timed, with the
max error of each against fp64 (put the 60 ms of big TN weight gradients on an x6 TN form, or
show they cannot beat 0.8 of fp32).
    python tools/gemm_tn_probe.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

# (M, N, K, lda, ldb): the batched bi-LSTM BPTT's dW_ih = dgatesᵀ x (dgates rows 8H apart) and dW_hh (h read
# from the output at stride 2H), and two deferred decoder weight gradients (K = steps x batch)
SHAPES = [(4096, 768, 112000, 8192, 768), (4096, 1024, 111999, 8192, 2048), (4096, 2240, 1400, 4096, 2240),
          (2048, 2176, 1400, 2048, 2176), (1024, 4096, 16384, 1024, 4096)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K, lda, ldb in SHAPES:
        Abuf = torch.randn(K, lda, device=dev, generator=g) * 0.1
        Bbuf = torch.randn(K, ldb, device=dev, generator=g)
        A, B = Abuf[:, :M], Bbuf[:, :N]
        ref = A.double().t() @ B.double()
        scale = ref.abs().max().item()
        y = torch.empty(M, N, device=dev)

        def native():
            ops.gemm(A, B, y, M=M, N=N, K=K, opA=1, opB=0, lda=lda, ldb=ldb, ldc=N)
        us = _time_graph(native, reps)
        native()
        err_n = (y.double() - ref).abs().max().item() / scale
        tf = 2.0 * M * N * K / us / 1e6
        print(f"{M}x{N}x{K} native   {us:9.1f} us {tf:6.1f} TF ({tf / 157.3:.2f} of fp32) err {err_n:.2e}", flush=True)
        for form in (1, 0):
            for spl in (-1, 1, 2, 4, 8):
                L.dasa_gemm_x6_tn_config(form, spl)

                def x6():
                    ops.gemm_f32x6_tn(A, B, y, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N)
                try:
                    us = _time_graph(x6, reps)
                    x6()
                    torch.cuda.synchronize()
                finally:
                    L.dasa_gemm_x6_tn_config(-1, -1)
                err = (y.double() - ref).abs().max().item() / scale
                tf = 2.0 * M * N * K / us / 1e6
                print(f"{M}x{N}x{K} x6tn f{form} s{spl:2d} {us:9.1f} us {tf:6.1f} TF ({tf / 416.7:.2f} of x6 roof) "
                      f"err {err:.2e}", flush=True)
        del Abuf, Bbuf, A, B, ref, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
