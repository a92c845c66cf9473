"""GEMM shape sweep: dasa_gemm_f32 vs torch.matmul (hipBLASLt fp32) on the policy's shapes."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops

SHAPES = [  # (M, N, K, name)
    (1600, 768, 768, "lang qkv/out"), (1600, 3072, 768, "lang ffn1"), (1600, 768, 3072, "lang ffn2"),
    (720, 768, 768, "visn qkv"), (720, 3072, 768, "visn ffn1"), (720, 768, 3072, "visn ffn2"),
    (720, 768, 2176, "visn_fc"), (1040, 2048, 2048, "adain"), (1600, 4096, 768, "lstm xproj"),
    (20, 4096, 2240, "dec lstm ih"), (20, 2176, 1024, "dec linear_in"), (20, 1024, 3072, "dec linear_out"),
    (4096, 768, 1600, "dW_ih (tn)"), (2048, 2048, 1040, "dW adain (tn)"), (4096, 4096, 4096, "square 4k"),
]


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def sweep():
    from dasa_amd import _lib
    L = _lib.lib()
    n = L.dasa_gemm_force_config(-1)
    dev = torch.device("cuda")
    print(f"{'shape':<18}" + "".join(f"{c:>7}" for c in range(n)) + "   auto  torch")
    for M, N, K, name in SHAPES:
        if "(tn)" in name:
            A = torch.randn(K, M, device=dev)
            B = torch.randn(K, N, device=dev)
            f1 = lambda: ops.matmul_tn(A, B)
            f2 = lambda: A.t() @ B
        else:
            A = torch.randn(M, K, device=dev)
            W = torch.randn(N, K, device=dev)
            f1 = lambda: ops.linear(A, W)
            f2 = lambda: A @ W.t()
        fl = 2.0 * M * N * K
        row = []
        for c in range(n):
            L.dasa_gemm_force_config(c)
            row.append(fl / bench(f1) / 1e9)
        L.dasa_gemm_force_config(-1)
        row.append(fl / bench(f1) / 1e9)
        row.append(fl / bench(f2) / 1e9)
        print(f"{name:<18}" + "".join(f"{x:>7.1f}" for x in row), flush=True)


def main():
    if "--sweep" in sys.argv:
        return sweep()
    dev = torch.device("cuda")
    torch.backends.cuda.matmul.allow_tf32 = False
    print(f"{'shape':<18}{'M':>6}{'N':>6}{'K':>6}{'dasa us':>10}{'TF':>8}{'torch us':>10}{'TF':>8}")
    for M, N, K, name in SHAPES:
        if "(tn)" in name:
            A = torch.randn(K, M, device=dev)
            B = torch.randn(K, N, device=dev)
            f1 = lambda: ops.matmul_tn(A, B)
            f2 = lambda: A.t() @ B
        else:
            A = torch.randn(M, K, device=dev)
            W = torch.randn(N, K, device=dev)
            f1 = lambda: ops.linear(A, W)
            f2 = lambda: A @ W.t()
        t1, t2 = bench(f1), bench(f2)
        fl = 2.0 * M * N * K
        print(f"{name:<18}{M:>6}{N:>6}{K:>6}{1e3*t1:>10.1f}{fl/t1/1e9:>8.1f}{1e3*t2:>10.1f}{fl/t2/1e9:>8.1f}")


if __name__ == "__main__":
    main()
