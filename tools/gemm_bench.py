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


def make_fn(M, N, K, opA, opB, dev):
    """dasa and torch closures for C[M,N] = opA(A) opB(B) in the descriptor's layouts."""
    A = torch.randn(K, M, device=dev) if opA else torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev) if opB else torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)
    f1 = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, opA=opA, opB=opB, lda=A.shape[1], ldb=B.shape[1], ldc=N)
    At = A.t() if opA else A
    Bt = B.t() if opB else B
    f2 = lambda: torch.mm(At, Bt, out=C)
    return f1, f2


def grid(shapes):
    """Every (tile config, split-K) pair on each shape: best five, the automatic plan and torch."""
    from dasa_amd import _lib
    L = _lib.lib()
    n = L.dasa_gemm_force_config(-1)
    dev = torch.device("cuda")
    for M, N, K, opA, opB in shapes:
        f1, f2 = make_fn(M, N, K, opA, opB, dev)
        fl = 2.0 * M * N * K
        res = []
        for c in range(n):
            for sk in (1, 2, 3, 4, 6, 8, 12):
                if K // sk < 128:
                    continue
                L.dasa_gemm_force_config(c + 64 * sk)
                res.append((fl / bench(f1, 10) / 1e9, c, sk))
        L.dasa_gemm_force_config(-1)
        auto = fl / bench(f1) / 1e9
        tor = fl / bench(f2) / 1e9
        res.sort(reverse=True)
        best = " ".join(f"c{c}s{sk}:{tf:.0f}" for tf, c, sk in res[:5])
        print(f"M{M} N{N} K{K} op{opA}{opB}  auto {auto:.1f}  torch {tor:.1f}  best {best}", flush=True)


def main():
    if "--sweep" in sys.argv:
        return sweep()
    if "--grid" in sys.argv:
        import json
        path = sys.argv[sys.argv.index("--grid") + 1]
        rows = json.load(open(path))
        if isinstance(rows, dict):
            rows = rows["shapes"]
        return grid([tuple(r["shape"][:3]) + tuple(r["shape"][4:6]) for r in rows])
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
