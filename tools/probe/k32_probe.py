"""Double-buffered 32-deep K NT GEMM configs (36-38) and the L2-grouped tile order: correctness vs
fp64 host math, then timing against the automatic plan and torch on the policy's large NT shapes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dasa_amd import ops, _lib
L = _lib.lib()
torch.cuda.set_device(0)
dev = torch.device("cuda")
CF = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "27,25,36,37,38").split(",")]
GR = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,4,8").split(",")]


def force(c, s=0, g=0):
    L.dasa_gemm_force_config(c + 64 * s + 4096 * g)


def check():
    g = torch.Generator(device="cpu").manual_seed(0)
    bad = 0
    for M, N, K in ((37, 70, 64), (200, 130, 768), (1000, 770, 2176), (300, 2048, 2048), (1300, 520, 128)):
        A = torch.randn(M, K, generator=g); W = torch.randn(N, K, generator=g); b = torch.randn(N, generator=g)
        ref = torch.tanh(A.double() @ W.double().t() + b.double())
        scale = (A.double().abs() @ W.double().abs().t()).max().item()
        Ad, Wd, bd = A.to(dev), W.to(dev), b.to(dev)
        for c in CF:
            for grp in GR:
                for sk in (1, 2):
                    if K // sk < 64:
                        continue
                    force(c, sk, grp)
                    y = ops.linear(Ad, Wd, bd, act="tanh")
                    torch.cuda.synchronize()
                    err = (y.double().cpu() - ref).abs().max().item()
                    if not err < 2e-6 * scale:
                        bad += 1
                        print(f"FAIL cfg {c} g {grp} sk {sk} M{M} N{N} K{K}: max err {err:.3e}", flush=True)
    L.dasa_gemm_force_config(-1)
    print("correctness failures:", bad, flush=True)
    return bad


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


def timing():
    shapes = ((12800, 3072, 768), (12800, 768, 3072), (12800, 2304, 768), (12800, 768, 768), (12800, 8192, 768),
              (6400, 3072, 768), (1600, 3072, 768), (1040, 2048, 2048), (4096, 4096, 4096))
    for M, N, K in shapes:
        A = torch.rand(M, K, device=dev) * 2 - 1
        W = torch.rand(N, K, device=dev) * 2 - 1
        fl = 2.0 * M * N * K
        f = lambda: ops.linear(A, W)
        L.dasa_gemm_force_config(-1)
        auto = fl / bench(f) / 1e9
        tor = fl / bench(lambda: A @ W.t()) / 1e9
        res = []
        for c in CF:
            for grp in GR:
                force(c, 1, grp)
                res.append((fl / bench(f) / 1e9, f"c{c}g{grp}"))
        L.dasa_gemm_force_config(-1)
        res.sort(reverse=True)
        print(f"M{M} N{N} K{K}: auto {auto:.1f} torch {tor:.1f} | " + " ".join(f"{n}:{t:.0f}" for t, n in res), flush=True)


if check() == 0:
    timing()
