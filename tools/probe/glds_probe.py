"""glds NT GEMM configs (15-20): correctness vs fp64 host math (ragged shapes, epilogues, split-K)
and timing against the current automatic plan and torch on the policy's NT shapes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dasa_amd import ops, _lib
L = _lib.lib()
torch.cuda.set_device(0)
dev = torch.device("cuda")
n = L.dasa_gemm_force_config(-1)
GL = list(range(15, n)) if len(sys.argv) < 2 else [int(x) for x in sys.argv[1].split(",")]

def check():
    g = torch.Generator(device="cpu").manual_seed(0)
    bad = 0
    for M, N, K in ((1, 64, 32), (37, 70, 96), (200, 130, 768), (1000, 770, 2176), (130, 2048, 2048)):
        A = torch.randn(M, K, generator=g); W = torch.randn(N, K, generator=g); b = torch.randn(N, generator=g)
        ref = torch.tanh(A.double() @ W.double().t() + b.double())
        scale = (A.double().abs() @ W.double().abs().t()).max().item()   # f32 error ~ 1e-7 * sum|a*b|
        Ad, Wd, bd = A.to(dev), W.to(dev), b.to(dev)
        for c in GL:
            for sk in (1, 2, 3):
                if K // sk < 64:
                    continue
                L.dasa_gemm_force_config(c + 64 * sk)
                y = ops.linear(Ad, Wd, bd, act="tanh")
                torch.cuda.synchronize()
                err = (y.double().cpu() - ref).abs().max().item()
                ok = err < 2e-6 * scale
                bad += not ok
                if not ok:
                    print(f"FAIL cfg {c} sk {sk} M{M} N{N} K{K}: max err {err:.3e}", flush=True)
    L.dasa_gemm_force_config(-1)
    print("correctness failures:", bad, flush=True)
    return bad

def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it

def timing():
    shapes = ((12800, 3072, 768), (12800, 768, 3072), (12800, 2304, 768), (12800, 768, 768),
              (1600, 768, 768), (1600, 3072, 768), (1600, 768, 3072), (1600, 2304, 768), (1600, 4096, 768),
              (720, 768, 768), (720, 3072, 768), (720, 768, 3072), (720, 2304, 768), (1040, 2048, 2048),
              (5760, 768, 768), (4096, 4096, 4096))
    if os.environ.get("PROBE_SKINNY"):
        shapes = ((20, 4096, 2240), (20, 2176, 1024), (20, 1024, 3072), (20, 1024, 2048), (20, 2048, 1024),
                  (20, 1024, 2176), (20, 5, 1024), (20, 1024, 1024), (1400, 1024, 1024), (700, 1024, 1024))
    for M, N, K in shapes:
        A = torch.rand(M, K, device=dev) * 2 - 1; W = torch.rand(N, K, device=dev) * 2 - 1
        fl = 2.0 * M * N * K
        f = lambda: ops.linear(A, W)
        auto = fl / bench(f) / 1e9
        tor = fl / bench(lambda: A @ W.t()) / 1e9
        res = []
        for c in GL:
            for sk in (1, 2, 3, 4):
                if K // sk < 256 and sk > 1:
                    continue
                L.dasa_gemm_force_config(c + 64 * sk)
                res.append((fl / bench(f, 10) / 1e9, c, sk))
        L.dasa_gemm_force_config(-1)
        res.sort(reverse=True)
        print(f"M{M} N{N} K{K}: auto {auto:.1f} torch {tor:.1f} glds " +
              " ".join(f"c{c}s{s}:{t:.0f}" for t, c, s in res[:6]), flush=True)

if os.environ.get("PROBE_SKINNY") or check() == 0:
    timing()
