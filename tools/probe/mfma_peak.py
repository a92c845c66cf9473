"""Sustained fp32 MFMA rate vs duration (clock held under load), plus dasa GEMM vs torch on the
bench's top shapes in isolation."""
import ctypes, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_peak.so"))
torch.cuda.set_device(0)
out = torch.empty(4096 * 256, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for blocks in (256, 1024):
    for iters in (200, 2000, 20000, 100000):
        lib.mfma_peak_launch(ctypes.c_void_p(out.data_ptr()), blocks, iters, ctypes.c_void_p(st))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.mfma_peak_launch(ctypes.c_void_p(out.data_ptr()), blocks, iters, ctypes.c_void_p(st))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        fl = blocks * 4 * iters * 32 * 4096.0
        print(f"blocks {blocks} iters {iters}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOP/s", flush=True)
from dasa_amd import ops
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it
for M, N, K in ((12800, 3072, 768), (12800, 768, 3072), (12800, 2304, 768), (12800, 768, 768),
                (1600, 768, 768), (1600, 3072, 768), (1600, 768, 3072), (720, 768, 768), (720, 3072, 768)):
    A = torch.randn(M, K, device="cuda"); W = torch.randn(N, K, device="cuda")
    fl = 2.0 * M * N * K
    t1 = bench(lambda: ops.linear(A, W)); t2 = bench(lambda: A @ W.t())
    print(f"M{M} N{N} K{K}: dasa {fl / t1 / 1e9:.1f}  torch {fl / t2 / 1e9:.1f} TFLOP/s", flush=True)
