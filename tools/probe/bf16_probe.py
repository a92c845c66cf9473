"""bf16 NT GEMM (configs[4]) timing on the B=256 policy shapes: both tile configs vs the fp32 kernel."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dasa_amd import ops, _lib
L = _lib.lib()
torch.cuda.set_device(0)
dev = torch.device("cuda")


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


for M, N, K in ((20480, 3072, 768), (20480, 768, 3072), (20480, 2304, 768), (20480, 768, 768), (20480, 8192, 768),
                (9216, 3072, 768), (9216, 768, 2176), (13312, 2048, 2048), (256, 4096, 2240), (4096, 4096, 4096)):
    A = torch.rand(M, K, device=dev) * 2 - 1
    W = torch.rand(N, K, device=dev) * 2 - 1
    fl = 2.0 * M * N * K
    f32 = fl / bench(lambda: ops.linear(A, W)) / 1e9
    res = []
    with torch.no_grad(), ops.bf16_matmul():
        for c in (-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10):
            L.dasa_gemm_force_config(c if c < 0 else (1 << 20) + c)
            res.append(fl / bench(lambda: ops.linear(A, W)) / 1e9)
        L.dasa_gemm_force_config(-1)
        tb = fl / bench(lambda: A.to(torch.bfloat16) @ W.to(torch.bfloat16).t()) / 1e9
    print(f"M{M} N{N} K{K}: fp32 {f32:.0f} | bf16 auto {res[0]:.0f} c128x128w4 {res[1]:.0f} c256x128w8 {res[2]:.0f} "
          f"c128x128w8 {res[3]:.0f} c128x64w4 {res[4]:.0f} c128x128w16 {res[5]:.0f} c256x128w16 {res[6]:.0f} "
          f"c128x256w8 {res[7]:.0f} c256x128w8pf2 {res[8]:.0f} c128x128w8pf2 {res[9]:.0f} c256x256w16 {res[10]:.0f} "
          f"c128x256w8pf2 {res[11]:.0f} | torch bf16 (incl. casts) {tb:.0f} TFLOP/s", flush=True)
