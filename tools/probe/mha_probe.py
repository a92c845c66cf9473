"""Isolated dasa_mha_fwd timing at the policy's shapes, with and without attention dropout."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dasa_amd import ops
torch.cuda.set_device(0)
dev = torch.device("cuda")

def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3

for B, Lq, Lk in ((160, 80, 80), (20, 80, 80), (20, 36, 36), (20, 80, 36), (20, 36, 80), (1280, 80, 80)):
    qkv = torch.randn(B, Lq, 2304, device=dev) * 0.3
    kv = torch.randn(B, Lk, 2304, device=dev) * 0.3
    Q, K, V = qkv[..., :768], kv[..., 768:1536], kv[..., 1536:]
    m = torch.zeros(B, Lk, device=dev)
    for p in (0.0, 0.1):
        us = bench(lambda: ops.mha(Q, K, V, m, 12, 0.125, p, 1234))
        fl = 4.0 * B * Lq * Lk * 768
        print(f"B{B} Lq{Lq} Lk{Lk} p={p}: {us:8.1f} us  {fl / us / 1e6:6.2f} TFLOP/s", flush=True)
