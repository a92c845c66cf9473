"""GPU probe: the bf16x6 fp32-emulated GEMM (dasa_gemm_f32x6) against the native fp32 MFMA GEMM
(dasa_gemm_f32) and torch's fp32 matmul (hipBLASLt / rocBLAS) on the policy's nn.Linear shapes:
time per launch, TFLOP/s, and accuracy of each against an fp64 reference.

    python tools/gemm_x6_probe.py [--reps 20] [--shapes M,N,K ...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402

SHAPES = [(12800, 3072, 768), (12800, 768, 3072), (12800, 2304, 768), (12800, 768, 768), (1600, 768, 768),
          (1600, 768, 3072), (1600, 3072, 768), (1600, 4096, 768), (1600, 2304, 768), (720, 768, 768),
          (720, 3072, 768), (720, 768, 3072), (720, 2048, 2048), (5760, 768, 768), (20480, 3072, 768),
          (20480, 768, 3072)]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", nargs="*")
    ap.add_argument("--sweep", type=int, default=0, help="also time bf16x6 tile forms 0..N-1 (forced)")
    ap.add_argument("--forms", nargs="*", default=[], help="forced bf16x6 form:splitk pairs to time, e.g. 8:3 4:2")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split(",")) for s in a.shapes] if a.shapes else SHAPES
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for M, N, K in shapes:
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.02
        bias = torch.randn(N, device=dev, generator=g) * 0.1
        ref = (A.double() @ W.double().t() + bias.double())
        scale = ref.abs().max().item()
        fl = 2.0 * M * N * K
        out = {}
        ops.set_gemm_emulation(False)
        y = ops.linear(A, W, bias)
        out["native"] = dict(us=timeit(lambda: ops.linear(A, W, bias, out=y), a.reps),
                             err=(y.double() - ref).abs().max().item() / scale,
                             rel_fro=((y.double() - ref).norm() / ref.norm()).item())
        planes = ops._x6_weight(W)
        y2 = torch.empty_like(y)

        def x6():
            ops.gemm_f32x6(A, planes, y2, M=M, N=N, K=K, lda=K, ldc=N, bias=bias)
        x6()
        out["x6"] = dict(us=timeit(x6, a.reps),
                         err=(y2.double() - ref).abs().max().item() / scale,
                         rel_fro=((y2.double() - ref).norm() / ref.norm()).item())
        out["split_us"] = timeit(lambda: ops.split3_bf16(W), a.reps)
        if a.sweep:
            from dasa_amd import _lib
            L = _lib.lib()
            forms = {}
            for cfg in range(a.sweep):
                L.dasa_gemm_force_config((1 << 21) + cfg)
                x6()
                us = timeit(x6, a.reps)
                forms[cfg] = (round(fl / us / 1e6, 1), (y2.double() - ref).abs().max().item() / scale)
            L.dasa_gemm_force_config(-1)
            out["x6_forms"] = forms
            print("   forms:", " ".join(f"{c}:{v[0]}TF/{v[1]:.1e}" for c, v in forms.items()), flush=True)
        if a.forms:
            from dasa_amd import _lib
            L = _lib.lib()
            forms = {}
            for f in a.forms:
                cfg, spl = (int(v) for v in f.split(":"))
                L.dasa_gemm_force_config((1 << 21) + cfg + 32 * spl)
                x6()
                us = timeit(x6, a.reps)
                forms[f] = (round(fl / us / 1e6, 1), (y2.double() - ref).abs().max().item() / scale)
            L.dasa_gemm_force_config(-1)
            out["x6_split_forms"] = forms
            print("   form:split:", " ".join(f"{c}={v[0]}TF/{v[1]:.1e}" for c, v in forms.items()), flush=True)
        y3 = torch.addmm(bias, A, W.t())
        out["torch"] = dict(us=timeit(lambda: torch.addmm(bias, A, W.t(), out=y3), a.reps),
                            err=(y3.double() - ref).abs().max().item() / scale,
                            rel_fro=((y3.double() - ref).norm() / ref.norm()).item())
        for k in ("native", "x6", "torch"):
            out[k]["TFLOPs"] = round(fl / out[k]["us"] / 1e6, 1)
        rows.append({"shape": [M, N, K], **out})
        print(f"{M:>6}x{N:>5}x{K:>5}  native {out['native']['TFLOPs']:>6.1f} TF err {out['native']['err']:.1e}"
              f" | x6 {out['x6']['TFLOPs']:>6.1f} TF err {out['x6']['err']:.1e}"
              f" | torch {out['torch']['TFLOPs']:>6.1f} TF err {out['torch']['err']:.1e}"
              f" | split {out['split_us']:.1f} us", flush=True)
        del planes
        ops._X6.clear()
        ops.set_gemm_emulation(True)
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
