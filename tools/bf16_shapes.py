"""GPU probe: the configs[4] bf16 GEMM (dasa_gemm_bf16 through ops.linear under ops.bf16_matmul) on the
B=256 language / vision / LXRT shapes, graph-replayed back to back (dasa_amd.kbench._time_graph): us per
launch and TFLOP/s of the default plan, and of each form listed with `--forms 9,11,12`
(dasa_gemm_force_config(1 << 20 | form)) with its max |difference| from the default."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(20480, 3072, 768), (20480, 768, 3072), (20480, 2304, 768), (9216, 3072, 768), (9216, 768, 3072),
          (9216, 2304, 768), (9216, 768, 768), (13312, 2048, 2048)]


def main():
    dev = torch.device("cuda", 0)
    forms = []
    if "--forms" in sys.argv:
        forms = [int(f) for f in sys.argv[sys.argv.index("--forms") + 1].split(",")]
    lib = _lib.lib()
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev)
        with torch.no_grad(), ops.bf16_matmul():
            us = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)
            us = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)   # (the first timing of a shape runs slow)
            line = f"{M:>6}x{N:>5}x{K:>5}  {us:8.1f} us  {2.0 * M * N * K / us / 1e6:6.1f} TF"
            if "--abf" in sys.argv:   # the same GEMM with A already bf16 (a producer that rounded it)
                xb = ops.to_bf16(x)
                ub = _time_graph(lambda: ops.linear(xb, W, b, out=y), reps=20)
                line += f" | bf16 A {ub:7.1f} us {2.0 * M * N * K / ub / 1e6:6.1f} TF"
            if "--torch" in sys.argv:   # hipBLASLt (torch bf16 linear, bf16 out) on the same shape: what a library reaches
                xb16, Wb16, bb16 = x.to(torch.bfloat16), W.to(torch.bfloat16), b.to(torch.bfloat16)
                ut = _time_graph(lambda: torch.nn.functional.linear(xb16, Wb16, bb16), reps=20)
                line += f" | torch {ut:7.1f} us {2.0 * M * N * K / ut / 1e6:6.1f} TF"
            ref = y.clone()
            for f in forms:
                lib.dasa_gemm_force_config((1 << 20) + f)
                try:
                    uf = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)
                    torch.cuda.synchronize()
                    line += f" | form {f} {uf:7.1f} us {2.0 * M * N * K / uf / 1e6:6.1f} TF d={(y - ref).abs().max().item():.1e}"
                finally:
                    lib.dasa_gemm_force_config(-1)
        print(line, flush=True)


if __name__ == "__main__":
    main()
