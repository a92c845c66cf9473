"""GPU probe: the bf16x6 fp32 GEMM (dasa_gemm_f32x6_ws, default plan) on the language / LXRT / LSTM
shapes of the cfg2 iteration, graph-replayed back to back (dasa_amd.kbench._time_graph): us per launch
and fp32-equivalent TFLOP/s. `--forms 6,7,8` also times each listed tile form forced
(dasa_gemm_force_config(1 << 21 | form)) and its max |difference| from the default form."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

SHAPES = [(12800, 3072, 768), (12800, 2304, 768), (12800, 768, 3072), (12800, 768, 768), (1600, 3072, 768),
          (1600, 768, 3072), (720, 3072, 768), (720, 768, 3072), (1600, 4096, 768), (720, 2048, 2048),
          (1600, 768, 768), (720, 768, 768), (720, 1536, 768), (720, 2304, 768)]
# tail-free shapes (whole rounds of 256 workgroups for 256 x 128 AND 128 x 128 tiles): the per-CU rate of a form
SHAPES_ROUND = [(8192, 1024, 3072), (8192, 1024, 768), (8192, 2048, 768), (16384, 1024, 3072)]


def main():
    dev = torch.device("cuda", 0)
    forms = []
    if "--forms" in sys.argv:
        forms = [int(f) for f in sys.argv[sys.argv.index("--forms") + 1].split(",")]
    lib = _lib.lib()
    shapes = SHAPES_ROUND + SHAPES if "--round" in sys.argv else SHAPES
    if "--lang" in sys.argv:
        shapes = [s for s in shapes if s[0] >= 8192]
    for M, N, K in shapes:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev)
        us = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)
        line = f"{M:>6}x{N:>5}x{K:>5}  {us:8.1f} us  {2.0 * M * N * K / us / 1e6:6.1f} TF"
        ref = y.clone()
        for f in forms:
            lib.dasa_gemm_force_config((1 << 21) + f)
            ops._X6_WS_NEED.clear()      # the forced plan has its own split / workspace
            try:
                uf = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)
                torch.cuda.synchronize()
                line += f" | form {f} {uf:7.1f} us {2.0 * M * N * K / uf / 1e6:6.1f} TF d={(y - ref).abs().max().item():.1e}"
            finally:
                lib.dasa_gemm_force_config(-1)
                ops._X6_WS_NEED.clear()
        print(line, flush=True)


if __name__ == "__main__":
    main()
