"""Cost of the erf-GELU epilogue in the FFN-up GEMMs: the same GEMM with act='gelu' and with no
activation, graph-timed — the bf16x6 fp32 path (cfg2's language pipe, 12800 x 3072 x 768) and the bf16 path
(configs[4], 20480 x 3072 x 768, bf16 A and bf16 C as in the FFN hand-off).
    python tools/gelu_epilogue_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K in ((12800, 3072, 768), (1600, 3072, 768)):
        x = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g)
        y = torch.empty(M, N, device=dev)
        for _ in range(2):
            t_g = _time_graph(lambda: ops.linear(x, W, b, act="gelu", out=y), reps=20)
            t_n = _time_graph(lambda: ops.linear(x, W, b, out=y), reps=20)
        print(f"x6   {M}x{N}x{K}: gelu {t_g:7.1f} us  none {t_n:7.1f} us  epilogue {t_g - t_n:6.1f} us", flush=True)
    for M, N, K in ((20480, 3072, 768), (9216, 3072, 768)):
        x = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g)
        with torch.no_grad(), ops.bf16_matmul():
            xb = ops.to_bf16(x)
            for _ in range(2):
                t_g = _time_graph(lambda: ops.linear(xb, W, b, act="gelu", out_dtype=torch.bfloat16), reps=20)
                t_n = _time_graph(lambda: ops.linear(xb, W, b, out_dtype=torch.bfloat16), reps=20)
        print(f"bf16 {M}x{N}x{K}: gelu {t_g:7.1f} us  none {t_n:7.1f} us  epilogue {t_g - t_n:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
