"""GPU probe: the skinny NT GEMMs (M <= 64, the decoder / critic linears at B = 20) in isolation,
back-to-back launches: us per launch and GB/s of weight + activation traffic. Run it under
rocprofv3 --kernel-trace --stats for the kernels' own durations. (A VALU weight-streaming kernel tried
in round 2 measured 18-20 us per launch against 8.8 us for the MFMA tile kernel + 5 us split-K reduce,
and was dropped; the env switch DASA_GEMM_SKINNY_OFF it compared against no longer exists.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402

SHAPES = [(20, 2176, 1024), (20, 1024, 2048), (20, 4096, 2240), (20, 4096, 1024), (20, 1024, 3072),
          (20, 2048, 1024), (20, 768, 768), (20, 5, 1024), (20, 64, 128), (256, 2176, 1024)]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda", 0)
for M, N, K in SHAPES:
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev)
    res = {}
    for mode in ("skinny", "tiles"):
        if mode == "tiles":
            os.environ["DASA_GEMM_SKINNY_OFF"] = "1"
        else:
            os.environ.pop("DASA_GEMM_SKINNY_OFF", None)
        res[mode] = timeit(lambda: ops.linear(A, W, b, out=y))
    os.environ.pop("DASA_GEMM_SKINNY_OFF", None)
    gb = 4.0 * (N * K + M * K + M * N) / 1e9
    print(f"{M:>4}x{N:>5}x{K:>5}  skinny {res['skinny']:7.2f} us ({gb / res['skinny'] * 1e6:7.1f} GB/s)"
          f"  tiles {res['tiles']:7.2f} us ({gb / res['tiles'] * 1e6:7.1f} GB/s)", flush=True)
