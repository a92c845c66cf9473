"""GPU probe: the skinny (M <= 32) weight-streaming GEMMs of the decision step in isolation, graph-replayed
back to back (dasa_amd.kbench._time_graph), for each plan form: the tile kernels + split-K reduce used
before (target waves 0), and the gemm_skinny_* kernels at several target wave counts / pinned K steps.
"hot": one weight, cache-resident across replays; "cold": rotating over > 512 MB of weight copies so
every launch streams its weight from HBM. Prints us per launch and GB/s of weight + activation bytes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402
from dasa_amd.kbench import _time_graph  # noqa: E402

NT = [(20, 2176, 1024), (20, 2048, 1024), (20, 4096, 2240), (20, 4096, 1024), (20, 1024, 3072), (2, 2176, 1024)]
NN = [(20, 1024, 2176), (20, 2240, 4096), (20, 1024, 4096), (20, 1024, 2048)]
MODES = [(0, -1), (-1, -1), (-1, 16), (-1, 8), (-1, 24), (-1, 4), (-1, 20), (-1, 2)]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    for kind, shapes in (("nt", NT), ("nn", NN)):
        for M, N, K in shapes:
            x = torch.randn(M, K, device=dev)
            ncopy = max(2, int(512e6 // (4 * N * K)) + 1)
            Ws = [torch.randn(*((N, K) if kind == "nt" else (K, N)), device=dev) * 0.05 for _ in range(ncopy)]
            y = torch.empty(M, N, device=dev)
            gb = 4.0 * (N * K + M * K + M * N) / 1e9
            line = f"{kind} {M:>3}x{N:>5}x{K:>5}"
            for waves, ks in MODES:
                lib.dasa_gemm_skinny_tune(waves, ks)
                it = iter(range(1 << 30))
                if kind == "nt":
                    hot = _time_graph(lambda: ops.linear(x, Ws[0], out=y))
                    cold = _time_graph(lambda: ops.linear(x, Ws[next(it) % ncopy], out=y))
                else:
                    hot = _time_graph(lambda: ops.matmul_nn(x, Ws[0], out=y))
                    cold = _time_graph(lambda: ops.matmul_nn(x, Ws[next(it) % ncopy], out=y))
                tag = "tiles" if waves == 0 else (f"k{ks - 16 if ks > 16 else 'plan'}-2tile" if ks >= 16 else f"k{ks}")
                line += f" | {tag} {hot:6.2f}/{cold:6.2f}us {gb / cold * 1e6:5.0f}GB/s"
            lib.dasa_gemm_skinny_tune(-1, -1)
            print(line, flush=True)
            del Ws


if __name__ == "__main__":
    main()
