"""Host-side (Python) cost of one bench training iteration: cProfile of train_step, top functions."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    a = bench.parse()
    rank, world = bench.setup_dist(a)
    from dasa_amd import functional as DF
    DF.reseed(1234)
    agent, env = bench.build_agent(a, rank, world)
    bench.train_step(agent)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.train_step(agent)
    torch.cuda.synchronize()
    print(f"wall {1e3 * (time.perf_counter() - t0):.1f} ms")
    pr = cProfile.Profile()
    pr.enable()
    bench.train_step(agent)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
