"""cProfile of the cfg2 training iteration's HOST side (after warm-up): where the Python time between the
kernel launches goes (the sampled rollout's host gap). cProfile's own overhead inflates
every call; read the ratios, not the absolute times.
    python tools/host_profile.py [iterations]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    sys.argv = sys.argv[:1]
    a = bench.parse()
    import torch
    torch.cuda.set_device(0)
    agent, _ = bench.build_agent(a, 0, 1)
    bench._warm(agent, 2)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        bench.train_step(agent)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(60)


if __name__ == "__main__":
    main()
