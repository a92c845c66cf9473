"""Host-side (Python) profile of the bench training iteration's phases: cProfile over
accumulate_gradient (both rollouts) and optim_step (backward + RMSprop) after warm-up, top functions by
own time. Shows where the host spends the ~15 ms per iteration the GPU idles in the backward phase.
    python tools/host_prof.py"""
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    sys.argv = sys.argv[:1]
    a = bench.parse()
    agent, _ = bench.build_agent(a, 0, 1)
    for _ in range(2):
        bench.train_step(agent)
    torch.cuda.synchronize()
    for name, fn in (("rollouts", lambda: (agent.zero_grad(), agent.accumulate_gradient("sample"))),
                     ("optim_step", lambda: agent.optim_step())):
        pr = cProfile.Profile()
        pr.enable()
        fn()
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(f"==== {name}")
        print(s.getvalue()[:6000])


if __name__ == "__main__":
    main()
