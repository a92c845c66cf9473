"""Phase breakdown of one bench training iteration: for each phase (teacher rollout, sampled
rollout, backward + all-reduce + optimizer) the host enqueue time, and the GPU time between HIP
events recorded at the phase boundaries (no syncs inside the iteration), plus per-phase device
time per kernel family (dasa_amd.prof, a separate instrumented iteration)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def phases(agent):
    from dasa_amd.r2r.param import args
    marks = []

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((name, time.perf_counter(), e))
    mark("start")
    agent.zero_grad()
    agent.feedback = "teacher"
    agent.vl_rollout(train_ml=args.ml_weight, train_rl=False)
    mark("teacher")
    agent.feedback = "sample"
    agent.vl_rollout(train_ml=None, train_rl=True)
    mark("sample")
    agent.optim_step()
    mark("optim")
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    out = {}
    for (n0, h0, e0), (n1, h1, e1) in zip(marks, marks[1:]):
        out[n1] = {"host_ms": round(1e3 * (h1 - h0), 1), "gpu_ms": round(e0.elapsed_time(e1), 1)}
    out["total_wall_ms"] = round(1e3 * (t_end - marks[0][1]), 1)
    out["steps"] = {"teacher": agent.logs["viewsteps/teacher"][-1], "sample": agent.logs["viewsteps/sample"][-1]}
    return out


def main():
    a = bench.parse()
    rank, world = bench.setup_dist(a)
    from dasa_amd import functional as DF
    from dasa_amd import prof
    DF.reseed(1234)
    agent, env = bench.build_agent(a, rank, world)
    bench.train_step(agent)
    for _ in range(2):
        print(json.dumps(phases(agent)), flush=True)
    from dasa_amd.r2r.param import args
    for name, fn in (("teacher", lambda: (setattr(agent, "feedback", "teacher"),
                                          agent.vl_rollout(train_ml=args.ml_weight, train_rl=False))),
                     ("sample", lambda: (setattr(agent, "feedback", "sample"),
                                         agent.vl_rollout(train_ml=None, train_rl=True))),
                     ("optim", lambda: agent.optim_step())):
        if name == "teacher":
            agent.zero_grad()
        with prof.collect() as rec:
            fn()
        s = rec.summary()
        print(name, json.dumps({k: (v["launches"], v["device_ms"]) for k, v in s["kernels"].items()}), flush=True)


if __name__ == "__main__":
    main()
