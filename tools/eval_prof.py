"""Per-family device time of one eval/argmax rollout at the headline config (B=20, vl=3, maxAction=35)
next to its wall time: what bounds the forward-only decision step.

    python tools/eval_prof.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    torch.cuda.set_device(0)
    agent, _ = bench.build_agent(a, 0, 1)
    bench.fwd_rollout(agent)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = bench.fwd_rollout(agent)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    from dasa_amd import prof
    with prof.collect(20) as rec:
        n2 = bench.fwd_rollout(agent)
    s = rec.summary()
    out = {"wall_ms": round(wall * 1e3, 2), "decisions": n, "steps": n // a.batch,
           "profiled_decisions": n2, "profiled_device_ms": s["profiled_device_ms"],
           "families": {k: (v["launches"], v["device_ms"], v["avg_launch_us"]) for k, v in s["kernels"].items()},
           "shapes": s.get("shapes")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
