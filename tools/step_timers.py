"""Host wall-clock per phase of the cfg2 training iteration (the sampled rollout's GPU idles
~0.6 ms per late step while the host syncs on the action, steps the env and stages the next step; r06 trace,
profiles/r06/timeline_r06c.txt). Wraps the agent's per-step methods with perf_counter accumulators (no
cProfile: its per-call overhead would swamp ~100 us phases) and prints calls / total / mean per phase.
    python tools/step_timers.py [iterations]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ACC = collections.defaultdict(lambda: [0, 0.0])


def wrap(obj, name, label=None):
    fn = getattr(obj, name)
    label = label or f"{type(obj).__name__}.{name}"

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            e = ACC[label]
            e[0] += 1
            e[1] += time.perf_counter() - t0
    setattr(obj, name, w)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sys.argv = sys.argv[:1]
    a = bench.parse()
    import torch
    torch.cuda.set_device(0)
    agent, _ = bench.build_agent(a, 0, 1)
    bench._warm(agent, 2)
    torch.cuda.synchronize()
    for name in ("make_equiv_action", "_step_reward", "_teacher_action_np", "_to_dev", "_step_inputs",
                 "_adain_decode", "_encode_steps", "_decode", "_graph_step", "get_input_feat", "_lens_dev",
                 "_teacher_plan", "_fused_head"):
        if hasattr(agent, name):
            wrap(agent, name)
    wrap(agent.env, "_get_obs", "env._get_obs")
    wrap(agent.encoder, "forward", "encoder.forward")
    wrap(agent.encoder.bert, "forward", "bert.forward (LXRT region)")
    from dasa_amd.r2r import r2rmodel
    from dasa_amd import functional as DF
    wrap(r2rmodel._LangPipe, "pump", "_LangPipe.pump")
    wrap(r2rmodel._LangPipe, "take", "_LangPipe.take")
    wrap(DF.BiLSTMFn, "apply", "BiLSTMFn.apply")
    # (not agent.decoder.forward: a wrapped forward makes the agent run the decoder eagerly, _train_graph_ok)
    store = getattr(agent.env, "_store", None)
    if store is not None:   # the device feature store's host staging (DeviceFeatureEnv)
        wrap(store, "_step_arrays", "store._step_arrays")
        wrap(store, "input_feat_steps", "store.input_feat_steps")
    from dasa_amd import ops
    wrap(ops, "gather_rows", "ops.gather_rows")
    orig_pin = torch.Tensor.pin_memory

    def pin(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return orig_pin(self, *a, **k)
        finally:
            e = ACC["Tensor.pin_memory"]
            e[0] += 1
            e[1] += time.perf_counter() - t0
    torch.Tensor.pin_memory = pin
    orig_cpu = torch.Tensor.cpu

    def cpu(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return orig_cpu(self, *a, **k)
        finally:
            e = ACC["Tensor.cpu (device sync)"]
            e[0] += 1
            e[1] += time.perf_counter() - t0
    torch.Tensor.cpu = cpu
    t0 = time.perf_counter()
    for _ in range(n):
        bench.train_step(agent)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    torch.Tensor.cpu = orig_cpu
    torch.Tensor.pin_memory = orig_pin
    print(f"{n} iterations, {wall / n * 1e3:.1f} ms each")
    print(f"{'phase':42s} {'calls/it':>9s} {'ms/it':>8s} {'us/call':>8s}")
    for k, (c, s) in sorted(ACC.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:42s} {c / n:9.1f} {s / n * 1e3:8.2f} {s / c * 1e6:8.1f}")


if __name__ == "__main__":
    main()
