"""CPU baseline of the policy path (BASELINE.md "CPU baseline"): the oracle's from-scratch CPU
restatement (oracle/policy.py, test infrastructure — the checker, never the product) timed on the
host's cores on bounded samples of the benchmark workloads:

  * cfg2 train: accumulate_gradient('sample') + backward (teacher + sampled rollout), B=20, vl=3,
    L=80, maxAction 2 (the per-step cost is flat in T: every step re-runs the full encoder);
  * cfg2 fwd:   eval / no_grad rollout, B=20, vl=3, L=80, 5 steps, language stack recomputed every
    step as the reference does (agent_dg.py:793 -> vilmodel.py:1366-1372);
  * cfg1 fwd:   B=2, vl=1, 5 steps.

torch.set_num_threads(cores), 1 warm-up + median of 3 timed runs each. `cores` defaults to the CPUs
this process may run on (the GPU box grants a share of its host: OMP_NUM_THREADS there).

    python tools/cpu_baseline.py [--cores N] [--reference]   # --reference: also time the reference
                                                             # itself (survey container only)
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def default_cores():
    env = os.environ.get("OMP_NUM_THREADS")
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    if env and env.isdigit() and int(env) > 0:
        return min(int(env), aff)
    return aff


def _median_rate(fn, reps=3):
    fn()                                   # warm-up
    rates, times = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        n = fn()
        dt = time.perf_counter() - t0
        rates.append(n / dt)
        times.append(dt)
    return statistics.median(rates), times


def oracle_workloads(viewpoints=64):
    """name -> callable running one sample with the oracle; returns decisions made."""
    from oracle import policy as O
    from tests.helpers import oracle_weights
    from dasa_amd.synth import SynthR2RBatch, SynthWorld
    world = SynthWorld(viewpoints, 0, 3)
    W3 = oracle_weights(3, requires_grad=True)
    for k, v in W3.enc.items():          # the BERT stack is detached in the train config
        if k.startswith("bert."):
            v.requires_grad_(False)
    W3e = oracle_weights(3)
    W1 = oracle_weights(1)
    env20 = SynthR2RBatch(world, 20, seed=1000, mode="wander", instr_len=80)
    env2 = SynthR2RBatch(world, 2, seed=1001, mode="wander", instr_len=80)

    def train_cfg2(T=2):
        r1 = O.vl_rollout(W3, env20, "teacher", la_layers=9, vl_layers=3, episode_len=T, train=True, train_ml=0.4)
        r2 = O.vl_rollout(W3, env20, "sample", la_layers=9, vl_layers=3, episode_len=T, train=True, train_rl=True)
        (r1["loss"] + r2["loss"]).backward()
        for d in (W3.enc, W3.dec, W3.critic, W3.ada):
            for v in d.values():
                v.grad = None
        return (r1["steps"] + r2["steps"]) * 20

    def fwd(W, env, vl, B, T=5):
        with torch.no_grad():
            r = O.vl_rollout(W, env, "argmax", la_layers=9, vl_layers=vl, episode_len=T, hoist_lang=False)
        return r["steps"] * B

    return {"cfg2_train": (train_cfg2, "teacher + sampled rollout + backward, B=20, vl=3, L=80, maxAction=2"),
            "cfg2_train_35": (lambda: train_cfg2(35),
                              "teacher + sampled rollout + backward, B=20, vl=3, L=80, maxAction=35 (the headline length)"),
            "cfg2_fwd": (lambda: fwd(W3e, env20, 3, 20), "eval rollout, B=20, vl=3, L=80, 5 steps"),
            "cfg1_fwd": (lambda: fwd(W1, env2, 1, 2), "eval rollout, B=2, vl=1, L=80, 5 steps")}


def run(cores=None, which=("cfg2_train", "cfg2_fwd", "cfg1_fwd"), reps=3):
    cores = cores or default_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        wl = oracle_workloads()
        res = {}
        for name in which:
            fn, desc = wl[name]
            rate, times = _median_rate(fn, reps)
            res[name] = {"value": round(rate, 3), "unit": "agent-decisions/s", "sample": desc,
                         "times_s": [round(t, 2) for t in times]}
        return {"cores": cores, "cpu_model": cpu_model(), "kind": "port", "workloads": res,
                "method": f"1 warm-up + median of {reps}; torch.set_num_threads(cores); oracle/policy.py (CPU restatement)"}
    finally:
        torch.set_num_threads(prev)


def reference_rates(cores, which=("cfg2_train", "cfg2_fwd", "cfg1_fwd"), reps=3):
    """Survey container only: the reference r2r_src itself (imported behind the offline shims) on the
    same bounded samples, to validate the restatement as a timing proxy."""
    import contextlib
    import io
    from oracle.golden.refimport import import_reference
    from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
    torch.set_num_threads(cores)
    R = import_reference()
    A = R.args
    world = SynthWorld(64, 0, 3)
    out = {}

    def agent(B, vl, T, seed):
        A.d_vl_layers, A.batchSize, A.maxAction, A.views = vl, B, T, 36
        env = SynthR2RBatch(world, B, seed=seed, mode="wander", instr_len=80)
        with contextlib.redirect_stdout(io.StringIO()):
            ag = R.agent_dg.Seq2SeqAgent(env, "", None, T, "Dic")
        for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
            init_params(m, s)
        return ag

    for name, T in (("cfg2_train", 2), ("cfg2_train_35", 35)):
        if name not in which:
            continue
        ag = agent(20, 3, T, 1000)
        A.ml_weight = A.ml_weight_org

        def train(ag=ag):
            ag.zero_grad()
            ag.accumulate_gradient("sample")
            ag.loss.backward()
            return (ag.logs["viewsteps/teacher"][-1] + ag.logs["viewsteps/sample"][-1]) * 20
        out[name] = _median_rate(train, reps)[0]
    for name, (B, vl) in (("cfg2_fwd", (20, 3)), ("cfg1_fwd", (2, 1))):
        if name not in which:
            continue
        agf = agent(B, vl, 5, 1001)

        def fwd(agf=agf, B=B):
            for m in (agf.encoder, agf.decoder, agf.critic):
                m.eval()
            agf.feedback = "argmax"
            agf.loss = 0
            with torch.no_grad():
                agf.vl_rollout(train_ml=None, train_rl=False, reset=True)
            return agf.logs["viewsteps/argmax"][-1] * B
        out[name] = _median_rate(fwd, reps)[0]
    return {k: round(v, 3) for k, v in out.items()}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cores", type=int, default=0)
    ap.add_argument("--reference", action="store_true")
    ap.add_argument("--workloads", default="cfg2_train,cfg2_fwd,cfg1_fwd")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    which = tuple(a.workloads.split(","))
    res = run(a.cores or None, which, a.reps)
    if a.reference:
        res["reference"] = reference_rates(res["cores"], which, a.reps)
        res["restatement_over_reference"] = {k: round(res["workloads"][k]["value"] / v, 3)
                                             for k, v in res["reference"].items()}
    print(json.dumps(res, indent=1))
