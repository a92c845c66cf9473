"""DASA agent_dg policy benchmark on MI355X (BASELINE.json metric: agent decision-steps/sec at B=20,
36x2048 feats, maxAction=35).

One "step" = one training iteration of the README auglistener loop on the GT env
(agent_dg.py:1347-1372, 1389-1405): a teacher-forced rollout + a sampled A2C rollout, both through
AdaIN -> DicEncoder (9 language + 3 LXRT layers + bi-LSTM) -> decoder every step, then backward,
data-parallel gradient all-reduce (RCCL), clip and RMSprop. Episodes are synthetic 'wander' episodes
(the teacher never stops, so the teacher rollout always runs maxAction steps); the sampled rollout
stops when the policy says so, exactly as the reference. value = decisions / s where decisions =
sum over rollouts of (batched steps x B), summed over all ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 20] [--max-action 35] [--vl 3]
        (N > 1: bench.py starts the N rank processes itself, one per GPU, RCCL)
    torchrun --nproc-per-node N bench.py --gpus N ...      (the same under an external launcher)
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TF = 157.3      # MI355X_MICROARCH.md: peak FP32 matrix (= vector) rate
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E peak (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch", type=int, default=20)
    p.add_argument("--max-action", type=int, default=35)
    p.add_argument("--vl", type=int, default=3)
    p.add_argument("--viewpoints", type=int, default=64)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-fwd", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0, help="0: the CPUs this process may use (OMP_NUM_THREADS share)")
    p.add_argument("--no-profile", action="store_true")
    p.add_argument("--no-kbench", action="store_true",
                   help="skip the isolated HBM-kernel table (dasa_amd.kbench at B=20 and B=256)")
    p.add_argument("--shapes", type=int, default=0, help="add the top-N GEMM shapes by device time")
    p.add_argument("--profile-only", action="store_true",
                   help="warm-up + the HIP-event profile iteration only (for rocprofv3 runs of that iteration)")
    p.add_argument("--fast-exit", action="store_true",
                   help="os._exit after the JSON line (skips interpreter teardown; used under rocprofv3)")
    p.add_argument("--no-cfg5", action="store_true", help="skip the BASELINE configs[4] (B=256, vl=6, bf16) leg")
    p.add_argument("--no-host-input", action="store_true", help="skip the host-input (PCIe-inclusive) leg")
    p.add_argument("--no-hoist", action="store_true", help="skip the --hoist_language (non-default mode) leg")
    p.add_argument("--cfg5-only", action="store_true", help="run only the configs[4] leg (tuning)")
    p.add_argument("--only", choices=("cfg4", "cfg5", "aug"), default=None,
                   help="run only that leg and print it (the per-workload rocprofv3 --pmc passes)")
    p.add_argument("--no-cfg4", action="store_true", help="skip the configs[3] (finetune, B=2, vl=3) leg")
    p.add_argument("--no-aug", action="store_true", help="skip the full auglistener (GT + aug half) leg")
    p.add_argument("--cfg5-steps", type=int, default=6, help="decision steps per configs[4] rollout")
    p.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) | gloo (rehearsal only)")
    p.add_argument("--same-device", action="store_true",
                   help="map every rank to cuda:0 (rehearsing the DP path on a one-GPU box with gloo)")
    p.add_argument("--dist-check", action="store_true",
                   help="launch the ranks, build the process group, all-reduce once, print the world; no model")
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(a):
    """`--gpus N` (N > 1) without a launcher environment: start the N ranks here, one process per GPU,
    as torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT),
    each re-running this script with the same arguments. The parent never touches the GPU (it only
    waits), rank 0 prints the JSON line, and the exit code is the first failing rank's (the others are
    stopped). Reference DP launch: tasks/R2R/nav_dic_pretrain.py:252,765 (one process per GPU, NCCL)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:          # a failed rank leaves the others in a collective: stop them
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def setup_dist(a):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher's WORLD_SIZE is {world}", file=sys.stderr)
        sys.exit(3)
    cpu = a.dist_check and a.backend == "gloo" and not torch.cuda.is_available()
    if world > 1:
        dev = 0 if a.same_device else local
        if not cpu:
            torch.cuda.set_device(dev)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(a.backend)
        if dist.get_world_size() != a.gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {a.gpus}", file=sys.stderr)
            sys.exit(3)
    elif not cpu:
        torch.cuda.set_device(0)
    return rank, world


def dist_check(a, rank, world):
    """`--dist-check`: the launch path alone (rank processes, process group, one all-reduce), no model:
    prints {"world_size", "backend", "rank_sum"} from rank 0 (tests rehearse it with gloo on the CPU)."""
    dev = "cpu" if (a.backend == "gloo" and not torch.cuda.is_available()) else "cuda"
    t = torch.tensor([float(rank)], device=dev)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world_size": world, "n_gpus": a.gpus,
                          "backend": dist.get_backend() if world > 1 else None, "rank_sum": float(t.item())}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def build_agent(a, rank, world, finetune=False):
    from dasa_amd.r2r import param
    flags = ["--d_vl_layers", str(a.vl), "--batchSize", str(a.batch), "--maxAction", str(a.max_action)]
    (param.readme_finetune if finetune else param.readme_train)(flags)
    param.args.ml_weight = param.args.ml_weight_org     # train.py:233 (GT env)
    from dasa_amd import dp
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
    world_obj = SynthWorld(a.viewpoints, feat_seed=0, graph_seed=3)
    env = SynthR2RBatch(world_obj, a.batch, seed=1000 + rank, mode="wander", instr_len=80, lazy_features=True)
    with contextlib.redirect_stdout(io.StringIO()):
        agent = Seq2SeqAgent(env, "", None, a.max_action, "Dic")
    for m, s in ((agent.encoder, 1), (agent.decoder, 2), (agent.critic, 3), (agent.adaIn, 4)):
        init_params(m, s)        # random-init weights of the reference architecture (seeded)
    if world > 1:
        dp.attach(agent)         # broadcast from rank 0 + flat-bucket RCCL all-reduce in optim_step
    return agent, env


def train_step(agent):
    agent.zero_grad()
    agent.accumulate_gradient("sample")
    n = agent.logs["viewsteps/teacher"][-1] + agent.logs["viewsteps/sample"][-1]
    agent.optim_step()
    return n * agent.env.batch_size


def fwd_rollout(agent):
    agent.feedback = "argmax"
    for m in (agent.encoder, agent.decoder, agent.critic):
        m.eval()
    agent.loss = 0
    with torch.no_grad():
        agent.vl_rollout(train_ml=None, train_rl=False, reset=True)
    return agent.last_rollout_steps * agent.env.batch_size


def timed(fn, n, rank, world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    units = 0
    for _ in range(n):
        units += fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        u = torch.tensor([float(units)], device="cuda", dtype=torch.float64)
        dist.all_reduce(u)
        units = float(u.item())
    return units, dt


def kernel_profile(agent, fn, shapes=0):
    """One extra (untimed) iteration with HIP events around every libdasa_hip launch on its stream:
    per-kernel-family device time + algorithmic FLOPs/bytes for the roofline. It runs the timed path's
    kernels at the timed path's shapes, except that the hipGraph-captured VL stack is launched eagerly
    (graph.py: events need per-launch boundaries). Returns (summary, decisions of that iteration)."""
    from dasa_amd import prof
    with prof.collect(shapes) as rec:
        units = fn()
    return rec.summary(), units


def cpu_baseline(a):
    """BASELINE.md's CPU baseline (tools/cpu_baseline.py): the oracle's CPU restatement (oracle/policy.py)
    on bounded samples of the workloads — cfg2 train (the headline metric's iteration, maxAction 2),
    cfg2 fwd and cfg1 fwd — 1 warm-up + median of 3 on this host's CPU share."""
    from tools import cpu_baseline as CB
    r = CB.run(a.cpu_threads or None)
    w = r["workloads"]
    return {"value": w["cfg2_train"]["value"], "unit": "agent-decisions/s", "cores": r["cores"], "kind": "port",
            "cpu_model": r["cpu_model"],
            "sample": (f"oracle/policy.py {w['cfg2_train']['sample']} ({r['method']}, {r['cores']} threads, "
                       f"{r['cpu_model']})"),
            "fwd_cfg2": w["cfg2_fwd"]["value"], "fwd_cfg1": w["cfg1_fwd"]["value"], "workloads": w,
            "validation": "profiles/r02/cpu_restatement_vs_reference.json (restatement / reference in the survey "
                          "container, 8 threads: cfg2 train 0.97, cfg2 fwd 0.86, cfg1 fwd 0.70); at the headline "
                          "length (maxAction 35) profiles/r06/cpu_baseline_t35_vs_reference.json: restatement 1.96, "
                          "reference 4.82 decisions/s (0.41) - the sample above overstates the per-decision CPU "
                          "rate of the full-length iteration"}


class _HostInputEnv:
    """The env without device_input_feat: the agent takes the reference's own input path (numpy panorama /
    candidate features in the obs dicts, packed on the host and copied H2D from pinned memory every step,
    agent_dg.py:286-323)."""

    def __init__(self, env):
        self._e = env

    def __getattr__(self, k):
        if k in ("device_input_feat", "device_input_feat_steps"):
            raise AttributeError(k)
        return getattr(self._e, k)


def hoist_leg(agent, steps=2):
    """The headline iteration with --hoist_language (not a reference flag): the detached
    language stack computed once per rollout in train mode (one dropout draw per rollout instead of one
    per step; no gradient changes). A different workload than `value`: reported beside it, never as it."""
    from dasa_amd.r2r.param import args
    prev = args.hoist_language
    args.hoist_language = True
    try:
        train_step(agent)
        u, dt = timed(lambda: train_step(agent), steps, 0, 1)
    finally:
        args.hoist_language = prev
    return {"value": round(u / dt, 2), "unit": "agent-decisions/s", "ms_per_step": round(dt / steps * 1e3, 2),
            "note": "cfg2 training iteration with --hoist_language (language stack once per rollout; "
                    "non-default, not reference-faithful dropout draws)"}


def host_input_leg(a, steps=2):
    """The headline iteration with host-resident inputs (PCIe-inclusive): same config, features built on the
    host per observation and copied to the device each step. Reported beside `value`, never as it."""
    from dasa_amd.synth import SynthR2RBatch
    agent, env = build_agent(a, 0, 1)
    agent.env = _HostInputEnv(SynthR2RBatch(env.world, a.batch, seed=1000, mode="wander", instr_len=80))
    train_step(agent)
    u, dt = timed(lambda: train_step(agent), steps, 0, 1)
    return {"value": round(u / dt, 2), "unit": "agent-decisions/s", "ms_per_step": round(dt / steps * 1e3, 2),
            "note": "cfg2 training iteration with host-built observation features copied H2D (pinned) each step"}


def aug_leg(a, steps=2):
    """The WHOLE auglistener iteration of train.py:226-243 (the README --accumulateGrad loop): zero_grad;
    GT half on the bench's env (ml_weight_org: teacher + sampled rollout); aug half on a second env
    with the speaker back-translating each rollout's teacher path (speaker.py:265-350: decode word by
    word, one host sync per word) and the shared env-drop noise (ml_weight_aug: teacher + sampled
    rollout); then optim_step. The aug env holds 'goal' episodes (the speaker walks the teacher path to
    its stop); the speaker is random-init (scaled x10 so rows decode different words), so it decodes
    until <EOS> or maxDecode. Decisions = the four rollouts' batched steps x B. Beside `value`, never
    as it."""
    from dasa_amd.r2r import speaker as S
    from dasa_amd.r2r import utils
    from dasa_amd.r2r.param import args
    from dasa_amd.synth import HashBTokenizer, SynthR2RBatch, init_params, speaker_vocab
    agent, env = build_agent(a, 0, 1)
    agent.tok = HashBTokenizer(80)
    aug_env = SynthR2RBatch(env.world, a.batch, seed=3000, mode="goal", instr_len=80, lazy_features=True)
    with contextlib.redirect_stdout(io.StringIO()):
        spk = S.Speaker(aug_env, agent, utils.Tokenizer(vocab=speaker_vocab(), encoding_length=80))
    for m, s in ((spk.encoder, 61), (spk.decoder, 62)):
        init_params(m, s)
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(10.0)
    words = []
    infer = spk.infer_batch

    def infer_rec(*x, **k):
        r = infer(*x, **k)
        words.append(r.shape[1])
        return r
    spk.infer_batch = infer_rec

    def iteration():
        agent.zero_grad()
        agent.env = env
        args.ml_weight = args.ml_weight_org
        agent.accumulate_gradient("sample")
        n = agent.logs["viewsteps/teacher"][-1] + agent.logs["viewsteps/sample"][-1]
        agent.env = aug_env
        args.ml_weight = args.ml_weight_aug
        agent.accumulate_gradient("sample", speaker=spk)
        n += agent.logs["viewsteps/teacher"][-1] + agent.logs["viewsteps/sample"][-1]
        agent.optim_step()
        args.ml_weight = args.ml_weight_org
        return n * a.batch
    extra = _warm(agent, 1, step=iteration)
    words.clear()
    cap0 = _captures(agent)
    u, dt = timed(iteration, steps, 0, 1)
    res = {"workload": "full auglistener iteration (train.py:226-243): GT half + aug half (speaker "
                       "back-translation + env-drop noise, teacher + sampled rollout) + optim_step",
           "value": round(u / dt, 2), "unit": "agent-decisions/s", "ms_per_step": round(1000 * dt / steps, 2),
           "decisions_per_iteration": u / steps, "speaker_words_per_decode": words,
           "capture_warmup_iterations": extra, "train_graph_captures_in_timed": _captures(agent) - cap0}
    del agent, spk
    torch.cuda.empty_cache()
    return res


def _captures(agent):
    """Captured training regions + their backward graphs so far (graph.AutogradGraphs): a capture inside the
    timed region (a slot first seen there) is reported beside the number it slowed."""
    n = 0
    for tg in (getattr(agent, "_train_graphs", None), getattr(agent.encoder.bert, "_tgraphs", None)):
        if tg is not None:      # (the second: the finetune config's captured VisionEncoder + LXRT regions)
            n += tg.captures + tg.captures_bwd
    return n


def _warm(agent, n, world=1, step=None):
    """n untimed iterations; then, while the last one still captured training regions (graph.AutogradGraphs
    records a slot the first time a step index / padded shape occurs), up to two more, so that the timed
    iterations replay. Every rank runs the same count (the decision is all-reduced: the ranks' episodes
    differ, and optim_step's gradient all-reduce needs them in step). Returns the extra count."""
    step = step or (lambda: train_step(agent))
    last = 0
    for _ in range(n):
        c = _captures(agent)
        step()
        last = _captures(agent) - c
    extra = 0
    while n > 0 and extra < 2:
        flag = torch.tensor([float(last > 0)], device=torch.device("cuda", torch.cuda.current_device()))
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item() == 0:
            break
        c = _captures(agent)
        step()
        last = _captures(agent) - c
        extra += 1
    return extra


def _collect():
    """Between bench legs: collect the previous leg's agent (reference cycles through its graphs and hooks)
    and return its cached blocks, so each leg's host-bound loop starts without the others' live objects."""
    import gc
    gc.collect()
    torch.cuda.empty_cache()


def cfg4_leg(a, steps=3):
    """BASELINE configs[3] per rank: the README finetune iteration (README.md:104-116:
    --d_update_add_layer True, so the LXRT layers and the VisionEncoder train; d_vl_layers 3, batchSize 2,
    maxAction 35, lr 2e-6, no LR scheduler), teacher + sampled rollout, backward, RMSprop, on one GPU
    (the 8-rank DP form is the driver's scaling run). Kernel table + roofline of the dominant family
    from an extra HIP-event iteration, PMC values only from this workload's own rocprofv3 passes."""
    from types import SimpleNamespace
    from dasa_amd import prof
    c = SimpleNamespace(**vars(a))
    c.batch, c.vl = 2, 3
    agent, _ = build_agent(c, 0, 1, finetune=True)
    assert agent.encoder.bert.update_add_layer
    extra = _warm(agent, max(1, a.warmup))
    cap0 = _captures(agent)
    u, dt = timed(lambda: train_step(agent), steps, 0, 1)
    res = {"workload": "configs[3] per rank: README finetune iteration (d_update_add_layer, vl=3, B=2, "
                       f"maxAction {c.max_action}, teacher + sample rollout, backward, RMSprop)",
           "value": round(u / dt, 2), "unit": "agent-decisions/s", "ms_per_step": round(1000 * dt / steps, 2),
           "warmup": max(1, a.warmup), "capture_warmup_iterations": extra,
           "train_graph_captures_in_timed": _captures(agent) - cap0}
    with prof.collect(a.shapes) as rec:
        train_step(agent)
    summ = rec.summary(pmc_workload="cfg4")
    res["roofline"] = summ["roofline"]
    res["kernels"] = dict(list(summ["kernels"].items())[:8])
    if "shapes" in summ:
        res["shapes"] = summ["shapes"]
    del agent
    torch.cuda.empty_cache()
    return res


def cfg5_leg(a):
    """BASELINE configs[4]: B=256, d_vl_layers=6, 36x2048 synthetic feats, forward (eval/argmax rollout)
    with bf16 GEMM operands and fp32 accumulation (ops.bf16_matmul); the same rollout in fp32 beside it.
    A decision step here is one batched step of 256 agents; the roofline is the bf16 GEMM family's."""
    from types import SimpleNamespace
    from dasa_amd import ops, prof
    c = SimpleNamespace(**vars(a))
    c.batch, c.vl, c.max_action = 256, 6, a.cfg5_steps
    agent, _ = build_agent(c, 0, 1)
    res = {"workload": f"configs[4]: eval/argmax rollout, B=256, vl=6, la=9, L=80, {c.max_action} steps, "
                       "36x2048 synthetic feats", "unit": "agent-decisions/s"}
    for mode in ("bf16", "fp32"):
        def run():
            if mode == "bf16":
                with torch.no_grad(), ops.bf16_matmul():
                    return fwd_rollout(agent)
            return fwd_rollout(agent)
        run()
        u, dt = timed(run, 2, 0, 1)
        ent = {"value": round(u / dt, 2), "ms_per_step": round(1000 * dt * c.batch / u, 2)}
        with prof.collect() as rec:
            run()
        summ = rec.summary(pmc_workload="cfg5")
        ent["kernels"] = {k: v for k, v in summ["kernels"].items() if k in ("gemm", "gemm_x6", "gemm_bf16", "mha",
                                                                              "bilstm", "layernorm", "elementwise")}
        fam = "gemm_bf16" if mode == "bf16" else ("gemm_x6" if "gemm_x6" in summ["kernels"] else "gemm")
        if fam in summ["kernels"]:
            k = summ["kernels"][fam]
            ent["roofline"] = {"kernel": fam, "bound": "mfma", "achieved": k["achieved"], "peak": k["peak"],
                               "unit": "TFLOP/s", "frac": k["frac"]}
            if summ["roofline"]["kernel"] == fam and summ["roofline"].get("traffic") is not None:
                for key in ("traffic", "mfma_busy", "traffic_source"):
                    if key in summ["roofline"]:
                        ent["roofline"][key] = summ["roofline"][key]
        res[mode] = ent
    res["dtype_note"] = ("bf16: nn.Linear operands bf16 (weights converted once; activations handed on as bf16 by "
                         "their producers - LayerNorm twin, GELU, attention core - or rounded on load), Q/K/V and the "
                         "attention core bf16 (P rounded to bf16), the B=256 bi-LSTM recurrence on bf16 W_hh / h; "
                         "fp32 accumulation, epilogues, softmax, LayerNorm statistics and the residual stream")
    del agent
    torch.cuda.empty_cache()
    return res


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))        # before any GPU call in this process
    rank, world = setup_dist(a)
    if a.dist_check:
        dist_check(a, rank, world)
        return
    torch.manual_seed(1 + rank)
    from dasa_amd import functional as DF
    DF.reseed(1234 + rank)
    if a.cfg5_only or a.only == "cfg5":
        print(json.dumps({"cfg5": cfg5_leg(a)}), flush=True)
        return
    if a.only == "cfg4":
        print(json.dumps({"cfg4": cfg4_leg(a)}), flush=True)
        return
    if a.only == "aug":
        print(json.dumps({"aug": aug_leg(a)}), flush=True)
        return
    agent, env = build_agent(a, rank, world)
    extra = _warm(agent, a.warmup, world)
    if a.profile_only:
        summ, punits = kernel_profile(agent, lambda: train_step(agent), a.shapes)
        print(json.dumps({"profile_only": True, "decisions": punits, **summ}), flush=True)
        return
    cap0 = _captures(agent)
    units, dt = timed(lambda: train_step(agent), a.steps, rank, world)
    cap_timed = _captures(agent) - cap0
    value = units / dt
    out = {
        "metric": "agent decision-steps/sec at B=20, 36x2048 feats, maxAction=35; 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "agent-decisions/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 2),
        "batched_steps_per_s": round(value / (a.batch * world), 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": "cfg2 training iteration on the GT env: accumulate_gradient('sample') (teacher + "
                               "sampled rollout) + optim_step (backward, " +
                               ("RCCL grad all-reduce, " if world > 1 else "") + "clip, RMSprop), README flags; "
                               "the GT half of train.py's auglistener loop (the full loop: `auglistener`)",
                   "global_batch": a.batch * world, "per_rank_batch": a.batch, "max_action": a.max_action,
                   "instr_len": 80, "vl_layers": a.vl, "la_layers": 9, "parallelism": f"dp{world}",
                   "world_size": world, "backend": (dist.get_backend() if world > 1 else None)},
        "train_graph_captures_in_timed": cap_timed, "capture_warmup_iterations": extra,
    }
    if not a.no_fwd:
        fwd_rollout(agent)
        fu, fdt = timed(lambda: fwd_rollout(agent), 2, rank, world)
        out["fwd_value"] = round(fu / fdt, 2)
        out["fwd_note"] = "eval/argmax rollout decisions/s (language stack computed once per batch: exact in eval)"
    if not a.no_profile:
        summ, punits = kernel_profile(agent, lambda: train_step(agent), a.shapes)
        if rank == 0:
            out.update(summ)
            # whole-iteration roofline: the algorithmic FLOPs of every launch of one iteration (GEMMs,
            # attention, recurrences; fp32-equivalent) per decision x the timed decisions/s, vs fp32 peak
            fpd = summ["profiled_alg_flops"] / max(1, punits)
            ach = fpd * value / 1e12
            out["whole_step"] = {"alg_gflop_per_decision": round(fpd / 1e9, 3), "achieved": round(ach, 2),
                                 "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TF, 4),
                                 "note": "sum of per-launch algorithmic FLOPs of the profiled iteration / its "
                                         "decisions x timed decisions/s"}
    if rank == 0 and world == 1 and not a.no_kbench:
        from dasa_amd import kbench
        out["hbm_kernels"] = kbench.hbm_kernels((a.batch, 256))
        out["hbm_kernels_note"] = ("AdaIN gate / mu-sigma and attention kernels in isolation, graph-replayed back to back "
                                   "(no host gaps); B=256 is BASELINE configs[4]'s batch; algorithmic bytes / time vs 8 TB/s")
    if rank == 0 and world == 1 and not a.no_hoist:
        out["hoist_language"] = hoist_leg(agent)
    if rank == 0 and world == 1:
        # the remaining legs build their own agents: free the cfg2 agent (and its captured graphs) first, so
        # their host-bound iterations do not pay for its live objects in every GC pass or share its pools
        del agent, env
        _collect()
    if rank == 0 and world == 1 and not a.no_host_input:
        out["host_input"] = host_input_leg(a)
        _collect()
    if rank == 0 and world == 1 and not a.no_aug:
        out["auglistener"] = aug_leg(a)
        _collect()
    if rank == 0 and world == 1 and not a.no_cfg4:
        out["cfg4"] = cfg4_leg(a)
        _collect()
    if rank == 0 and world == 1 and not a.no_cfg5:
        out["cfg5"] = cfg5_leg(a)
        _collect()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if a.fast_exit:
        torch.cuda.synchronize()
        sys.stdout.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
