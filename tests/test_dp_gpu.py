"""Data-parallel training of the real agent (BASELINE configs[2]) on the GPU box.

Two ranks share the one GPU over gloo (the 8-GPU RCCL run belongs to the driver). Each rank builds
the cfg2 agent (B=20, vl=3; dropout 0, maxAction 3; the one-kernel policy head of the timed path with
the sampled draws from a forced table), `dp.attach(agent)`, and runs two optimizer steps on its own
episodes (env seed differs per rank). After each step:
  (a) every parameter is bitwise identical on both ranks;
  (b) the synchronised gradient equals the mean of the two ranks' own gradients (each rank's
      pre-sync gradient is captured in-process and exchanged for the check);
  (c) the set of parameters left with grad=None equals the single-rank set.
The persistent bi-LSTM needs every CU to itself, so the two ranks that share the device use the
per-timestep LSTM kernels (DASA_LSTM_MODE=1). test_dp_rccl_world1_persistent runs the collective
path over RCCL ("nccl") at world size 1 with the default persistent bi-LSTM instead.
Reference: agent_dg.py:1389-1405 (optim_step); tasks/R2R/nav_dic_pretrain.py:252,765 (the reference's
own NCCL process group).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DASA_LSTM_MODE="1")
    import contextlib
    import io
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dasa_amd import dp
        from dasa_amd.r2r import param
        param.readme_train(["--d_vl_layers", "3", "--batchSize", "20", "--maxAction", "3"])
        param.args.ml_weight = param.args.ml_weight_org
        from dasa_amd.r2r.agent_dg import Seq2SeqAgent
        from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
        torch.manual_seed(1)                   # the same seed on every rank, as train.py:521 does
        env = SynthR2RBatch(SynthWorld(32, 0, 5), 20, seed=500 + rank, mode="goal", instr_len=80, variable_len=True)
        with contextlib.redirect_stdout(io.StringIO()):
            ag = Seq2SeqAgent(env, "", None, 3, "Dic")
        # replicas start DIFFERENT (rank-specific weights) until dp.attach broadcasts rank 0's
        for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
            init_params(m, s + 100 * rank)
            for sub in m.modules():
                if isinstance(sub, torch.nn.Dropout):
                    sub.p = 0.0
        from tests import golden_inputs as GI
        table = GI.forced_table(3, 20, seed=GI.FORCED_SEED + rank)
        ag.sample_fn = None
        ag.force_action_fn = lambda t, lens: GI.forced_actions(table, t, lens)
        heads = []
        from dasa_amd import functional as DF
        orig_head = DF.policy_head
        DF.policy_head = lambda *a, **k: (heads.append(a[3]), orig_head(*a, **k))[1]
        sync = dp.attach(ag)
        assert sync is not None and sync.world == world
        named = [(f"{i}.{k}", p) for i, m in enumerate(ag.models) for k, p in m.named_parameters()]
        captured = {}
        inner = ag.grad_sync

        def capturing_sync():
            captured["local"] = {k: (p.grad.detach().clone() if p.grad is not None else None) for k, p in named}
            inner()     # (clip_grad_norm_ then scales .grad in place: keep the synchronised values)
            captured["synced"] = {k: (p.grad.detach().clone() if p.grad is not None else None) for k, p in named}
        ag.grad_sync = capturing_sync
        report = []
        for step in range(2):
            ag.zero_grad()
            ag.accumulate_gradient("sample")
            ag.optim_step()
            torch.cuda.synchronize()
            local = captured["local"]
            none_local = sorted(k for k, g in local.items() if g is None)
            synced = captured["synced"]
            none_after = sorted(k for k, g in synced.items() if g is None)
            # exchange the pre-sync gradients and the post-step parameters (CPU tensors over gloo)
            max_grad_err, n_grads = 0.0, 0
            for k, p in named:
                if local[k] is None:
                    continue
                mine = local[k].float().cpu()
                bufs = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(bufs, mine)
                mean = (bufs[0] + bufs[1]) / 2
                err = (synced[k].float().cpu() - mean).abs().max().item()
                max_grad_err = max(max_grad_err, err / max(1e-30, mean.abs().max().item()))
                n_grads += 1
            params_equal = True
            for k, p in named:
                mine = p.detach().float().cpu()
                bufs = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(bufs, mine)
                params_equal = params_equal and torch.equal(bufs[0], bufs[1])
            report.append(dict(step=step, none_local=none_local, none_after=none_after, n_grads=n_grads,
                               max_grad_rel_err=max_grad_err, params_equal=params_equal,
                               finite=all(torch.isfinite(p).all().item() for _, p in named),
                               losses=list(ag.logs["ml_loss"][-2:]),
                               fused_heads=sorted(set(heads))))
        q.put((rank, report, None))
        dist.barrier()
    except Exception as e:   # report instead of hanging the peer
        import traceback
        q.put((rank, None, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_dp_agent_two_ranks_same_gpu(dev):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, rep, err = q.get(timeout=240)
            assert err is None, f"rank {r} failed:\n{err}"
            res[r] = rep
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    for step in range(2):
        a, b = res[0][step], res[1][step]
        assert a["params_equal"] and b["params_equal"], "replicas diverged after optim_step"
        assert a["finite"] and b["finite"]
        assert a["n_grads"] == b["n_grads"] >= 30
        # exact: gloo's sum of two fp32 addends, then / 2 — same as the host mean
        assert a["max_grad_rel_err"] <= 1e-6 and b["max_grad_rel_err"] <= 1e-6, (a, b)
        assert a["none_after"] == a["none_local"] == b["none_after"] == b["none_local"]
        assert a["losses"] != b["losses"], "the ranks must have run different episodes"
        assert a["fused_heads"] == b["fused_heads"] == ["forced", "teacher"]   # the timed path's head


def _rank_rccl(port, q):
    """World size 1 over RCCL: the collective path (mask + bucket all-reduce, / world) inside optim_step
    with the DEFAULT persistent bi-LSTM, the fused head and the batched BPTT."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("DASA_LSTM_MODE", None)
    import contextlib
    import io
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        from dasa_amd import dp, ops
        from dasa_amd.r2r import param
        from tests import golden_inputs as GI
        param.readme_train(["--d_vl_layers", "3", "--batchSize", "20", "--maxAction", "4"])
        param.args.ml_weight = param.args.ml_weight_org
        from dasa_amd.r2r.agent_dg import Seq2SeqAgent
        from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
        torch.manual_seed(1)
        env = SynthR2RBatch(SynthWorld(32, 0, 5), 20, seed=600, mode="wander", instr_len=80, variable_len=True)
        with contextlib.redirect_stdout(io.StringIO()):
            ag = Seq2SeqAgent(env, "", None, 4, "Dic")
        for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
            init_params(m, s)
        table = GI.forced_table(4, 20)
        ag.force_action_fn = lambda t, lens: GI.forced_actions(table, t, lens, no_stop=True)
        fwd_rows = []
        orig = ops.bilstm_fwd
        ops.bilstm_fwd = lambda x, *a, **k: (fwd_rows.append(x.shape[0]), orig(x, *a, **k))[1]
        sync = dp.attach(ag, force=True)
        assert sync is not None and sync.world == 1
        named = [(f"{i}.{k}", p) for i, m in enumerate(ag.models) for k, p in m.named_parameters()]
        captured = {}
        inner = ag.grad_sync

        def capturing_sync():
            captured["local"] = {k: p.grad.detach().clone() for k, p in named if p.grad is not None}
            inner()
            captured["synced"] = {k: p.grad.detach().clone() for k, p in named if p.grad is not None}
        ag.grad_sync = capturing_sync
        rep = []
        for _ in range(2):
            ag.zero_grad()
            ag.accumulate_gradient("sample")
            ag.optim_step()            # raises on a persistent-kernel barrier timeout (error word)
            torch.cuda.synchronize()
            loc, syn = captured["local"], captured["synced"]
            rep.append(dict(same_keys=sorted(loc) == sorted(syn), n=len(loc), recv=sum(g.numel() for g in loc.values()), sent=sync.sent,
                            bitwise=all(torch.equal(loc[k], syn[k]) for k in loc),
                            finite=all(torch.isfinite(p).all().item() for _, p in named)))
        q.put((dict(numel=sync.numel, trainable=sum(t.numel() for t in dp._trainable(ag)), steps=rep, fwd_rows=sorted(set(fwd_rows)),
                    lstm_mode=os.environ.get("DASA_LSTM_MODE")), None))
    except Exception:
        import traceback
        q.put((None, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_rccl_world1_persistent(dev):
    """RCCL ("nccl" = RCCL on ROCm) opened on the GPU box: GradSync over the real bucket (every trainable
    parameter; 47.23 M of its floats receive a gradient) inside optim_step, with the persistent bi-LSTM kernels on (teacher chunks at 80 / 160 rows, sampled
    steps at 20). After sum / 1 every gradient is bitwise the rank's own; no barrier timeout."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_rccl, args=(_free_port(), q))
    p.start()
    try:
        res, err = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert p.exitcode == 0
    assert res["numel"] == res["trainable"], res
    assert res["lstm_mode"] is None and 20 in res["fwd_rows"], res
    for st in res["steps"]:
        assert st["same_keys"] and st["n"] >= 30 and st["bitwise"] and st["finite"], st
        assert 47.2e6 < st["recv"] < 47.3e6, st        # 47.23 M gradient-receiving floats
        assert st["sent"] == st["recv"], st             # only those travel in the all-reduce
