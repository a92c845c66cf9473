"""Captured training decision steps (dasa_amd.graph.AutogradGraphs): the decoder step +
one-kernel policy head of a training rollout replays as a hipGraph recorded with autograd, and its
backward runs the recorded autograd graph.

* dropout / Categorical draws inside a replay are fresh per replay, and the backward regenerates the
  forward's masks (the slot's device seed counter is the seed source of both);
* a cfg2 training iteration (B=20, vl=3, 4 + 4 steps, dropout 0, forced draws) gives the same losses
  and the same gradients with the capture as eagerly, over two iterations with RMSprop steps in
  between (in-place parameter updates are read by the replays; no re-capture);
* slots: one per (rollout, step) — captured in the first iteration, only replayed after.
Reference: agent_dg.py:725-936 (the step loop), 1389-1405 (optim_step)."""
import contextlib
import io

import numpy as np
import pytest
import torch

from tests import golden_inputs as GI

pytestmark = pytest.mark.gpu


def test_autograd_graph_dropout_masks(dev):
    from dasa_amd import functional as DF
    from dasa_amd import graph
    g = graph.AutogradGraphs([])
    x = torch.ones(64, 1024, device=dev, requires_grad=True)

    def fn(x):
        return (DF.dropout(x, 0.5, True),)
    outs = []
    for it in range(3):
        g.new_iteration()
        (y,) = g.run("drop", fn, (x,))
        y.backward(torch.ones_like(y))
        outs.append(y.detach().clone())
        # d/dx sum(mask / (1 - p) * x) = mask / (1 - p) = y (x = 1): the backward used the replay's mask
        assert torch.equal(x.grad, y.detach()), it
        x.grad = None
    assert g.captures == 1 and g.replays == 3
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])   # fresh masks per replay
    keep = (outs[0] != 0).float().mean().item()
    assert 0.45 < keep < 0.55


def test_autograd_graph_sampling_fresh_per_replay(dev):
    from dasa_amd import functional as DF
    from dasa_amd import graph
    g = graph.AutogradGraphs([])
    logit = torch.zeros(256, 16, device=dev, requires_grad=True)
    lens = torch.full((256,), 16, dtype=torch.int32, device=dev)

    def fn(logit, lens):
        return DF.policy_head(logit, lens, None, "sample")
    acts = []
    for _ in range(2):
        g.new_iteration()
        ce, ent, lpa, act = g.run("head", fn, (logit, lens))
        acts.append(act.cpu())
        lpa.sum().backward()
        # uniform logits: d log p(a) / dz_j = onehot_a - 1/16, summed over rows
        want = torch.zeros(256, 16)
        want[torch.arange(256), act.cpu()] = 1.0
        want -= 1.0 / 16
        assert torch.allclose(logit.grad.cpu(), want, atol=1e-6)
        logit.grad = None
    assert not torch.equal(acts[0], acts[1])


def _agent(seed_env):
    from dasa_amd.r2r import param
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
    env = SynthR2RBatch(SynthWorld(32, 0, 5), 20, seed=seed_env, mode="wander", instr_len=80, variable_len=True)
    with contextlib.redirect_stdout(io.StringIO()):
        ag = Seq2SeqAgent(env, "", None, 4, "Dic")
    for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
        init_params(m, s)
        for sub in m.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    param.args.ml_weight = param.args.ml_weight_org
    return ag


def _iteration(ag, it):
    from dasa_amd import functional as DF
    table = GI.forced_table(4, 20, seed=GI.FORCED_SEED + it)
    ag.force_action_fn = lambda t, lens: GI.forced_actions(table, t, lens, no_stop=True)
    ag.zero_grad()
    ag.accumulate_gradient("sample")
    loss = ag.loss.item()
    with DF.defer_bilstm_backward(), DF.defer_weight_grads():
        ag.loss.backward()
    DF.flush_bilstm_backward()
    DF.flush_weight_grads()
    grads = {f"{i}.{k}": p.grad.detach().clone() for i, m in enumerate(ag.models) for k, p in m.named_parameters()
             if p.grad is not None}
    for opt in ag.optimizers:
        opt.step()
    if ag._train_graphs is not None:
        ag._train_graphs.new_iteration()
    return loss, list(ag.logs["entropy"][-4:]), grads


@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream does not match")
def test_train_graph_matches_eager(dev, monkeypatch):
    """... and without torch's AccumulateGrad stream-mismatch warning (the captured
    backward feeding accumulators of another stream), here an error."""
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "3", "--batchSize", "20", "--maxAction", "4"])
    try:
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("DASA_TRAIN_GRAPH", mode)
            torch.manual_seed(3)
            ag = _agent(700)
            res[mode] = [_iteration(ag, it) for it in range(2)]
            if mode == "1":
                tg = ag._train_graphs
                assert tg is not None and tg.captures == 8 and len(tg.slots) == 8, (tg and tg.captures)
                assert tg.replays == 16
                from dasa_amd import graph as G
                # every slot's backward captured once (iteration 0) and replayed after
                assert tg.captures_bwd == (8 if G.BWD_GRAPH else 0), tg.captures_bwd
            else:
                assert ag._train_graphs is None
            del ag
        for it in range(2):
            (l0, e0, g0), (l1, e1, g1) = res["0"][it], res["1"][it]
            assert abs(l0 - l1) <= 1e-6 * max(1.0, abs(l0)), (it, l0, l1)
            assert np.allclose(e0, e1, rtol=1e-6, atol=0), (it, e0, e1)
            assert sorted(g0) == sorted(g1)
            for k in g0:
                err = (g0[k] - g1[k]).abs().max().item()
                assert err <= 1e-5 * max(1e-30, g0[k].abs().max().item()), (it, k, err)
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


@pytest.mark.parametrize("bwd_graph", [True, False])
def test_captured_backward_regenerates_replay_masks(dev, monkeypatch, bwd_graph):
    """a captured region WITH dropout (p = 0.3 on the input, 0.2 on the output of a linear): the
    gradient its backward returns (captured backward graph, or the recorded autograd graph run eagerly) is
    the gradient of the forward the replay computed, masks included. The region is linear in x for fixed
    masks, so <dx, d> must equal <gy, y(x + d) - y(x)> with y(x + d) replayed on the SAME masks (the slot's
    seed counter stepped back by the one bump a replay adds). A backward that regenerated other masks than
    the replay drew fails by O(1)."""
    from dasa_amd import functional as DF
    from dasa_amd import graph
    monkeypatch.setattr(graph, "BWD_GRAPH", bwd_graph)
    torch.manual_seed(5)
    lin = torch.nn.Linear(256, 128).to(dev)
    g = graph.AutogradGraphs([lin])
    x = torch.randn(64, 256, device=dev, requires_grad=True)

    def fn(x):
        h = DF.dropout(x, 0.3, True)
        y = DF.linear(h, lin.weight, lin.bias)
        return (DF.dropout(y, 0.2, True),)
    seen = []
    for it in range(3):            # capture (+ backward capture), then replays of both
        g.new_iteration()
        (y,) = g.run("r", fn, (x,))
        gy = torch.randn_like(y)
        x.grad = None
        y.backward(gy)
        gx = x.grad.detach().clone()
        d = torch.randn_like(x)
        slot = next(iter(g.slots.values()))
        slot.counter.sub_(1)       # the next replay draws this replay's masks again
        g.new_iteration()
        with torch.no_grad():
            (y2,) = g.run("r", fn, (x.detach() + d,))
        lhs = (gx.double() * d.double()).sum().item()
        rhs = (gy.double() * (y2.double() - y.detach().double())).sum().item()
        assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(rhs)), (it, lhs, rhs)
        seen.append(y.detach().clone())
        assert lin.weight.grad is not None          # parameter gradients reach the real parameters
        lin.weight.grad = None
        lin.bias.grad = None
    assert g.captures == 1 and g.captures_bwd == (1 if bwd_graph else 0)
    assert not torch.equal(seen[0], seen[1])        # fresh masks per replay


@pytest.mark.parametrize("bwd_graph", [True, False])
def test_slot_captured_mid_iteration_keeps_saved_tensors(dev, monkeypatch, bwd_graph):
    """A slot captured in a later iteration between replays of earlier slots (a new step key mid-rollout)
    keeps the tensors its backward saved. Each region saves tanh(x) and frees a same-sized temporary at
    the end of its capture; with one memory pool across slots, the new slot's saved tensor could land in an
    earlier slot's freed temporary, which that slot's next replay overwrites before the backward reads it.
    Gradients are checked against the region's closed form."""
    from dasa_amd import graph
    monkeypatch.setattr(graph, "BWD_GRAPH", bwd_graph)
    torch.manual_seed(11)
    g = graph.AutogradGraphs([])

    def fn(x):
        h = torch.tanh(x)                           # saved by tanh's backward
        with torch.no_grad():
            s = (h.abs() + 1.0).sum(1, keepdim=True)    # temporary freed at the end of the capture
        return (h * s,)

    def expect(x, gy):
        h = torch.tanh(x.detach())
        s = (h.abs() + 1.0).sum(1, keepdim=True)
        return (1 - h * h) * s * gy

    kept = []
    for keys in (("a", "b"), ("a", "c", "b"), ("a", "c", "b")):
        g.new_iteration()
        xs = [torch.randn(64, 256, device=dev, requires_grad=True) for _ in keys]
        ys = [g.run(k, fn, (x,))[0] for k, x in zip(keys, xs)]
        gys = [torch.randn_like(y) for y in ys]
        torch.autograd.backward(ys, gys)
        for k, x, gy in zip(keys, xs, gys):
            torch.testing.assert_close(x.grad, expect(x, gy), rtol=1e-5, atol=1e-5, msg=lambda m: f"{keys} {k}: {m}")
            kept.append((x, gy))
    assert g.captures == 3
    for x, gy in kept:      # a leaf's .grad is its own tensor, not a static buffer later replays rewrite
        torch.testing.assert_close(x.grad, expect(x, gy), rtol=1e-5, atol=1e-5)


def test_backward_graph_keyed_by_weight_grad_deferral(dev):
    """a slot's backward captured under defer_weight_grads (as optim_step runs it) only queues the
    weight / bias products. A later plain loss.backward() on the same slot must not replay that graph (its
    products would be queued with nothing to flush them, and leak into the next flush): it captures its own
    graph, which computes dW / db itself. Checked against the closed form dW = gyᵀx, db = Σ gy, in both modes
    and alternating."""
    from dasa_amd import functional as DF
    from dasa_amd import graph
    torch.manual_seed(13)
    lin = torch.nn.Linear(256, 128).to(dev)
    g = graph.AutogradGraphs([lin])

    def fn(x):
        return (DF.linear(x, lin.weight, lin.bias),)
    for it, deferred in enumerate((True, False, True, False)):
        g.new_iteration()
        x = torch.randn(64, 256, device=dev, requires_grad=True)     # (the bridge links the region via its inputs)
        (y,) = g.run("lin", fn, (x,))
        gy = torch.randn_like(y)
        lin.weight.grad = None
        lin.bias.grad = None
        if deferred:
            with DF.defer_weight_grads():
                y.backward(gy)
            DF.flush_weight_grads()
        else:
            y.backward(gy)
        assert not DF._WG.w and not DF._WG.b, it              # nothing left queued
        want_w = gy.double().t() @ x.detach().double()
        want_b = gy.double().sum(0)
        torch.testing.assert_close(lin.weight.grad.double(), want_w, rtol=1e-5, atol=1e-4, msg=lambda m: f"{it}: {m}")
        torch.testing.assert_close(lin.bias.grad.double(), want_b, rtol=1e-5, atol=1e-4, msg=lambda m: f"{it}: {m}")
    if graph.BWD_GRAPH:
        assert g.captures_bwd == 2, g.captures_bwd              # one per deferral mode


def test_finetune_vl_region_matches_eager(dev, monkeypatch):
    """The finetune configuration's VisionEncoder + LXRT stack as a captured training region (vilmodel.py
    DicModel._vl_train_region): two finetune iterations (README finetune flags, B = 2,
    vl = 3, 4 + 4 steps, dropout 0, forced draws, RMSprop steps between) give the same losses and gradients —
    the LXRT / VisionEncoder parameters' included — with the region captured and replayed as eagerly
    (DASA_TRAIN_GRAPH_VL=0); the regions are captured in iteration 0 and only replayed in iteration 1."""
    from dasa_amd.r2r import param
    param.readme_finetune(["--d_vl_layers", "3", "--batchSize", "2", "--maxAction", "4"])
    try:
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("DASA_TRAIN_GRAPH_VL", mode)
            torch.manual_seed(3)
            from dasa_amd.r2r.agent_dg import Seq2SeqAgent
            from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
            env = SynthR2RBatch(SynthWorld(32, 0, 5), 2, seed=701, mode="wander", instr_len=80, variable_len=True)
            with contextlib.redirect_stdout(io.StringIO()):
                ag = Seq2SeqAgent(env, "", None, 4, "Dic")
            for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
                init_params(m, s)
                for sub in m.modules():
                    if isinstance(sub, torch.nn.Dropout):
                        sub.p = 0.0
            param.args.ml_weight = param.args.ml_weight_org
            assert ag.encoder.bert.update_add_layer
            out = []
            from dasa_amd import functional as DF
            for it in range(2):
                table = GI.forced_table(4, 2, seed=GI.FORCED_SEED + it)
                ag.force_action_fn = lambda t, lens, table=table: GI.forced_actions(table, t, lens, no_stop=True)
                ag.zero_grad()
                ag.accumulate_gradient("sample")
                loss = ag.loss.item()
                with DF.defer_bilstm_backward(), DF.defer_weight_grads():     # optim_step's backward,
                    ag.loss.backward()                                        # gradients before clipping
                    DF.flush_bilstm_backward()
                DF.flush_weight_grads()
                grads = {f"{i}.{k}": p.grad.detach().clone() for i, m in enumerate(ag.models)
                         for k, p in m.named_parameters() if p.grad is not None}
                for opt in ag.optimizers:
                    opt.step()
                if ag._train_graphs is not None:
                    ag._train_graphs.new_iteration()
                ag.encoder.bert.train_graphs_new_iteration()
                out.append((loss, grads))
                if mode == "1" and it == 0:
                    tg = ag.encoder.bert._tgraphs
                    assert tg is not None and tg.captures > 0
                    n0 = (tg.captures, tg.captures_bwd)
            if mode == "1":
                tg = ag.encoder.bert._tgraphs
                assert (tg.captures, tg.captures_bwd) == n0 and tg.replays > tg.captures   # iteration 1 replays
            else:
                assert ag.encoder.bert._tgraphs is None
            res[mode] = out
            del ag
        for it in range(2):
            (l0, g0), (l1, g1) = res["0"][it], res["1"][it]
            assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0)), (it, l0, l1)
            assert sorted(g0) == sorted(g1)
            assert any(k.startswith("0.bert.addlayer") for k in g0)      # the LXRT layers trained
            ratios = {k: (g1[k].norm() / g0[k].norm()).item() for k in g0 if g0[k].norm() > 1e-6}   # (not the ~1e-10 noise of vanishing grads)
            bad = {k: r for k, r in ratios.items() if abs(r - 1) > 1e-3}
            assert not bad, (it, len(bad), sorted(bad.items())[:12])
            for k in g0:
                # (+1e-8: gradients that vanish analytically, e.g. the attention key biases — softmax is shift
                # invariant — are fp32 rounding noise of ~1e-10 that the padded region sums in another order)
                err = (g0[k] - g1[k]).abs().max().item()
                assert err <= 2e-5 * g0[k].abs().max().item() + 1e-8, (it, k, err)
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
