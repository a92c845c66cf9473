"""Paths off the README configuration, all on the kernels (no torch-eager head or attention remains):

* SoftDotAttention's other output combinations (model.py:268-296: output_tilde=False with the softmax,
  output_prob=False with the -inf-masked raw scores, and tilde + raw scores) against fp64 torch math,
  forward and backward (dasa_softdot_fwd / _bwd through functional.SoftDotFn);
* the policy head's sample_argmax mode (sample_fn = "argmax": Categorical entropy / log-prob with the
  draw replaced by the argmax) against the same quantities computed in fp64;
* --submit (agent_dg.py:852-858: visited candidates masked) and --pred_back (the back-prediction CE,
  agent_dg.py:872-876) driven through the one-kernel head: an argmax eval rollout never re-enters a
  visited viewpoint through a masked candidate, and a pred_back training iteration adds a finite back
  loss with gradients on back_candidate_att_layer."""
import contextlib
import io

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_softdot(h, ctx, mask, W_in):
    q = h @ W_in.t()
    s = torch.einsum("bnd,bd->bn", ctx, q)
    if mask is not None:
        s = s.masked_fill(mask, -float("inf"))
    p = torch.softmax(s, 1)
    return torch.einsum("bn,bnd->bd", p, ctx), p, s


@pytest.mark.parametrize("output_tilde,output_prob", [(False, True), (False, False), (True, False)])
def test_softdot_general_combinations(dev, output_tilde, output_prob):
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
    from dasa_amd.r2r import model
    g = torch.Generator().manual_seed(5)
    B, N, D, H = 3, 12, 2048, 1024
    att = model.SoftDotAttention(H, D)
    with torch.no_grad():
        for p in att.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.02)
    h = torch.randn(B, H, generator=g) * 0.5
    ctx = torch.randn(B, N, D, generator=g) * 0.2
    mask = torch.zeros(B, N, dtype=torch.bool)
    mask[1, 7:] = True
    gw = torch.randn(B, H if output_tilde else D, generator=g)
    gs = torch.randn(B, N, generator=g)
    # fp64 reference
    hr, cr = h.double().requires_grad_(), ctx.double().requires_grad_()
    Wr, Wo = att.linear_in.weight.detach().double().requires_grad_(), att.linear_out.weight.detach().double()
    w, p, s = _ref_softdot(hr, cr, mask, Wr)
    out = torch.tanh(torch.cat((w, hr), 1) @ Wo.t()) if output_tilde else w
    loss = (out * gw.double()).sum()
    if not output_prob:
        loss = loss + (s.masked_fill(mask, 0.0) * gs.double()).sum()
    loss.backward()
    # kernels
    att = att.to(dev)
    hd, cd = h.to(dev).requires_grad_(), ctx.to(dev).requires_grad_()
    o, a = att(hd, cd, mask.to(dev), output_tilde=output_tilde, output_prob=output_prob)
    assert (o.detach().cpu().double() - out.detach()).abs().max() < 1e-4
    if output_prob:
        assert (a.detach().cpu().double() - p.detach()).abs().max() < 1e-5
    else:
        assert torch.equal(torch.isinf(a.detach().cpu()), mask)
        fin = ~mask
        assert (a.detach().cpu().double()[fin] - s.detach()[fin]).abs().max() < 1e-4
    kl = (o * gw.to(dev)).sum()
    if not output_prob:
        kl = kl + (a.masked_fill(mask.to(dev), 0.0) * gs.to(dev)).sum()
    kl.backward()
    for got, want in ((hd.grad, hr.grad), (cd.grad, cr.grad), (att.linear_in.weight.grad, Wr.grad)):
        err = (got.cpu().double() - want).abs().max().item()
        assert err < 2e-4 * max(1.0, want.abs().max().item()), err


def test_policy_head_sample_argmax(dev):
    from dasa_amd import functional as DF
    g = torch.Generator().manual_seed(9)
    B, C = 7, 12
    logit = torch.randn(B, C, generator=g) * 2
    lens = torch.tensor([12, 5, 1, 9, 12, 3, 7], dtype=torch.int32)
    ld = logit.to(dev).requires_grad_()
    ce, ent, lpa, act = DF.policy_head(ld, lens.to(dev), None, "sample_argmax")
    masked = logit.masked_fill(torch.arange(C)[None, :] >= lens[:, None].long(), -float("inf")).double()
    p = torch.softmax(masked, 1)
    want_act = masked.argmax(1)
    assert torch.equal(act.cpu(), want_act)
    lc = torch.log(p.clamp(1.1920928955078125e-07, 1 - 1.1920928955078125e-07))
    assert (lpa.cpu().double() - lc.gather(1, want_act[:, None])[:, 0]).abs().max() < 1e-5
    assert (ent.cpu().double() - (-(p * lc).nan_to_num().sum(1))).abs().max() < 1e-5
    (lpa.sum() + ent.sum()).backward()
    assert torch.isfinite(ld.grad).all()


def _agent(env, T):
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    from dasa_amd.synth import init_params
    with contextlib.redirect_stdout(io.StringIO()):
        ag = Seq2SeqAgent(env, "", None, T, "Dic")
    for m, s in ((ag.encoder, 1), (ag.decoder, 2), (ag.critic, 3), (ag.adaIn, 4)):
        init_params(m, s)
    return ag


def test_submit_masks_visited_candidates(dev):
    from dasa_amd.r2r import param
    from dasa_amd.synth import SynthR2RBatch, SynthWorld
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "4", "--maxAction", "8", "--submit"])
    try:
        assert param.args.submit
        env = SynthR2RBatch(SynthWorld(16, 0, 3), 4, seed=31, mode="goal", instr_len=80, variable_len=True)
        ag = _agent(env, 8)
        ag.feedback = "argmax"
        for m in (ag.encoder, ag.decoder, ag.critic):
            m.eval()
        ag.loss = 0
        with torch.no_grad():
            traj = ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
        for tr in traj:
            vps = [p[0] for p in tr["path"]]
            moves = [v for i, v in enumerate(vps) if i == 0 or v != vps[i - 1]]
            assert len(moves) == len(set(moves)), moves     # never re-enters a visited viewpoint
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_pred_back_iteration(dev):
    from dasa_amd.r2r import param
    from dasa_amd.synth import SynthR2RBatch, SynthWorld
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "4", "--maxAction", "4", "--pred_back"])
    try:
        assert param.args.pred_back
        env = SynthR2RBatch(SynthWorld(16, 0, 3), 4, seed=33, mode="goal", instr_len=80, variable_len=True)
        ag = _agent(env, 4)
        param.args.ml_weight = param.args.ml_weight_org
        ag.zero_grad()
        ag.accumulate_gradient("sample")
        assert ag.logs["back_loss"] and all(torch.isfinite(torch.tensor(ag.logs["back_loss"])))
        ag.optim_step()
        g = ag.decoder.back_candidate_att_layer.linear_in.weight.grad
        assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
