"""GPU parity of the product modules (dasa_amd.r2r on libdasa_hip.so) against the reference's golden
vectors (tests/golden, produced by the reference itself) and the CPU oracle. Tolerance: the north
star's 1e-4 fp32 on logits / critic values / states; gradients to 1e-3 relative."""
import numpy as np
import pytest
import torch

from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
from tests import golden_inputs as GI
from tests.helpers import check_grads, close, golden

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def R(dev):
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
    from dasa_amd.r2r import agent_dg, model, r2rmodel, vilmodel
    return param, agent_dg, model, r2rmodel, vilmodel


def _req(t, dev):
    return t.to(dev).requires_grad_(True)


def test_ada_channel(R, dev):
    param, agent_dg, *_ = R
    G = golden("ops")
    ada = init_params(agent_dg.DGAdaChannel(2048), GI.SEED_ADA).to(dev)
    f, d, g = GI.ada_inputs()
    y = ada(f.to(dev), d.to(dev))
    close(y.detach().cpu(), G["ada/out"], 1e-5, "ada")
    (y * g.to(dev)).sum().backward()
    assert check_grads(G, "ada/", [(k, p.grad) for k, p in ada.named_parameters()], rtol=1e-3) == 2
    # the fused 2176-wide feature path used by the rollout (AdaFeatFn) agrees with forward()
    fa = torch.cat([f, torch.rand(2, 10, 128)], -1).to(dev)
    da = torch.cat([d, torch.rand(2, 10, 128)], -1).to(dev)
    with torch.no_grad():
        out = ada.feature(fa, da)
    close(out[..., :2048].cpu(), G["ada/out"], 1e-5, "ada feature rgb")
    close(out[..., 2048:].cpu(), fa[..., 2048:].cpu(), 0.0, "ada feature angle")


@pytest.mark.parametrize("K", [5, 3])
def test_shift_attention(R, dev, K):
    model = R[2]
    G = golden("ops")
    m = init_params(model.ShiftSoftDotAttention(1024, 2176, K), 20 + K).to(dev)
    h, ctx, gw = GI.shift_inputs(K)
    h, ctx = _req(h, dev), _req(ctx, dev)
    wctx, attn = m(h, ctx, output_tilde=False)
    close(wctx.detach().cpu(), G[f"shift{K}/wctx"], TOL, "wctx")
    close(attn.detach().cpu(), G[f"shift{K}/attn"], 1e-5, "attn")
    (wctx * gw.to(dev)).sum().backward()
    close(h.grad.cpu(), G[f"shift{K}/dh"], 1e-3 * np.abs(G[f"shift{K}/dh"]).max(), "dh")
    assert check_grads(G, f"shift{K}/", [("ctx", ctx.grad)] + [(k, p.grad) for k, p in m.named_parameters()],
                       rtol=1e-3) >= 3


def test_softdot(R, dev):
    model = R[2]
    G = golden("ops")
    h, ctx, mask, cand, g1, g2 = GI.softdot_inputs()
    att = init_params(model.SoftDotAttention(1024, 2048), 30).to(dev)
    h1 = _req(h, dev)
    ht, alpha = att(h1, ctx.to(dev), mask.to(dev))
    close(ht.detach().cpu(), G["softdot/h_tilde"], 1e-5, "h_tilde")
    # probabilities of scores summed over K = 2048 products: summation order moves them by ~2e-6
    close(alpha.cpu(), G["softdot/alpha"], 1e-5, "alpha")
    (ht * g1.to(dev)).sum().backward()
    # input gradients are sums over K = 2048..3200 products with |dh| up to ~40: bound relative to scale
    close(h1.grad.cpu(), G["softdot/dh"], max(1e-4, 1e-5 * np.abs(G["softdot/dh"]).max()), "dh")
    assert check_grads(G, "softdot/", [(k, p.grad) for k, p in att.named_parameters()], rtol=1e-3) == 2
    catt = init_params(model.SoftDotAttention(1024, 2176), 31).to(dev)
    h2, cd = _req(h, dev), _req(cand, dev)
    _, logit = catt(h2, cd, output_prob=False, output_tilde=False)
    close(logit.detach().cpu(), G["cand/logit"], TOL, "cand logit")
    (logit * g2.to(dev)).sum().backward()
    close(h2.grad.cpu(), G["cand/dh"], max(1e-4, 1e-5 * np.abs(G["cand/dh"]).max()), "cand dh")
    check_grads(G, "cand/", [("cand", cd.grad), ("linear_in.weight", catt.linear_in.weight.grad)], rtol=1e-3)


def test_decoder_and_critic(R, dev):
    param, agent_dg, model = R[0], R[1], R[2]
    A = param.args
    G = golden("ops")
    dec = init_params(model.BAttnDecoderLSTM(A.aemb, A.d_hidden_size, A.dropout, feature_size=2176), GI.SEED_DEC)
    dec = dec.to(dev).eval()
    ins = [t.to(dev) for t in GI.decoder_inputs()]
    h1, c1, logit, ht, _ = dec(*ins)
    for k, v in dict(h1=h1, c1=c1, logit=logit, h_tilde=ht).items():
        close(v.detach().cpu(), G["dec/" + k], TOL, k)
    rng = np.random.default_rng(121)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)).to(dev) for t in (h1, c1, logit, ht)]
    ((h1 * w[0]).sum() + (c1 * w[1]).sum() + (logit * w[2]).sum() + (ht * w[3]).sum()).backward()
    assert check_grads(G, "dec/", [(k, p.grad) for k, p in dec.named_parameters() if p.grad is not None],
                       rtol=1e-3) >= 10
    cr = init_params(model.Critic(), GI.SEED_CRITIC).to(dev).eval()
    v = cr(GI.critic_inputs().to(dev))
    close(v.detach().cpu(), G["critic/value"], TOL, "critic")
    (v * torch.arange(1.0, 5.0, device=dev)).sum().backward()
    assert check_grads(G, "critic/", [(k, p.grad) for k, p in cr.named_parameters()], rtol=1e-3) == 4


def test_lxrt_layer(R, dev):
    vilmodel = R[4]
    G = golden("ops")
    lx = init_params(vilmodel.LXRTXLayer(vilmodel.BertConfig()), 40).to(dev).eval()
    lang, lmask, visn, vmask = GI.lxrt_inputs()
    with torch.no_grad():
        lo, vo = lx(lang.to(dev), lmask[:, None, None, :].to(dev), visn.to(dev), vmask[:, None, None, :].to(dev))
    close(lo.cpu(), G["lxrt/lang"], TOL, "lang")
    close(vo.cpu(), G["lxrt/visn"], TOL, "visn")


def test_lxrt_layer_backward(R, dev):
    """LXRTXLayer backward (the finetune path, cfg4): parameter and input gradients vs the reference."""
    vilmodel = R[4]
    G = golden("cfg4_finetune")
    lx = init_params(vilmodel.LXRTXLayer(vilmodel.BertConfig()), 40).to(dev).eval()
    lang, lmask, visn, vmask = GI.lxrt_inputs()
    lang, visn = _req(lang, dev), _req(visn, dev)
    lo, vo = lx(lang, lmask[:, None, None, :].to(dev), visn, vmask[:, None, None, :].to(dev))
    rng = np.random.default_rng(141)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)).to(dev) for t in (lo, vo)]
    ((lo * w[0]).sum() + (vo * w[1]).sum()).backward()
    n = check_grads(G, "lxrt/", [(k, p.grad) for k, p in lx.named_parameters()], rtol=1e-3)
    assert n == sum(1 for k in G if k.startswith("gnorm/lxrt/"))
    assert check_grads(G, "lxrt_in/", [("lang", lang.grad), ("visn", visn.grad)], rtol=1e-3) == 2


def test_dic_encoder(R, dev):
    param, r2rmodel = R[0], R[3]
    A = param.args
    G = golden("ops")
    enc = r2rmodel.DicEncoder(2176, A.d_enc_hidden_size, A.d_hidden_size, A.d_dropout_ratio, A.d_bidirectional,
                              A.d_transformer_update, A.d_bert_n_layers, A.d_reverse_input, A.d_top_lstm, 1,
                              A.d_la_layers, A.d_bert_type, update_add_layer=A.d_update_add_layer)
    enc = init_params(enc, GI.SEED_ENC).to(dev).eval()
    seq, mask, lengths, f = GI.encoder_inputs()
    ctx, dinit, ct, _, vis = enc(seq.to(dev), mask.to(dev), torch.tensor(lengths), f_t_all=f.to(dev))
    close(ctx.detach().cpu(), G["enc/ctx"], TOL, "ctx")
    close(dinit.detach().cpu(), G["enc/decoder_init"], TOL, "decoder_init")
    close(ct.detach().cpu(), G["enc/c_t"], TOL, "c_t")
    close(vis.detach().cpu(), G["enc/vision"], TOL, "vision")
    rng = np.random.default_rng(151)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)).to(dev) for t in (ctx, dinit, ct)]
    ((ctx * w[0]).sum() + (dinit * w[1]).sum() + (ct * w[2]).sum()).backward()
    assert check_grads(G, "enc/", [(k, p.grad) for k, p in enc.named_parameters() if p.grad is not None],
                       rtol=1e-3) == 12


def _agent(R, env, T, seed_weights=True):
    agent_dg = R[1]
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        ag = agent_dg.Seq2SeqAgent(env, "", None, T, "Dic")
    if seed_weights:
        init_params(ag.encoder, GI.SEED_ENC)
        init_params(ag.decoder, GI.SEED_DEC)
        init_params(ag.critic, GI.SEED_CRITIC)
        init_params(ag.adaIn, GI.SEED_ADA)
    return ag


class _HostOnlyEnv:
    """Hides device_input_feat so the agent takes the reference numpy + H2D path."""

    def __init__(self, env):
        self._e = env

    def __getattr__(self, k):
        if k == "device_input_feat":
            raise AttributeError(k)
        return getattr(self._e, k)


@pytest.mark.parametrize("host_path", [False, True])
def test_rollout_eval_argmax(R, dev, host_path):
    G = golden("cfg1_rollout")
    cfg = GI.CFG1
    env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=7, mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    if host_path:
        env = _HostOnlyEnv(env)
    ag = _agent(R, env, cfg["max_action"])
    rec = {"logit": [], "h1": [], "h_tilde": []}
    fwd = ag.decoder.forward

    def wrap(*a, **k):
        r = fwd(*a, **k)
        rec["logit"].append(r[2].detach().cpu())
        rec["h1"].append(r[0].detach().cpu())
        rec["h_tilde"].append(r[3].detach().cpu())
        return r
    ag.decoder.forward = wrap
    ag.loss = 0
    ag.feedback = "argmax"
    for m in (ag.encoder, ag.decoder, ag.critic):
        m.eval()
    with torch.no_grad():
        traj = ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
    assert len(rec["logit"]) == int(G["eval/steps"])
    for t in range(len(rec["logit"])):
        close(rec["logit"][t], G[f"eval/logit/{t}"], TOL, f"logit{t}")
        close(rec["h1"][t], G[f"eval/h1/{t}"], TOL, f"h1{t}")
        close(rec["h_tilde"][t], G[f"eval/h_tilde/{t}"], TOL, f"h_tilde{t}")
    assert abs(ag.logs["ml_loss"][-1] - float(G["eval/ml_loss"])) < 1e-3
    assert ["|".join(p[0] for p in tr["path"]) for tr in traj] == list(G["eval/paths"])


def test_rollout_bf16_matmul_first_step(R, dev):
    """configs[4] numerics: the eval rollout under ops.bf16_matmul (bf16 GEMM operands, fp32 accumulation)
    against the reference's fp32 golden. Only step 0 is compared (argmax paths may legitimately part
    once logits differ at bf16 precision); tolerance 3e-2 of the logit range, 2e-2 on the states."""
    from dasa_amd import ops
    G = golden("cfg1_rollout")
    cfg = GI.CFG1
    env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=7, mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    ag = _agent(R, env, cfg["max_action"])
    rec = []
    fwd = ag.decoder.forward

    def wrap(*a, **k):
        r = fwd(*a, **k)
        rec.append((r[2].detach().cpu(), r[0].detach().cpu()))
        return r
    ag.decoder.forward = wrap
    ag.loss = 0
    ag.feedback = "argmax"
    for m in (ag.encoder, ag.decoder, ag.critic):
        m.eval()
    with torch.no_grad(), ops.bf16_matmul():
        ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
    logit, h1 = rec[0]
    ref = torch.from_numpy(G["eval/logit/0"])
    fin = torch.isfinite(ref)
    span = (ref[fin].max() - ref[fin].min()).item()
    close(logit[fin], ref[fin], 3e-2 * span, "bf16 logit0")
    close(h1, G["eval/h1/0"], 2e-2, "bf16 h1")
    assert (logit[fin] - ref[fin]).abs().max().item() > 0.0     # the bf16 GEMM actually ran


@pytest.mark.parametrize("deferred", [False, True])
def test_train_iteration_grads(R, dev, deferred):
    """accumulate_gradient('sample') + backward with every dropout p = 0 and argmax 'sampling'.
    deferred: the bi-LSTM BPTTs of all encoder calls run as one batched recurrence and the decoder /
    critic weight gradients of all steps as one GEMM per parameter (optim_step's path)."""
    from dasa_amd import functional as DF
    param = R[0]
    G = golden("cfg1_rollout")
    cfg = GI.CFG1
    env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=8, mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    ag = _agent(R, env, cfg["max_action"])
    for m in ag.models:
        for sub in m.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    param.args.ml_weight = param.args.ml_weight_org
    ag.sample_fn = "argmax"
    ag.zero_grad()
    ag.accumulate_gradient("sample")
    assert abs(ag.loss.item() - float(G["train/loss"])) < TOL * max(1.0, abs(float(G["train/loss"])))
    assert abs(ag.logs["ml_loss"][0] - float(G["train/ml_loss_teacher"])) < 1e-3
    assert abs(ag.logs["ml_loss"][1] - float(G["train/ml_loss_sample"])) < 1e-3
    assert abs(ag.logs["normalized_rl_loss"][-1] - float(G["train/rl_loss"])) < TOL
    assert ag.logs["viewsteps/teacher"][-1] == int(G["train/steps_teacher"])
    assert ag.logs["viewsteps/sample"][-1] == int(G["train/steps_sample"])
    if deferred:    # optim_step's path: batched bi-LSTM BPTT + per-parameter weight-gradient GEMMs
        with DF.defer_bilstm_backward(), DF.defer_weight_grads():
            ag.loss.backward()
        DF.flush_bilstm_backward()
        DF.flush_weight_grads()
    else:
        ag.loss.backward()
    n = 0
    for name, mod in (("encoder", ag.encoder), ("decoder", ag.decoder), ("critic", ag.critic), ("adaIn", ag.adaIn)):
        n += check_grads(G, f"train/{name}.", [(k, p.grad) for k, p in mod.named_parameters()], rtol=2e-3)
    assert n == 30


def test_hoist_language_train(R, dev):
    """--hoist_language (non-default): (1) with every dropout p = 0 the detached language
    stack is deterministic, so the hoisted iteration reproduces the reference's loss and gradients
    (cfg1 golden); (2) with dropout on, the stack runs once per rollout (twice per iteration: teacher +
    sample) instead of once per step."""
    param = R[0]
    G = golden("cfg1_rollout")
    cfg = GI.CFG1

    def make(p0):
        env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=8, mode="goal", instr_len=cfg["instr_len"],
                            variable_len=True)
        ag = _agent(R, env, cfg["max_action"])
        if p0:
            for m in ag.models:
                for sub in m.modules():
                    if isinstance(sub, torch.nn.Dropout):
                        sub.p = 0.0
        ag.sample_fn = "argmax"
        return ag
    param.args.ml_weight = param.args.ml_weight_org
    param.args.hoist_language = True
    try:
        ag = make(True)
        ag.zero_grad()
        ag.accumulate_gradient("sample")
        assert abs(ag.loss.item() - float(G["train/loss"])) < TOL * max(1.0, abs(float(G["train/loss"])))
        ag.loss.backward()
        n = 0
        for name, mod in (("encoder", ag.encoder), ("decoder", ag.decoder), ("critic", ag.critic),
                          ("adaIn", ag.adaIn)):
            n += check_grads(G, f"train/{name}.", [(k, p.grad) for k, p in mod.named_parameters()], rtol=2e-3)
        assert n == 30
        counts = {}
        for hoist in (True, False):
            param.args.hoist_language = hoist
            ag = make(False)
            calls = []
            lang = ag.encoder.bert.language
            ag.encoder.bert.language = lambda *a, **k: (calls.append(1), lang(*a, **k))[1]
            ag.zero_grad()
            ag.accumulate_gradient("sample")
            assert torch.isfinite(ag.loss).item()
            counts[hoist] = (len(calls), ag.logs["viewsteps/teacher"][-1] + ag.logs["viewsteps/sample"][-1])
        # one stack per rollout; the default path computes one per step (the teacher's batched encoder
        # call over T x B sequences and the sampled rollout's language pipe)
        assert counts[True][0] == 2, counts
    finally:
        param.args.hoist_language = False


@pytest.mark.parametrize("deferred", [0, 1, 2])
def test_finetune_train_iteration_grads(R, dev, monkeypatch, deferred):
    """cfg4 finetune path (--d_update_add_layer True): the LXRT stack and VisionEncoder are trained.
    accumulate_gradient('sample') + backward with dropout 0 and argmax 'sampling' vs the reference.
    deferred 1: batched weight gradients, per-call bi-LSTM BPTT (its input trains); 2: optim_step's path,
    the bi-LSTM BPTTs batched with their input gradients and the backward continued from there."""
    from dasa_amd import functional as DF
    param = R[0]
    G = golden("cfg4_finetune")
    cfg = GI.CFG4
    monkeypatch.setattr(param.args, "d_vl_layers", cfg["vl_layers"])
    monkeypatch.setattr(param.args, "maxAction", cfg["max_action"])
    monkeypatch.setattr(param.args, "d_update_add_layer", True)
    env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=9, mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    ag = _agent(R, env, cfg["max_action"])
    assert ag.encoder.bert.update_add_layer
    for m in ag.models:
        for sub in m.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    monkeypatch.setattr(param.args, "ml_weight", param.args.ml_weight_org)
    ag.sample_fn = "argmax"
    ag.zero_grad()
    ag.accumulate_gradient("sample")
    assert abs(ag.loss.item() - float(G["ft/loss"])) < TOL * max(1.0, abs(float(G["ft/loss"])))
    assert abs(ag.logs["ml_loss"][0] - float(G["ft/ml_loss_teacher"])) < 1e-3
    assert abs(ag.logs["ml_loss"][1] - float(G["ft/ml_loss_sample"])) < 1e-3
    assert abs(ag.logs["normalized_rl_loss"][-1] - float(G["ft/rl_loss"])) < TOL
    if deferred:
        with DF.defer_bilstm_backward(input_grads=deferred == 2), DF.defer_weight_grads():
            ag.loss.backward(retain_graph=deferred == 2)
            DF.flush_bilstm_backward()
        DF.flush_weight_grads()
    else:
        ag.loss.backward()
    n = 0
    for name, mod in (("encoder", ag.encoder), ("decoder", ag.decoder), ("critic", ag.critic), ("adaIn", ag.adaIn)):
        n += check_grads(G, f"ft/{name}.", [(k, p.grad) for k, p in mod.named_parameters()], rtol=2e-3)
    assert n == sum(1 for k in G if k.startswith("gnorm/ft/"))
    for k, p in ag.encoder.named_parameters():     # the same parameter set receives gradients
        assert (p.grad is not None) == (f"gnorm/ft/encoder.{k}" in G), k


@pytest.mark.parametrize("batched", ["1", "0"])
def test_cfg2_teacher_rollout_vs_oracle(R, dev, monkeypatch, batched):
    """A 3-step teacher-forced eval rollout at the cfg2 shape (B=20, L=80, vl=3, C<=16) against the CPU
    oracle, per step. batched=1: the encoder runs once over all steps (the train path's teacher
    rollout); batched=0: the step-by-step loop."""
    from oracle import policy as O
    from tests.helpers import oracle_weights
    monkeypatch.setenv("DASA_TEACHER_BATCH", batched)
    param = R[0]
    param.readme_train(["--d_vl_layers", "3"])
    T = 3
    try:
        world = SynthWorld(32, 0, 5)
        env = SynthR2RBatch(world, 20, seed=11, mode="wander", instr_len=80)
        env2 = SynthR2RBatch(world, 20, seed=11, mode="wander", instr_len=80)
        ag = _agent(R, env, T)
        W = oracle_weights(3)
        rec = {"logit": [], "h_tilde": []}
        fwd = ag.decoder.forward

        def wrap(*a, **k):
            r = fwd(*a, **k)
            rec["logit"].append(r[2].detach().cpu())
            rec["h_tilde"].append(r[3].detach().cpu())
            return r
        ag.decoder.forward = wrap
        ag.loss = 0
        ag.feedback = "teacher"
        for m in (ag.encoder, ag.decoder, ag.critic):
            m.eval()
        with torch.no_grad():
            ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
            r = O.vl_rollout(W, env2, "teacher", la_layers=9, vl_layers=3, episode_len=T)
        assert len(rec["logit"]) == r["steps"] == T
        for t in range(T):
            close(rec["logit"][t], r["logits"][t], TOL, f"cfg2 logit {t}")
            close(rec["h_tilde"][t], r["states"][t][2], TOL, f"cfg2 h_tilde {t}")
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_cfg2_step_vs_oracle(R, dev):
    """One eval policy step at the cfg2 shape (B=20, L=80, vl=3, C<=16) against the CPU oracle."""
    from oracle import policy as O
    from tests.helpers import oracle_weights
    param = R[0]
    param.readme_train(["--d_vl_layers", "3"])
    try:
        world = SynthWorld(32, 0, 5)
        env = SynthR2RBatch(world, 20, seed=11, mode="wander", instr_len=80)
        env2 = SynthR2RBatch(world, 20, seed=11, mode="wander", instr_len=80)
        ag = _agent(R, env, 1)
        W = oracle_weights(3)
        rec = {}
        fwd = ag.decoder.forward

        def wrap(*a, **k):
            r = fwd(*a, **k)
            rec["logit"] = r[2].detach().cpu()
            rec["h_tilde"] = r[3].detach().cpu()
            return r
        ag.decoder.forward = wrap
        ag.loss = 0
        ag.feedback = "teacher"
        for m in (ag.encoder, ag.decoder, ag.critic):
            m.eval()
        with torch.no_grad():
            ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
            r = O.vl_rollout(W, env2, "teacher", la_layers=9, vl_layers=3, episode_len=1)
        close(rec["logit"], r["logits"][0], TOL, "cfg2 logit")
        close(rec["h_tilde"], r["states"][0][2], TOL, "cfg2 h_tilde")
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_vl_stack_graph_replay(R, dev, monkeypatch):
    """The forward-only VisionEncoder + LXRT stack as a hipGraph replay (dasa_amd/graph.py): bitwise
    equal to the eager launches in eval; in train mode every replay draws fresh dropout masks (device
    seed counter) and stays a proper dropout of the same computation."""
    from dasa_amd import graph
    param, vilmodel = R[0], R[4]
    cfg = vilmodel.BertConfig()
    cfg.img_feature_dim, cfg.img_feature_type = 2176, ""
    cfg.update_lang_bert, cfg.update_add_layer, cfg.vl_layers, cfg.la_layers = False, False, 2, 1
    m = init_params(vilmodel.DicModel(cfg), 77).to(dev)
    g = torch.Generator().manual_seed(5)
    B, L = 3, 11
    ids = torch.randint(1, 1000, (B, L), generator=g).to(dev)
    att = torch.ones(B, L, dtype=torch.long, device=dev)
    att[1, 7:] = 0
    img = torch.rand(B, 36, 2176, generator=g).to(dev)
    m.eval()
    with torch.no_grad():
        monkeypatch.setattr(graph, "ENABLED", False)
        ref_l, _, ref_v = m(ids, None, att, img_feats=img)
        monkeypatch.setattr(graph, "ENABLED", True)
        for _ in range(2):
            out_l, _, out_v = m(ids, None, att, img_feats=img)
            assert torch.equal(out_l, ref_l) and torch.equal(out_v, ref_v)
    assert m._graphs is not None and m._graphs.captures == 1 and m._graphs.replays == 2
    m.train()
    text = m.language(ids, ((1.0 - att.float()) * -10000.0)[:, None, None, :]).detach()
    with torch.no_grad():
        a = m(ids, None, att, img_feats=img, text_embeds=text)[2]
        b = m(ids, None, att, img_feats=img, text_embeds=text)[2]
        monkeypatch.setattr(graph, "ENABLED", False)
        c = m(ids, None, att, img_feats=img, text_embeds=text)[2]
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    assert not torch.equal(a, b)                        # fresh masks per replay
    for x in (a, b):                                    # same distribution as the eager dropout draw
        assert abs(x.std().item() - c.std().item()) < 0.1 * c.std().item()
        assert (x - c).abs().mean().item() < 2.0 * (c - ref_v).abs().mean().item() + 1e-3


def test_vl_stack_without_vision_output(R, dev, monkeypatch):
    """want_visn=False / want_pooled=False (the agent without --ctx_v: the reference discards
    vision_outputs, agent_dg.py:807-808, and DicEncoder never reads the pooler): the last LXRT layer's
    vision branch and the pooler are skipped, the language output is bitwise the full stack's — eager,
    graph-replayed, and under autograd (update_add_layer), where the skipped branch's parameters get
    no gradient exactly as in the reference, whose loss never reaches them."""
    from dasa_amd import graph
    vilmodel = R[4]
    cfg = vilmodel.BertConfig()
    cfg.img_feature_dim, cfg.img_feature_type = 2176, ""
    cfg.update_lang_bert, cfg.update_add_layer, cfg.vl_layers, cfg.la_layers = False, False, 3, 1
    m = init_params(vilmodel.DicModel(cfg), 78).to(dev)
    g = torch.Generator().manual_seed(6)
    B, L = 4, 9
    ids = torch.randint(1, 1000, (B, L), generator=g).to(dev)
    att = torch.ones(B, L, dtype=torch.long, device=dev)
    att[2, 5:] = 0
    img = torch.rand(B, 36, 2176, generator=g).to(dev)
    m.eval()
    with torch.no_grad():
        for enabled in (False, True):
            monkeypatch.setattr(graph, "ENABLED", enabled)
            full_l, pooled, full_v = m(ids, None, att, img_feats=img)
            for _ in range(2):
                lang, p2, v2 = m(ids, None, att, img_feats=img, want_visn=False, want_pooled=False)
                assert torch.equal(lang, full_l) and p2 is None and v2 is None
            assert pooled is not None and full_v is not None
    cfg.update_add_layer = True
    m2 = init_params(vilmodel.DicModel(cfg), 78).to(dev)
    m2.update_add_layer = True
    m2.eval()
    monkeypatch.setattr(graph, "ENABLED", False)
    lang, _, _ = m2(ids, None, att, img_feats=img, want_visn=False)
    lang.square().sum().backward()
    last = m2.addlayer[-1]
    for name, p in last.named_parameters():
        if name.startswith(("visn_self_att", "visn_inter", "visn_output")):
            assert p.grad is None, name
        elif name.startswith(("lang_", "visual_attention")):
            assert p.grad is not None, name
    full_l2, _, _ = m2(ids, None, att, img_feats=img)
    assert torch.equal(lang.detach(), full_l2.detach())


def test_adain_musigma_vs_reference(R, dev):
    """mu/sigma AdaIN (adaIn_type default, model.py:1822-1840): forward and content/style gradients
    against the reference's golden."""
    model = R[2]
    G = golden("ops")
    c, s = GI.adain_inputs()
    c, s = _req(c, dev), _req(s, dev)
    y = model.adaptive_instance_normalization(c, s)
    close(y.detach().cpu(), G["adain/out"], 1e-5, "adain out")
    (y * GI.adain_grad_weights().to(dev)).sum().backward()
    assert check_grads(G, "adain/", [("content", c.grad), ("style", s.grad)], rtol=1e-4) == 2


def _record_eval(ag, feedback, bf16=False):
    """Eval rollout with per-step (logit, h1, c1, h_tilde) and the critic value of every step's state."""
    from dasa_amd import ops
    rec = []
    fwd = ag.decoder.forward

    def wrap(*a, **k):
        r = fwd(*a, **k)
        rec.append({"logit": r[2].detach().clone(), "h1": r[0].detach().clone(), "c1": r[1].detach().clone(),
                    "h_tilde": r[3].detach().clone()})
        return r
    ag.decoder.forward = wrap
    ag.loss = 0
    ag.feedback = feedback
    for m in (ag.encoder, ag.decoder, ag.critic):
        m.eval()
    with torch.no_grad(), (ops.bf16_matmul() if bf16 else _nullctx()):
        traj = ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
        for r in rec:
            r["value"] = ag.critic(r["h1"]).detach().cpu()
            for k in ("logit", "h1", "c1", "h_tilde"):
                r[k] = r[k].cpu()
    ag.decoder.forward = fwd
    return rec, traj


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _check_eval(G, prefix, rec, traj, ag, tol=TOL):
    assert len(rec) == int(G[prefix + "steps"])
    for t, r in enumerate(rec):
        close(r["logit"], G[f"{prefix}logit/{t}"], tol, f"{prefix}logit{t}")
        close(r["value"], G[f"{prefix}value/{t}"], tol, f"{prefix}value{t}")
        if f"{prefix}h_tilde/{t}" in G:
            close(r["h_tilde"], G[f"{prefix}h_tilde/{t}"], tol, f"{prefix}h_tilde{t}")
            close(r["c1"], G[f"{prefix}c1/{t}"], tol, f"{prefix}c1{t}")
    ref_ml = float(G[prefix + "ml_loss"])
    assert abs(ag.logs["ml_loss"][-1] - ref_ml) < 1e-4 * max(1.0, abs(ref_ml))
    assert ["|".join(p[0] for p in tr["path"]) for tr in traj] == list(G[prefix + "paths"])


def _cfg2_env(mode, seed):
    cfg = GI.CFG2
    return SynthR2RBatch(SynthWorld(cfg["viewpoints"], 0, cfg["graph_seed"]), cfg["batch"], seed=seed, mode=mode,
                         instr_len=cfg["instr_len"], variable_len=True)


@pytest.fixture
def cfg2_args(R):
    param = R[0]
    cfg = GI.CFG2
    param.readme_train(["--d_vl_layers", str(cfg["vl_layers"]), "--batchSize", str(cfg["batch"]),
                        "--maxAction", str(cfg["max_action"])])
    yield param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_cfg2_argmax_rollout(R, dev, cfg2_args):
    """Bench shape (B=20, vl=3, L<=80): the argmax eval rollout until every agent stops — logits and
    critic values within 1e-4 of the reference, identical argmax paths."""
    G = golden("cfg2")
    cfg = GI.CFG2
    ag = _agent(R, _cfg2_env("goal", cfg["eval_seed"]), cfg["max_action"])
    rec, traj = _record_eval(ag, "argmax")
    _check_eval(G, "eval/", rec, traj, ag)


@pytest.mark.parametrize("batched", ["1", "0"])
def test_cfg2_teacher_rollout_35(R, dev, cfg2_args, monkeypatch, batched):
    """Bench shape: a full 35-step teacher-forced eval rollout (B=20, vl=3) — every step's logits and
    critic values within 1e-4 of the reference. batched=1: the train path's chunked encoder."""
    monkeypatch.setenv("DASA_TEACHER_BATCH", batched)
    G = golden("cfg2")
    cfg = GI.CFG2
    ag = _agent(R, _cfg2_env("wander", cfg["eval_seed"]), cfg["max_action"])
    rec, traj = _record_eval(ag, "teacher")
    assert len(rec) == 35
    _check_eval(G, "teacher/", rec, traj, ag)


@pytest.mark.parametrize("deferred", [True, False])
def test_cfg2_train_iteration_grads(R, dev, cfg2_args, deferred):
    """Bench configuration's training iteration (B=20, vl=3, maxAction 5; dropout 0, argmax
    'sampling'): losses within 1e-4 relative, all 30 parameter gradients by norm, 8 sketches and a
    fixed row subset at rtol 1e-3 (tests/helpers.check_grads)."""
    from dasa_amd import functional as DF
    param = cfg2_args
    G = golden("cfg2")
    cfg = GI.CFG2
    param.args.maxAction = cfg["train_max_action"]
    ag = _agent(R, _cfg2_env("goal", cfg["train_seed"]), cfg["train_max_action"])
    for m in ag.models:
        for sub in m.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    param.args.ml_weight = param.args.ml_weight_org
    ag.sample_fn = "argmax"
    ag.zero_grad()
    ag.accumulate_gradient("sample")
    ref = float(G["train/loss"])
    assert abs(ag.loss.item() - ref) < TOL * max(1.0, abs(ref))
    assert abs(ag.logs["ml_loss"][0] - float(G["train/ml_loss_teacher"])) < TOL * max(1.0, float(G["train/ml_loss_teacher"]))
    assert abs(ag.logs["ml_loss"][1] - float(G["train/ml_loss_sample"])) < TOL * max(1.0, float(G["train/ml_loss_sample"]))
    assert abs(ag.logs["normalized_rl_loss"][-1] - float(G["train/rl_loss"])) < TOL
    assert ag.logs["viewsteps/teacher"][-1] == int(G["train/steps_teacher"])
    assert ag.logs["viewsteps/sample"][-1] == int(G["train/steps_sample"])
    if deferred:
        with DF.defer_bilstm_backward(), DF.defer_weight_grads():
            ag.loss.backward()
        DF.flush_bilstm_backward()
        DF.flush_weight_grads()
    else:
        ag.loss.backward()
    n = 0
    for name, mod in (("encoder", ag.encoder), ("decoder", ag.decoder), ("critic", ag.critic), ("adaIn", ag.adaIn)):
        n += check_grads(G, f"train/{name}.", [(k, p.grad) for k, p in mod.named_parameters()], rtol=1e-3)
    assert n == 30


# bf16-operand GEMMs (ops.bf16_matmul) against the fp32 reference: per-step logit tolerance as a
# fraction of that step's logit range. Teacher forcing keeps the paths identical, so every step compares.
BF16_LOGIT_FRAC = 5e-2


def test_cfg5_vl6_teacher_rollout(R, dev, monkeypatch):
    """d_vl_layers = 6 (BASELINE configs[4]) at B=4, 6 teacher-forced steps: the fp32 rollout within
    1e-4 of the reference at every step; the bf16-operand rollout within BF16_LOGIT_FRAC of each step's
    logit range (and 5e-2 on critic values)."""
    param = R[0]
    G = golden("cfg5")
    cfg = GI.CFG5
    param.readme_train(["--d_vl_layers", str(cfg["vl_layers"]), "--batchSize", str(cfg["batch"]),
                        "--maxAction", str(cfg["max_action"])])
    try:
        def env():
            return SynthR2RBatch(SynthWorld(cfg["viewpoints"], 0, cfg["graph_seed"]), cfg["batch"], seed=cfg["seed"],
                                 mode="wander", instr_len=cfg["instr_len"], variable_len=True)
        ag = _agent(R, env(), cfg["max_action"])
        rec, traj = _record_eval(ag, "teacher")
        _check_eval(G, "teacher/", rec, traj, ag)
        ag = _agent(R, env(), cfg["max_action"])
        rec, traj = _record_eval(ag, "teacher", bf16=True)
        assert len(rec) == cfg["max_action"]
        worst = 0.0
        for t, r in enumerate(rec):
            ref = torch.from_numpy(G[f"teacher/logit/{t}"])
            fin = torch.isfinite(ref)
            span = (ref[fin].max() - ref[fin].min()).item()
            err = (r["logit"][fin] - ref[fin]).abs().max().item()
            worst = max(worst, err / span)
            assert err <= BF16_LOGIT_FRAC * span, (t, err, span)
            close(r["value"], G[f"teacher/value/{t}"], 5e-2, f"bf16 value{t}")
        assert worst > 0.0      # the bf16 GEMM actually ran
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_cfg5_b256_vs_reference(R, dev):
    """configs[4] at its own size (B=256, vl=6, L<=80 variable; GI.CFG5_B256), 2 teacher-forced eval
    steps, against the REFERENCE run at that size (make_golden.py cfg5_b256): the fp32 rollout — the
    B >= 128 forms: whole-row shift / SoftDot attention (N = 80 included), the bf16x6 256-row plans, the
    bi-LSTM's 192-row tiles — within 1e-4 at every step (logits, critic values, last-step states); the
    bf16-operand rollout within BF16_LOGIT_FRAC of each step's logit range and 5e-2 on critic values."""
    param = R[0]
    G = golden("cfg5_b256")
    cfg = GI.CFG5_B256
    param.readme_train(["--d_vl_layers", str(cfg["vl_layers"]), "--batchSize", str(cfg["batch"]),
                        "--maxAction", str(cfg["max_action"])])
    try:
        def env():
            return SynthR2RBatch(SynthWorld(cfg["viewpoints"], 0, cfg["graph_seed"]), cfg["batch"], seed=cfg["seed"],
                                 mode="wander", instr_len=cfg["instr_len"], variable_len=True)
        ag = _agent(R, env(), cfg["max_action"])
        r32, traj = _record_eval(ag, "teacher")
        _check_eval(G, "b256/", r32, traj, ag)
        del ag
        ag2 = _agent(R, env(), cfg["max_action"])
        r16, _ = _record_eval(ag2, "teacher", bf16=True)
        assert len(r16) == cfg["max_action"]
        for t, b in enumerate(r16):
            ref = torch.from_numpy(G[f"b256/logit/{t}"])
            fin = torch.isfinite(ref)
            assert torch.equal(fin, torch.isfinite(b["logit"]))
            span = (ref[fin].max() - ref[fin].min()).item()
            assert (b["logit"][fin] - ref[fin]).abs().max().item() <= BF16_LOGIT_FRAC * span, t
            close(b["value"], G[f"b256/value/{t}"], 5e-2, f"bf16 b256 value{t}")
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_checkpoint_roundtrip(R, dev, tmp_path):
    """Seq2SeqAgent.save / load (agent_dg.py:1466-1510): (1) after one optimizer step the checkpoint
    has the reference's structure — top-level modules, per-module entries, state_dict keys, optimizer
    layout and state (tests/golden ckpt/schema, written by the reference's own save); (2) a checkpoint
    in the reference schema built from the golden weights loads into a fresh agent and reproduces the
    reference's eval rollout; (3) save -> load into a differently initialised agent gives bitwise the
    same rollout."""
    import json
    param = R[0]
    G = golden("cfg1_rollout")
    cfg = GI.CFG1

    def env(seed):
        return SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=seed, mode="goal", instr_len=cfg["instr_len"],
                             variable_len=True)
    ag = _agent(R, env(8), cfg["max_action"])
    for m in ag.models:
        for sub in m.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    param.args.ml_weight = param.args.ml_weight_org
    ag.zero_grad()
    ag.accumulate_gradient("teacher")
    ag.optim_step()
    path = str(tmp_path / "ckpt")
    ag.save(3, path)
    st = torch.load(path, map_location="cpu", weights_only=True)
    want = json.loads(str(G["ckpt/schema"]))
    assert sorted(st.keys()) == sorted(want.keys())
    for name, ent in st.items():
        w, opt = want[name], ent["optimizer"]
        assert sorted(ent.keys()) == w["entries"] and ent["epoch"] == w["epoch"], name
        assert sorted(ent["state_dict"].keys()) == w["state_dict"], name
        assert sorted(opt.keys()) == w["optimizer"], name
        assert [sorted(g.keys()) for g in opt["param_groups"]] == w["param_groups"], name
        assert [len(g["params"]) for g in opt["param_groups"]] == w["n_params"], name
        assert sorted({k for v in opt["state"].values() for k in v.keys()}) == w["state_keys"], name
        assert len(opt["state"]) == w["n_state"], name
    # (2) a reference-schema checkpoint of the golden weights (what the reference would have written)
    from tests.helpers import oracle_weights
    W = oracle_weights(cfg["vl_layers"])
    ref_ckpt = {name: {"epoch": 7, "state_dict": sd, "optimizer": st[name]["optimizer"]}
                for name, sd in (("encoder", W.enc), ("decoder", W.dec), ("critic", W.critic), ("adaIn", W.ada))}
    ref_path = str(tmp_path / "ref_ckpt")
    torch.save(ref_ckpt, ref_path)
    fresh = _agent(R, env(7), cfg["max_action"], seed_weights=False)
    assert fresh.load(ref_path) == 6
    rec, traj = _record_eval(fresh, "argmax")
    assert len(rec) == int(G["eval/steps"])
    for t, r in enumerate(rec):
        close(r["logit"], G[f"eval/logit/{t}"], TOL, f"ckpt logit{t}")
    assert ["|".join(p[0] for p in tr["path"]) for tr in traj] == list(G["eval/paths"])
    # (3) save -> load round trip of the trained agent
    other = _agent(R, env(7), cfg["max_action"], seed_weights=False)
    assert other.load(path) == 3
    ag.env = env(7)
    a, _ = _record_eval(ag, "argmax")
    b, _ = _record_eval(other, "argmax")
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert torch.equal(x["logit"], y["logit"]) and torch.equal(x["value"], y["value"])


@pytest.mark.parametrize("cfg_name", ["cfg1", "cfg2"])
def test_step_graph_matches_eager(R, dev, cfg_name, monkeypatch):
    """Forward-only argmax rollouts replay every decision step after the first as ONE captured hipGraph
    (Seq2SeqAgent._graph_step: AdaIN, encoder, decoder and policy head). Against the same rollout run
    eagerly (DASA_STEP_GRAPH=0): identical trajectories, the summed per-step CE within 1e-5, and the
    graphs were captured and replayed."""
    param = R[0]
    if cfg_name == "cfg1":
        cfg = GI.CFG1

        def env():
            return SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=7, mode="goal", instr_len=cfg["instr_len"],
                                 variable_len=True)
        T = cfg["max_action"]
    else:
        cfg = GI.CFG2
        param.readme_train(["--d_vl_layers", str(cfg["vl_layers"]), "--batchSize", str(cfg["batch"]),
                            "--maxAction", "12"])

        def env():
            return SynthR2RBatch(SynthWorld(32, 0, 5), cfg["batch"], seed=11, mode="wander", instr_len=80)
        T = 12
    try:
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("DASA_STEP_GRAPH", mode)
            ag = _agent(R, env(), T)
            ag.feedback = "argmax"
            ag.loss = 0
            for m in (ag.encoder, ag.decoder, ag.critic):
                m.eval()
            with torch.no_grad():
                traj = ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
            res[mode] = (traj, float(ag.logs["ml_loss"][-1]) if ag.logs.get("ml_loss") else None,
                         ag._step_graphs)
        (t0, l0, g0), (t1, l1, g1) = res["0"], res["1"]
        assert g0 is None and g1 is not None and g1.captures >= 1 and g1.replays >= 1
        assert [x["path"] for x in t0] == [x["path"] for x in t1]
        if l0 is not None:
            assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0)), (l0, l1)
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


def test_graph_cache_keyed_by_numerics_mode(R, dev):
    """Captured regions are keyed by the GEMM numerics mode: an fp32 rollout after a bf16 one on the same
    agent replays fp32 graphs (its logits equal a fresh agent's fp32 rollout), not the bf16 captures."""
    cfg = GI.CFG1

    def env():
        return SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=7, mode="goal", instr_len=cfg["instr_len"],
                             variable_len=True)
    ag = _agent(R, env(), cfg["max_action"])
    r16, _ = _record_eval(ag, "argmax", bf16=True)
    ag.env = env()
    r32, _ = _record_eval(ag, "argmax")
    ag2 = _agent(R, env(), cfg["max_action"])
    ref, _ = _record_eval(ag2, "argmax")
    assert len(r32) == len(ref)
    for a, b in zip(r32, ref):
        assert torch.allclose(a["logit"], b["logit"], rtol=1e-6, atol=1e-6)
    assert any(not torch.allclose(a["logit"], b["logit"], rtol=1e-6, atol=1e-6) for a, b in zip(r16, ref))
