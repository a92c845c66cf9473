"""Generate tests/golden/*.npz by running the REFERENCE r2r_src code (imported here behind offline
shims, CPU fp32) on seeded weights/inputs. Container-only test infrastructure: needs /root/reference.

    python oracle/golden/make_golden.py                 # every fixture
    python oracle/golden/make_golden.py cfg2 cfg5       # the named fixtures only

Fixtures hold outputs only (plus gradient norms and seeded random "sketches" <grad, r_name> for
large tensors); tests regenerate weights (dasa_amd.synth.init_params) and inputs
(tests/golden_inputs.py) from the same seeds.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params  # noqa: E402
from oracle.golden.refimport import import_reference  # noqa: E402
from tests import golden_inputs as GI  # noqa: E402
from tests import helpers as H  # noqa: E402

OUT_DIR = os.path.join(ROOT, "tests", "golden")


def grad_record(out, prefix, named_params):
    """Norm, max, 8 Gaussian sketches and full values / a fixed row subset of every gradient
    (tests/helpers.py grad_record / check_grads)."""
    for name, p in named_params:
        if p.grad is None:
            continue
        H.grad_record(out, prefix + name, p.grad)


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def per_op(R):
    A = R.args
    out = {}
    torch.manual_seed(0)
    # DGAdaChannel ------------------------------------------------------------------
    ada = init_params(R.agent_dg.DGAdaChannel(2048), GI.SEED_ADA)
    f, d, g = GI.ada_inputs()
    y = ada(f, d)
    out["ada/out"] = f32(y)
    (y * g).sum().backward()
    grad_record(out, "ada/", ada.named_parameters())
    # AdaIN mu/sigma ----------------------------------------------------------------
    c, s = GI.adain_inputs()
    c.requires_grad_(True)
    s.requires_grad_(True)
    y = R.model.adaptive_instance_normalization(c, s)
    out["adain/out"] = f32(y)
    (y * GI.adain_grad_weights()).sum().backward()
    grad_record(out, "adain/", [("content", c), ("style", s)])
    # Shift attention ---------------------------------------------------------------
    for K in (5, 3):
        m = init_params(R.model.ShiftSoftDotAttention(1024, 2176, K), 20 + K)
        h, ctx, gw = GI.shift_inputs(K)
        h.requires_grad_(True)
        ctx.requires_grad_(True)
        wctx, attn = m(h, ctx, output_tilde=False)
        out[f"shift{K}/wctx"] = f32(wctx)
        out[f"shift{K}/attn"] = f32(attn)
        (wctx * gw).sum().backward()
        out[f"shift{K}/dh"] = f32(h.grad)
        grad_record(out, f"shift{K}/", [("ctx", ctx)] + list(m.named_parameters()))
    # SoftDot: instruction attention (tilde) and candidate logits ------------------
    h, ctx, mask, cand, g1, g2 = GI.softdot_inputs()
    att = init_params(R.model.SoftDotAttention(1024, 2048), 30)
    h1 = h.clone().requires_grad_(True)
    ht, alpha = att(h1, ctx, mask)
    out["softdot/h_tilde"], out["softdot/alpha"] = f32(ht), f32(alpha)
    (ht * g1).sum().backward()
    out["softdot/dh"] = f32(h1.grad)
    grad_record(out, "softdot/", att.named_parameters())
    catt = init_params(R.model.SoftDotAttention(1024, 2176), 31)
    h2 = h.clone().requires_grad_(True)
    cand = cand.clone().requires_grad_(True)
    _, logit = catt(h2, cand, output_prob=False)
    out["cand/logit"] = f32(logit)
    (logit * g2).sum().backward()
    out["cand/dh"] = f32(h2.grad)
    grad_record(out, "cand/", [("cand", cand)] + list(catt.named_parameters()))
    # Decoder step (eval: dropout off) ----------------------------------------------
    dec = init_params(R.model.BAttnDecoderLSTM(A.aemb, A.d_hidden_size, A.dropout, feature_size=2048 + 128,
                                               pred_back=False), GI.SEED_DEC).eval()
    action, feature, cand, h0, prev_h1, c0, ctx, mask = GI.decoder_inputs()
    h_1, c_1, logit, h_tilde, _ = dec(action, feature.clone(), cand.clone(), h0, prev_h1, c0, ctx, mask)
    for k, v in dict(h1=h_1, c1=c_1, logit=logit, h_tilde=h_tilde).items():
        out["dec/" + k] = f32(v)
    rng = np.random.default_rng(121)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)) for t in (h_1, c_1, logit, h_tilde)]
    ((h_1 * w[0]).sum() + (c_1 * w[1]).sum() + (logit * w[2]).sum() + (h_tilde * w[3]).sum()).backward()
    grad_record(out, "dec/", dec.named_parameters())
    # Critic ------------------------------------------------------------------------
    cr = init_params(R.model.Critic(), GI.SEED_CRITIC).eval()
    st = GI.critic_inputs()
    v = cr(st)
    out["critic/value"] = f32(v)
    (v * torch.arange(1.0, 5.0)).sum().backward()
    grad_record(out, "critic/", cr.named_parameters())
    # LXRT layer --------------------------------------------------------------------
    from pytorch_transformers import BertConfig
    cfg = BertConfig.from_pretrained("bert-base-uncased")
    lx = init_params(R.vilmodel.LXRTXLayer(cfg), 40).eval()
    lang, lmask, visn, vmask = GI.lxrt_inputs()
    with torch.no_grad():
        lo, vo = lx(lang, lmask[:, None, None, :], visn, vmask[:, None, None, :])
    out["lxrt/lang"], out["lxrt/visn"] = f32(lo), f32(vo)
    # DicEncoder (vl = 1, la = 9) ----------------------------------------------------
    A.d_vl_layers = 1
    enc = R.r2rmodel.DicEncoder(2176, A.d_enc_hidden_size, A.d_hidden_size, A.d_dropout_ratio, A.d_bidirectional,
                                A.d_transformer_update, A.d_bert_n_layers, A.d_reverse_input, A.d_top_lstm, 1,
                                A.d_la_layers, A.d_bert_type, update_add_layer=A.d_update_add_layer)
    init_params(enc, GI.SEED_ENC).eval()
    seq, mask, lengths, fimg = GI.encoder_inputs()
    ctx, dinit, ct, _, vis = enc(seq, mask, torch.tensor(lengths), f_t_all=fimg)
    for k, t in dict(ctx=ctx, decoder_init=dinit, c_t=ct, vision=vis).items():
        out["enc/" + k] = f32(t)
    rng = np.random.default_rng(151)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)) for t in (ctx, dinit, ct)]
    ((ctx * w[0]).sum() + (dinit * w[1]).sum() + (ct * w[2]).sum()).backward()
    grad_record(out, "enc/", enc.named_parameters())
    return out


class Recorder:
    """Wraps encoder/decoder forward of the reference agent to capture per-step tensors."""

    def __init__(self, agent):
        self.rec = {"ctx": [], "en_ht": [], "en_ct": [], "h1": [], "c1": [], "logit": [], "h_tilde": []}
        enc_fwd, dec_fwd = agent.encoder.forward, agent.decoder.forward

        def enc_wrap(*a, **k):
            r = enc_fwd(*a, **k)
            self.rec["ctx"].append(f32(r[0]))
            self.rec["en_ht"].append(f32(r[1]))
            self.rec["en_ct"].append(f32(r[2]))
            return r

        def dec_wrap(*a, **k):
            r = dec_fwd(*a, **k)
            self.rec["h1"].append(f32(r[0]))
            self.rec["c1"].append(f32(r[1]))
            self.rec["logit"].append(f32(r[2]))   # raw, before agent_dg.py:841's in-place mask
            self.rec["h_tilde"].append(f32(r[3]))
            return r
        agent.encoder.forward = enc_wrap
        agent.decoder.forward = dec_wrap


def make_agent(R, env, episode_len, tok=None, skip_bert=False):
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        agent = R.agent_dg.Seq2SeqAgent(env, "", tok, episode_len, "Dic")
    init_params(agent.encoder, GI.SEED_ENC, skip_prefix=("bert.",) if skip_bert else ())
    init_params(agent.decoder, GI.SEED_DEC)
    init_params(agent.critic, GI.SEED_CRITIC)
    init_params(agent.adaIn, GI.SEED_ADA)
    return agent


def schemas(R, agent):
    import json
    out = {}
    for name, mod in (("encoder", agent.encoder), ("decoder", agent.decoder), ("critic", agent.critic),
                      ("adaIn", agent.adaIn)):
        out["schema/" + name] = np.array(json.dumps({k: list(v.shape) for k, v in mod.state_dict().items()}))
    return out


def rollouts(R):
    A = R.args
    cfg = GI.CFG1
    A.d_vl_layers = cfg["vl_layers"]
    A.batchSize = cfg["batch"]
    A.maxAction = cfg["max_action"]
    A.views = 36          # set by utils.read_img_features (utils.py:286), which needs the absent TSVs
    out = {}
    world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
    # ---- eval, argmax feedback (the reference's validation path, agent_dg.py:1327) ----
    env = SynthR2RBatch(world, cfg["batch"], seed=7, mode="goal", instr_len=cfg["instr_len"], variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    out.update(schemas(R, agent))
    rec = Recorder(agent)
    for m in (agent.encoder, agent.decoder, agent.critic):
        m.eval()
    agent.feedback = "argmax"
    agent.loss = 0          # BaseAgent.test sets this before vl_rollout (agent_dg.py:65)
    with torch.no_grad():
        traj = agent.vl_rollout(train_ml=None, train_rl=False, reset=True)
    for k, v in rec.rec.items():
        for t, a in enumerate(v):
            if k == "ctx" and t > 0:
                continue      # ctx [B, L, 2048] kept for step 0 only (later steps pinned by en_ht/logits)
            out[f"eval/{k}/{t}"] = a
    out["eval/steps"] = np.array(len(rec.rec["logit"]))
    out["eval/ml_loss"] = np.array(agent.logs["ml_loss"][-1])
    out["eval/paths"] = np.array(["|".join(p[0] for p in tr["path"]) for tr in traj])
    # ---- train iteration with all dropout p = 0: teacher + 'sample' (argmax-sampled) ----
    env = SynthR2RBatch(world, cfg["batch"], seed=8, mode="goal", instr_len=cfg["instr_len"], variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    for mod in (agent.encoder, agent.decoder, agent.critic, agent.adaIn):
        for sub in mod.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    A.ml_weight = A.ml_weight_org
    orig_sample = torch.distributions.Categorical.sample
    torch.distributions.Categorical.sample = lambda self, *a, **k: self.probs.argmax(-1)
    try:
        agent.zero_grad()
        agent.accumulate_gradient("sample")
    finally:
        torch.distributions.Categorical.sample = orig_sample
    out["train/loss"] = np.array(agent.loss.item())
    out["train/ml_loss_teacher"] = np.array(agent.logs["ml_loss"][0])
    out["train/ml_loss_sample"] = np.array(agent.logs["ml_loss"][1])
    out["train/rl_loss"] = np.array(agent.logs["normalized_rl_loss"][-1])
    out["train/steps_teacher"] = np.array(agent.logs["viewsteps/teacher"][-1])
    out["train/steps_sample"] = np.array(agent.logs["viewsteps/sample"][-1])
    agent.loss.backward()
    for name, mod in (("encoder", agent.encoder), ("decoder", agent.decoder), ("critic", agent.critic),
                      ("adaIn", agent.adaIn)):
        grad_record(out, f"train/{name}.", mod.named_parameters())
    return out


def _zero_dropout(agent):
    for mod in (agent.encoder, agent.decoder, agent.critic, agent.adaIn):
        for sub in mod.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0


def _train_iteration(R, agent, out, prefix, forced=None, no_stop=False, **kw):
    """accumulate_gradient('sample') with argmax 'sampling' (or, given `forced`, the seeded action table
    of GI.reference_forced_sample), then backward; losses, logs + gradients."""
    A = R.args
    A.ml_weight = A.ml_weight_org
    orig_sample = torch.distributions.Categorical.sample
    uninstall = None
    if forced is not None:
        sample, install, uninstall = GI.reference_forced_sample(forced, R.utils, no_stop)
        install()
    else:
        sample = lambda self, *a, **k: self.probs.argmax(-1)   # noqa: E731
    torch.distributions.Categorical.sample = sample
    try:
        agent.zero_grad()
        agent.accumulate_gradient("sample", **kw)
    finally:
        torch.distributions.Categorical.sample = orig_sample
        if uninstall:
            uninstall()
    _record_losses(agent, out, prefix)
    agent.loss.backward()
    for name, mod in (("encoder", agent.encoder), ("decoder", agent.decoder), ("critic", agent.critic),
                      ("adaIn", agent.adaIn)):
        grad_record(out, f"{prefix}{name}.", mod.named_parameters())


def _record_losses(agent, out, prefix):
    out[prefix + "loss"] = np.array(agent.loss.item())
    out[prefix + "ml_loss_teacher"] = np.array(agent.logs["ml_loss"][0])
    out[prefix + "ml_loss_sample"] = np.array(agent.logs["ml_loss"][1])
    out[prefix + "rl_loss"] = np.array(agent.logs["normalized_rl_loss"][-1])
    out[prefix + "steps_teacher"] = np.array(agent.logs["viewsteps/teacher"][-1])
    out[prefix + "steps_sample"] = np.array(agent.logs["viewsteps/sample"][-1])
    for k in ("entropy", "critic_loss", "forth_loss", "total"):
        if agent.logs.get(k):
            out[prefix + "logs/" + k] = np.array(agent.logs[k], np.float64)


def _eval_rollout(agent, feedback, out, prefix, keep_states=()):
    """An eval rollout (no dropout) with per-step logits, critic values of the decoder state, and the
    states of the steps in keep_states."""
    rec = Recorder(agent)
    for m in (agent.encoder, agent.decoder, agent.critic):
        m.eval()
    agent.feedback = feedback
    agent.loss = 0
    with torch.no_grad():
        traj = agent.vl_rollout(train_ml=None, train_rl=False, reset=True)
        steps = len(rec.rec["logit"])
        for t in range(steps):
            out[f"{prefix}logit/{t}"] = rec.rec["logit"][t]
            # critic values of every step's decoder state (Critic(h_t), agent_dg.py:977)
            out[f"{prefix}value/{t}"] = f32(agent.critic(torch.from_numpy(rec.rec["h1"][t])))
            if t in keep_states or t == steps - 1:
                out[f"{prefix}h_tilde/{t}"] = rec.rec["h_tilde"][t]
                out[f"{prefix}c1/{t}"] = rec.rec["c1"][t]
    out[prefix + "steps"] = np.array(steps)
    out[prefix + "ml_loss"] = np.array(agent.logs["ml_loss"][-1])
    out[prefix + "paths"] = np.array(["|".join(p[0] for p in tr["path"]) for tr in traj])


def cfg2(R):
    """The bench configuration (B=20, vl=3, L=80): an argmax eval rollout (it ends when every agent
    stops), a 35-step teacher-forced eval rollout, and one training iteration at maxAction 5 (dropout
    0, argmax 'sampling')."""
    A = R.args
    cfg = GI.CFG2
    A.d_vl_layers, A.batchSize, A.views = cfg["vl_layers"], cfg["batch"], 36
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    out = {}
    A.maxAction = cfg["max_action"]
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["eval_seed"], mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    _eval_rollout(agent, "argmax", out, "eval/", keep_states=(0, 1))
    # the full 35 steps: teacher forcing on 'wander' episodes (the teacher never stops; the bench's
    # teacher rollout), so logits / critic values are pinned over a whole episode at B=20
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["eval_seed"], mode="wander", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    _eval_rollout(agent, "teacher", out, "teacher/", keep_states=(0, 17))
    A.maxAction = cfg["train_max_action"]
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["train_seed"], mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["train_max_action"])
    _zero_dropout(agent)
    _train_iteration(R, agent, out, "train/")
    # the same iteration with the sampled rollout's draws replaced by a seeded action table (valid
    # candidates only): the product runs its one-kernel policy head (teacher CE, sampled entropy and
    # log-prob) in both rollouts against it
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["train_seed"], mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["train_max_action"])
    _zero_dropout(agent)
    _train_iteration(R, agent, out, "trainf/", forced=GI.forced_table(cfg["train_max_action"], cfg["batch"]))
    return out


def cfg2_full(R):
    """The headline training iteration at its real length (GI.CFG2_FULL: B=20, vl=3, maxAction 35,
    'wander' episodes, dropout 0, sampled draws from a no-stop forced table): one
    accumulate_gradient('sample') — 35 teacher steps, 35 sampled steps and the A2C bootstrap — then
    backward. Records the raw logits of every decoder call (agent_dg.py:817; before the in-place mask of
    :841), the losses / per-step logs and every gradient."""
    A = R.args
    cfg = GI.CFG2_FULL
    A.d_vl_layers, A.batchSize, A.views, A.maxAction = cfg["vl_layers"], cfg["batch"], 36, cfg["max_action"]
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="wander", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    _zero_dropout(agent)
    logits = []
    dec_fwd = agent.decoder.forward

    def dec_wrap(*a, **k):
        r = dec_fwd(*a, **k)
        logits.append(f32(r[2]))
        return r
    agent.decoder.forward = dec_wrap
    out = {}
    _train_iteration(R, agent, out, "full/", forced=GI.forced_table(cfg["max_action"], cfg["batch"],
                                                                   seed=cfg["forced_seed"]), no_stop=True)
    out["full/n_decoder_calls"] = np.array(len(logits))
    for t, lg in enumerate(logits):
        out[f"full/logit/{t}"] = lg
    return out


def aug(R):
    """The aug half of the auglistener iteration (train.py:237-239): accumulate_gradient('sample',
    speaker=...) — the speaker back-translates each rollout's teacher path with the shared env-drop
    noise (speaker.py:293-295), the listener re-tokenises the instructions (agent_dg.py:656-677), both
    rollouts apply the noise after AdaIN (:780-785) and the A2C bootstrap applies it to the raw
    features (:946-952), the decoder with already_dropfeat=True (model.py:506-508, 556-557). Dropout 0
    except the env-drop mask (GI.FixedEnvDrop); sampled draws from the forced table."""
    import contextlib
    import importlib
    import io
    A = R.args
    cfg = GI.CFG_AUG
    if not hasattr(np, "bool"):
        np.bool = bool
    A.d_vl_layers, A.batchSize, A.views, A.maxAction = cfg["vl_layers"], cfg["batch"], 36, cfg["max_action"]
    A.maxDecode = cfg["max_decode"]
    with contextlib.redirect_stdout(io.StringIO()):
        stok = R.utils.Tokenizer(vocab=R.utils.read_vocab(os.path.join(ROOT, "tests", "golden", "train_vocab.txt")),
                                 encoding_length=A.maxInput)
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80, variable_len=True)
    agent = make_agent(R, env, cfg["max_action"], tok=GI.WordHashBTokenizer(A.maxInput))
    _zero_dropout(agent)
    agent.decoder.drop_env = GI.FixedEnvDrop(GI.env_drop_mask())
    spk_mod = importlib.import_module("speaker")
    with contextlib.redirect_stdout(io.StringIO()):
        spk = spk_mod.Speaker(env, agent, stok)
    GI.scale_params(init_params(spk.encoder, cfg["seed_enc"]), cfg["spk_scale"])
    GI.scale_params(init_params(spk.decoder, cfg["seed_dec"]), cfg["spk_scale"])
    margins = []
    dec_fwd = spk.decoder.forward

    def dec_rec(*a, **k):      # top-2 logit margin of every decoded word (an argmax flip needs < ~1e-4)
        r = dec_fwd(*a, **k)
        lg = r[0].detach().view(r[0].shape[0], -1).clone()
        lg[:, stok.word_to_index["<UNK>"]] = -float("inf")
        top = lg.topk(2, dim=1).values
        margins.append(float((top[:, 0] - top[:, 1]).min()))
        return r
    spk.decoder.forward = dec_rec
    insts = []
    reset = env.reset

    def reset_rec(batch=None, **k):
        if batch is not None:
            insts.append(np.stack([np.asarray(d["instr_encoding"], np.int64) for d in batch]))
        return reset(batch, **k)
    env.reset = reset_rec
    rec = Recorder(agent)
    out = {}
    _train_iteration(R, agent, out, "aug/", forced=GI.forced_table(cfg["max_action"], cfg["batch"]), speaker=spk)
    assert len(insts) == 2, len(insts)       # one back-translation per rollout (teacher, sample)
    for i, x in enumerate(insts):
        out[f"aug/instr_encoding/{i}"] = x
    for t, lg in enumerate(rec.rec["logit"]):
        out[f"aug/logit/{t}"] = lg
    out["aug/n_decoder_calls"] = np.array(len(rec.rec["logit"]))
    out["aug/speaker_min_margin"] = np.array(min(margins))
    return out


def optim(R):
    """Two training iterations, each zero_grad -> accumulate_gradient('sample') -> optim_step
    (agent_dg.py:1340-1405: backward, clip_grad_norm 40 on encoder + decoder, RMSprop on all four
    optimizers, LambdaLR on decoder / critic / adaIn): per iteration the loss, the clip norms, every
    optimizer's learning rate, and per parameter the RMSprop square_avg and the parameter change. (The
    second iteration's policy is sharp after RMSprop's ~10 lr sign(g) first step: some candidate
    probabilities underflow, which is why the forced draws count candidates from length2mask.)"""
    A = R.args
    cfg = GI.CFG_OPTIM
    A.d_vl_layers, A.batchSize, A.maxAction, A.views = cfg["vl_layers"], cfg["batch"], cfg["max_action"], 36
    world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    _zero_dropout(agent)
    A.ml_weight = A.ml_weight_org
    mods = (("encoder", agent.encoder, agent.encoder_optimizer), ("decoder", agent.decoder, agent.decoder_optimizer),
            ("critic", agent.critic, agent.critic_optimizer), ("adaIn", agent.adaIn, agent.adaIn_optimizer))
    norms = []
    orig_clip = torch.nn.utils.clip_grad_norm
    orig_sample = torch.distributions.Categorical.sample
    out = {}
    try:
        torch.nn.utils.clip_grad_norm = lambda params, m, *a, **k: norms.append(float(orig_clip(params, m, *a, **k)))
        for it in range(cfg["iters"]):
            sample, install, uninstall = GI.reference_forced_sample(
                GI.forced_table(cfg["max_action"], cfg["batch"], seed=GI.FORCED_SEED + it), R.utils)
            install()
            torch.distributions.Categorical.sample = sample
            before = {name: {k: p.detach().clone() for k, p in m.named_parameters()} for name, m, _ in mods}
            agent.zero_grad()
            agent.accumulate_gradient("sample")
            norms.clear()
            loss = agent.loss.item()
            agent.optim_step()
            out[f"opt{it}/loss"] = np.array(loss)
            out[f"opt{it}/clip_norms"] = np.array(norms, np.float64)      # encoder, decoder
            for name, m, opt in mods:
                out[f"opt{it}/lr/{name}"] = np.array([g["lr"] for g in opt.param_groups], np.float64)
                for k, p in m.named_parameters():
                    if p.grad is None:
                        continue
                    H.grad_record(out, f"opt{it}/delta/{name}.{k}", p.detach() - before[name][k])
                    H.grad_record(out, f"opt{it}/sq/{name}.{k}", opt.state[p]["square_avg"])
            uninstall()
    finally:
        torch.nn.utils.clip_grad_norm = orig_clip
        torch.distributions.Categorical.sample = orig_sample
    return out


def cfg4_readme(R):
    """cfg4 at the README finetune configuration (README.md:104-116: --d_update_add_layer True,
    d_vl_layers 3, batchSize 2): one training iteration at maxAction 6 with dropout 0 and the sampled
    draws from the forced table, so the LXRT stack (vl=3) and VisionEncoder backward are pinned."""
    A = R.args
    cfg = GI.CFG4R
    A.d_vl_layers, A.batchSize, A.maxAction, A.views = cfg["vl_layers"], cfg["batch"], cfg["max_action"], 36
    A.d_update_add_layer = True
    out = {}
    try:
        world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
        env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=cfg["instr_len"],
                            variable_len=True)
        agent = make_agent(R, env, cfg["max_action"])
        assert agent.encoder.bert.update_add_layer
        _zero_dropout(agent)
        _train_iteration(R, agent, out, "ft3/", forced=GI.forced_table(cfg["max_action"], cfg["batch"]))
    finally:
        A.d_update_add_layer = False
    return out


def pretrain(R):
    """--pretrain_model_name (agent_dg.py:165-188, README train flag): a DicAddActionPreTrain checkpoint
    directory written here (config.json with vl_layers=2 — the command line says 3 — and
    pytorch_model.bin holding bert.* plus the next_action / mlmhead pretraining heads, bert weights from
    init_params(seed_bert)), loaded by the reference agent through from_pretrained; the non-bert weights
    seeded as usual; an argmax eval rollout's logits and critic values. Records the checkpoint's config
    and key layout so the product test writes the same directory."""
    import importlib
    import json
    import tempfile
    A = R.args
    cfg = GI.CFG_PRE
    A.d_vl_layers, A.batchSize, A.maxAction, A.views = 3, cfg["batch"], cfg["max_action"], 36
    from pytorch_transformers import BertConfig
    pc = importlib.import_module("r2rpretrain_class")
    conf = BertConfig.from_pretrained("bert-base-uncased")
    conf.img_feature_dim, conf.img_feature_type = 2048 + A.angle_feat_size, ""
    conf.update_lang_bert = conf.update_add_layer = True
    conf.vl_layers, conf.la_layers, conf.action_space = cfg["vl_layers_ckpt"], cfg["la_layers"], 36
    pre = pc.DicAddActionPreTrain(conf)
    init_params(pre.bert, cfg["seed_bert"])
    d = tempfile.mkdtemp(prefix="dasa_pre_")
    with open(os.path.join(d, "config.json"), "w") as f:
        f.write(conf.to_json_string())
    sd = pre.state_dict()
    torch.save(sd, os.path.join(d, "pytorch_model.bin"))
    out = {"pre/config": np.array(conf.to_json_string()),
           "pre/head_schema": np.array(json.dumps({k: list(v.shape) for k, v in sd.items()
                                                   if not k.startswith("bert.")}, sort_keys=True))}
    A.pretrain_model_name = d
    try:
        world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
        env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=cfg["instr_len"],
                            variable_len=True)
        agent = make_agent(R, env, cfg["max_action"], skip_bert=True)
    finally:
        A.pretrain_model_name = None
    assert len(agent.encoder.bert.addlayer) == cfg["vl_layers_ckpt"]
    out["pre/vl_layers"] = np.array(len(agent.encoder.bert.addlayer))
    _eval_rollout(agent, "argmax", out, "pre/", keep_states=(0,))
    return out


def cfg5(R):
    """vl=6 (BASELINE configs[4]'s depth) at B=4: a teacher-forced eval rollout, fp32 reference."""
    A = R.args
    cfg = GI.CFG5
    A.d_vl_layers, A.batchSize, A.views, A.maxAction = cfg["vl_layers"], cfg["batch"], 36, cfg["max_action"]
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["seed"], mode="wander", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    out = {}
    _eval_rollout(agent, "teacher", out, "teacher/", keep_states=tuple(range(cfg["max_action"])))
    return out


def cfg5_b256(R):
    """configs[4] at its own batch (GI.CFG5_B256: B=256, vl=6, L<=80 variable): a 2-step teacher-forced
    eval rollout, fp32 — per-step raw logits, critic values and the last step's states."""
    A = R.args
    cfg = GI.CFG5_B256
    A.d_vl_layers, A.batchSize, A.views, A.maxAction = cfg["vl_layers"], cfg["batch"], 36, cfg["max_action"]
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["seed"], mode="wander", instr_len=cfg["instr_len"],
                        variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    out = {}
    _eval_rollout(agent, "teacher", out, "b256/")
    return out


def cfg4_full(R):
    """The README finetune iteration at its real length (GI.CFG4_FULL: --d_update_add_layer True, vl=3,
    B=2, maxAction 35, 'wander' episodes, dropout 0, no-stop forced draws): one
    accumulate_gradient('sample') — 35 teacher + 35 sampled steps + the A2C bootstrap — then backward.
    Raw logits of every decoder call, losses / logs, every gradient (LXRT stack and VisionEncoder
    included)."""
    A = R.args
    cfg = GI.CFG4_FULL
    A.d_vl_layers, A.batchSize, A.views, A.maxAction = cfg["vl_layers"], cfg["batch"], 36, cfg["max_action"]
    A.d_update_add_layer = True
    out = {}
    try:
        world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
        env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="wander", instr_len=cfg["instr_len"],
                            variable_len=True)
        agent = make_agent(R, env, cfg["max_action"])
        assert agent.encoder.bert.update_add_layer
        _zero_dropout(agent)
        logits = []
        dec_fwd = agent.decoder.forward

        def dec_wrap(*a, **k):
            r = dec_fwd(*a, **k)
            logits.append(f32(r[2]))
            return r
        agent.decoder.forward = dec_wrap
        _train_iteration(R, agent, out, "ft35/", forced=GI.forced_table(cfg["max_action"], cfg["batch"],
                                                                       seed=cfg["forced_seed"]), no_stop=True)
        out["ft35/n_decoder_calls"] = np.array(len(logits))
        for t, lg in enumerate(logits):
            out[f"ft35/logit/{t}"] = lg
    finally:
        A.d_update_add_layer = False
    return out


def checkpoint_schema(R):
    """The structure of a reference checkpoint (Seq2SeqAgent.save, agent_dg.py:1466-1487) after one
    optimizer step: top-level names, per-module entry names, state_dict keys, optimizer state layout."""
    import json
    import tempfile
    A = R.args
    cfg = GI.CFG1
    A.d_vl_layers, A.batchSize, A.maxAction, A.views = cfg["vl_layers"], cfg["batch"], cfg["max_action"], 36
    world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
    env = SynthR2RBatch(world, cfg["batch"], seed=8, mode="goal", instr_len=cfg["instr_len"], variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    _zero_dropout(agent)
    A.ml_weight = A.ml_weight_org
    agent.zero_grad()
    agent.accumulate_gradient("teacher")
    agent.optim_step()
    path = os.path.join(tempfile.mkdtemp(prefix="dasa_ckpt_"), "ckpt")
    agent.save(3, path)
    st = torch.load(path, map_location="cpu", weights_only=True)
    desc = {}
    for name, ent in st.items():
        opt = ent["optimizer"]
        desc[name] = {"entries": sorted(ent.keys()), "epoch": ent["epoch"],
                      "state_dict": sorted(ent["state_dict"].keys()),
                      "optimizer": sorted(opt.keys()),
                      "param_groups": [sorted(g.keys()) for g in opt["param_groups"]],
                      "n_params": [len(g["params"]) for g in opt["param_groups"]],
                      "state_keys": sorted({k for v in opt["state"].values() for k in v.keys()}),
                      "n_state": len(opt["state"])}
    os.remove(path)
    return {"ckpt/schema": np.array(json.dumps(desc, sort_keys=True))}


def finetune(R):
    """cfg4: the finetune path (--d_update_add_layer True, agent_dg.py:152; vilmodel.py:1408-1410 no
    longer detaches), so the LXRT layers and the VisionEncoder receive gradients. Records the LXRT
    layer backward on its own and one accumulate_gradient('sample') + backward with dropout 0."""
    A = R.args
    out = {}
    # LXRT layer backward (eval): parameter and input gradients ------------------------------
    from pytorch_transformers import BertConfig
    lx = init_params(R.vilmodel.LXRTXLayer(BertConfig.from_pretrained("bert-base-uncased")), 40).eval()
    lang, lmask, visn, vmask = GI.lxrt_inputs()
    lang.requires_grad_(True)
    visn.requires_grad_(True)
    lo, vo = lx(lang, lmask[:, None, None, :], visn, vmask[:, None, None, :])
    rng = np.random.default_rng(141)
    w = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)) for t in (lo, vo)]
    ((lo * w[0]).sum() + (vo * w[1]).sum()).backward()
    grad_record(out, "lxrt/", lx.named_parameters())
    grad_record(out, "lxrt_in/", [("lang", lang), ("visn", visn)])
    # train iteration on the finetune path ------------------------------------------------------
    cfg = GI.CFG4
    A.d_vl_layers = cfg["vl_layers"]
    A.batchSize = cfg["batch"]
    A.maxAction = cfg["max_action"]
    A.views = 36
    A.d_update_add_layer = True
    world = SynthWorld(n_viewpoints=16, feat_seed=0, graph_seed=3)
    env = SynthR2RBatch(world, cfg["batch"], seed=9, mode="goal", instr_len=cfg["instr_len"], variable_len=True)
    agent = make_agent(R, env, cfg["max_action"])
    assert agent.encoder.bert.update_add_layer
    for mod in (agent.encoder, agent.decoder, agent.critic, agent.adaIn):
        for sub in mod.modules():
            if isinstance(sub, torch.nn.Dropout):
                sub.p = 0.0
    A.ml_weight = A.ml_weight_org
    orig_sample = torch.distributions.Categorical.sample
    torch.distributions.Categorical.sample = lambda self, *a, **k: self.probs.argmax(-1)
    try:
        agent.zero_grad()
        agent.accumulate_gradient("sample")
    finally:
        torch.distributions.Categorical.sample = orig_sample
        A.d_update_add_layer = False
    out["ft/loss"] = np.array(agent.loss.item())
    out["ft/ml_loss_teacher"] = np.array(agent.logs["ml_loss"][0])
    out["ft/ml_loss_sample"] = np.array(agent.logs["ml_loss"][1])
    out["ft/rl_loss"] = np.array(agent.logs["normalized_rl_loss"][-1])
    agent.loss.backward()
    for name, mod in (("encoder", agent.encoder), ("decoder", agent.decoder), ("critic", agent.critic),
                      ("adaIn", agent.adaIn)):
        grad_record(out, f"ft/{name}.", mod.named_parameters())
    return out


def io_readers(R):
    """The reference's feature readers on tiny real-format files: utils.read_img_features on a TSV and
    env.Depth_Features on a (viewpointIds, values) .npy pair; records the keys and a SHA-256 of every
    decoded array. (base64.decodestring, which utils.py:306 calls, is base64.decodebytes' pre-3.9
    alias; it is re-exposed for this run.)"""
    import base64
    import hashlib
    import importlib.util
    import tempfile
    from dasa_amd.features import write_img_features
    A = R.args
    d = tempfile.mkdtemp(prefix="dasa_io_")
    img, keys, vals = GI.io_tables()
    tsv = os.path.join(d, "feats.tsv")
    write_img_features(tsv, img)
    if not hasattr(base64, "decodestring"):
        base64.decodestring = base64.decodebytes
    np.save(os.path.join(d, "ids.npy"), keys)
    np.save(os.path.join(d, "vals.npy"), vals)
    A.depth_index_file, A.depth_value_file = os.path.join(d, "ids.npy"), os.path.join(d, "vals.npy")
    # env.py raises the csv field limit at import (env.py:19) before the reader runs, as in train.py
    spec = importlib.util.spec_from_file_location("ref_env_io", os.path.join("/root/reference/r2r_src", "env.py"))
    env_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(env_mod)
    depth = env_mod.depth_features.depth_map
    A.mini, A.features = False, "imagenet"
    feats = R.utils.read_img_features(tsv)
    out = {"img/keys": np.array(sorted(feats)), "depth/keys": np.array(sorted(depth))}
    for tag, tab in (("img", feats), ("depth", depth)):
        for k in sorted(tab):
            a = np.ascontiguousarray(tab[k])
            out[f"{tag}/sha256/{k}"] = np.array(hashlib.sha256(a.tobytes()).hexdigest())
            out[f"{tag}/shape/{k}"] = np.array(a.shape)
            out[f"{tag}/dtype/{k}"] = np.array(str(a.dtype))
    return out


EVAL_SCANS = ["17DRP5sb8fy", "8194nk5LbLH", "GdvgFV5R1Z5"]


def eval_score(R):
    """Evaluation.score (eval.py:74-108) of the reference on its own connectivity graphs (three scans,
    tests/golden/connectivity holds copies) for synthetic R2R items and synthetic trajectories
    (random walks on the graph, some along the shortest path); utils.load_datasets (which reads the
    absent R2R json) is replaced by the item list. Inputs and outputs are both recorded."""
    import importlib.util
    import json
    import random
    import networkx as nx
    R.args.depth_index_file, R.args.depth_value_file = _tiny_depth_files()
    if "env" not in sys.modules or not hasattr(sys.modules["env"], "R2RBatch"):
        spec = importlib.util.spec_from_file_location("env", "/root/reference/r2r_src/env.py")
        m = importlib.util.module_from_spec(spec)
        sys.modules["env"] = m
        spec.loader.exec_module(m)
    import eval as ref_eval
    cwd = os.getcwd()
    os.chdir("/root/reference")          # load_nav_graphs opens connectivity/<scan>_connectivity.json
    try:
        graphs = R.utils.load_nav_graphs(EVAL_SCANS)
    finally:
        os.chdir(cwd)
    rng = random.Random(17)
    items, results = [], []
    pid = 1000
    for scan in EVAL_SCANS:
        G = graphs[scan]
        nodes = sorted(G.nodes())
        for _ in range(5):
            a, b = rng.sample(nodes, 2)
            path = nx.shortest_path(G, a, b, weight="weight")
            items.append({"path_id": pid, "scan": scan, "path": path, "heading": 0.0,
                          "instructions": ["go", "walk there", "stop"]})
            for i in range(3):
                traj = [(a, rng.uniform(0, 6.28), 0.0)]
                if i == 0:
                    traj += [(v, rng.uniform(0, 6.28), 0.0) for v in path[1:]]      # the exact path
                else:
                    cur = a
                    for _ in range(rng.randint(0, 7)):
                        cur = rng.choice(sorted(G.neighbors(cur)))
                        for _ in range(rng.randint(0, 2)):                          # turns in place
                            traj.append((cur, rng.uniform(0, 6.28), 0.0))
                        traj.append((cur, rng.uniform(0, 6.28), 0.0))
                results.append({"instr_id": "%d_%d" % (pid, i), "trajectory": traj})
            pid += 1
    ref_eval.load_datasets = lambda splits: items
    cwd = os.getcwd()
    os.chdir("/root/reference")
    try:
        ev = ref_eval.Evaluation(["val_seen"], EVAL_SCANS, None)
    finally:
        os.chdir(cwd)
    summary, scores = ev.score(results)
    return {"eval/items": np.array(json.dumps(items)), "eval/results": np.array(json.dumps(results)),
            "eval/summary": np.array(json.dumps({k: float(v) for k, v in summary.items()}, sort_keys=True)),
            "eval/scores": np.array(json.dumps({k: [float(x) for x in v] for k, v in scores.items()}, sort_keys=True))}


def _tiny_depth_files():
    import tempfile
    d = tempfile.mkdtemp(prefix="dasa_dep_")
    _, keys, vals = GI.io_tables()
    np.save(os.path.join(d, "ids.npy"), keys)
    np.save(os.path.join(d, "vals.npy"), vals)
    return os.path.join(d, "ids.npy"), os.path.join(d, "vals.npy")


def speaker(R):
    """Speaker.infer_batch (speaker.py:265-350) of the reference: SpeakerEncoder over the teacher path's
    candidate / panorama features, SpeakerDecoder argmax decoding. The reference's own Tokenizer on its
    train_vocab.txt (a copy is tests/golden/train_vocab.txt). numpy 2 dropped the np.bool alias that
    speaker.py:308 uses; it is re-exposed for this run. Records ctx, per-step logits, words, lengths."""
    import contextlib
    import importlib
    import io
    A = R.args
    cfg = GI.SPEAKER
    if not hasattr(np, "bool"):
        np.bool = bool
    A.maxDecode, A.batchSize, A.views = cfg["max_decode"], cfg["batch"], 36
    with contextlib.redirect_stdout(io.StringIO()):
        tok = R.utils.Tokenizer(vocab=R.utils.read_vocab(os.path.join(ROOT, "tests", "golden", "train_vocab.txt")),
                                encoding_length=A.maxInput)
    world = SynthWorld(n_viewpoints=cfg["viewpoints"], feat_seed=0, graph_seed=cfg["graph_seed"])
    env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80, variable_len=True)
    listener = make_agent(R, env, 5)
    spk_mod = importlib.import_module("speaker")
    with contextlib.redirect_stdout(io.StringIO()):
        spk = spk_mod.Speaker(env, listener, tok)
    init_params(spk.encoder, cfg["seed_enc"])
    init_params(spk.decoder, cfg["seed_dec"])
    rec = {"ctx": None, "logits": [], "h": []}
    enc_fwd, dec_fwd = spk.encoder.forward, spk.decoder.forward

    def enc_wrap(*a, **k):
        r = enc_fwd(*a, **k)
        rec["ctx"] = f32(r)
        return r

    def dec_wrap(*a, **k):
        r = dec_fwd(*a, **k)
        rec["logits"].append(f32(r[0]))
        rec["h"].append(f32(r[1]))
        return r
    spk.encoder.forward, spk.decoder.forward = enc_wrap, dec_wrap
    env.reset()
    with torch.no_grad():
        insts = spk.infer_batch()
    out = {"spk/ctx": rec["ctx"], "spk/insts": np.asarray(insts, np.int64), "spk/steps": np.array(len(rec["logits"])),
           "spk/schema_encoder": np.array(__import__("json").dumps({k: list(v.shape) for k, v in spk.encoder.state_dict().items()})),
           "spk/schema_decoder": np.array(__import__("json").dumps({k: list(v.shape) for k, v in spk.decoder.state_dict().items()})),
           "spk/vocab_size": np.array(tok.vocab_size())}
    for t, (lg, h) in enumerate(zip(rec["logits"], rec["h"])):
        out[f"spk/logit/{t}"] = lg
        out[f"spk/h/{t}"] = h
    return out


FIXTURES = {
    "ops": per_op,
    "cfg1_rollout": lambda R: {**rollouts(R), **checkpoint_schema(R)},
    "cfg4_finetune": finetune,
    "cfg2": cfg2,
    "cfg2_full": cfg2_full,
    "cfg5": cfg5,
    "io": io_readers,
    "eval": eval_score,
    "speaker": speaker,
    "aug": aug,
    "optim": optim,
    "cfg4_readme": cfg4_readme,
    "pretrain": pretrain,
    "cfg5_b256": cfg5_b256,
    "cfg4_full": cfg4_full,
}


def main():
    R = import_reference()
    os.makedirs(OUT_DIR, exist_ok=True)
    names = sys.argv[1:] or list(FIXTURES)
    names = ["cfg4_finetune" if n == "finetune" else n for n in names]
    for name in names:
        torch.manual_seed(0)
        out = FIXTURES[name](R)
        np.savez_compressed(os.path.join(OUT_DIR, name + ".npz"), **out)
        print(f"{name}.npz:", len(out), "arrays", flush=True)


if __name__ == "__main__":
    main()
