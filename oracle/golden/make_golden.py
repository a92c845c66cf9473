"""Generate tests/golden/*.npz by running the REFERENCE r2r_src code (imported here behind offline
shims, CPU fp32) on seeded weights/inputs. Container-only test infrastructure: needs /root/reference.

    python oracle/golden/make_golden.py            # every fixture
    python oracle/golden/make_golden.py finetune   # tests/golden/cfg4_finetune.npz only

Fixtures hold outputs only (plus gradient norms and seeded random "sketches" <grad, r_name> for
large tensors); tests regenerate weights (dasa_amd.synth.init_params) and inputs
(tests/golden_inputs.py) from the same seeds.
"""
import os
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params  # noqa: E402
from oracle.golden.refimport import import_reference  # noqa: E402
from tests import golden_inputs as GI  # noqa: E402

OUT_DIR = os.path.join(ROOT, "tests", "golden")


def sketch_vec(name, n):
    return np.random.default_rng(zlib.crc32(name.encode())).standard_normal(n).astype(np.float64)


def grad_record(out, prefix, named_params, full_max=4096):
    for name, p in named_params:
        if p.grad is None:
            continue
        g = p.grad.detach().double().flatten().numpy()
        key = prefix + name
        out["gnorm/" + key] = np.array(np.linalg.norm(g))
        out["gsketch/" + key] = np.array(g @ sketch_vec(key, g.size))
        if g.size <= full_max:
            out["gfull/" + key] = p.grad.detach().numpy().astype(np.float32)


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
    out["adain/out"] = f32(R.model.adaptive_instance_normalization(c, s))
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


def make_agent(R, env, episode_len):
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        agent = R.agent_dg.Seq2SeqAgent(env, "", None, episode_len, "Dic")
    init_params(agent.encoder, GI.SEED_ENC)
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


def main():
    R = import_reference()
    os.makedirs(OUT_DIR, exist_ok=True)
    if sys.argv[1:] == ["finetune"]:
        ft = finetune(R)
        np.savez_compressed(os.path.join(OUT_DIR, "cfg4_finetune.npz"), **ft)
        print("cfg4_finetune.npz:", len(ft), "arrays")
        return
    ops = per_op(R)
    np.savez_compressed(os.path.join(OUT_DIR, "ops.npz"), **ops)
    print("ops.npz:", len(ops), "arrays")
    ro = rollouts(R)
    np.savez_compressed(os.path.join(OUT_DIR, "cfg1_rollout.npz"), **ro)
    print("cfg1_rollout.npz:", len(ro), "arrays")
    ft = finetune(R)
    np.savez_compressed(os.path.join(OUT_DIR, "cfg4_finetune.npz"), **ft)
    print("cfg4_finetune.npz:", len(ft), "arrays")


if __name__ == "__main__":
    main()
