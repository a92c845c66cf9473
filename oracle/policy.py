"""CPU oracle: a from-scratch restatement of the DASA agent_dg policy path in plain fp32 PyTorch-CPU.

TEST INFRASTRUCTURE ONLY. Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker / the reported CPU baseline — never by dasa_amd (the product path, which has no
CPU fallback). Pinned against tests/golden/*.npz, which were generated from the reference itself
imported in the survey container (oracle/golden/make_golden.py).

Parameters are passed as a flat dict keyed exactly like the reference modules' state_dicts
(SURVEY.md §8(b)): e.g. P["bert.lalayer.0.attention.self.query.weight"].
Every function cites the reference code it restates.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

ANGLE = 128
FEAT = 2048

# Dropout probabilities of the README config: decoder --dropout 0.5, --featdropout 0.4, encoder
# --d_dropout_ratio 0.4, BERT hidden/attention 0.1. Tests set them to 0 for deterministic train-mode runs.
DROP = dict(dec=0.5, feat=0.4, enc=0.4, bert=0.1)


def _drop(x, p, train, gen=None):
    if not train or p <= 0:
        return x
    return F.dropout(x, p, True)


def linear(x, W, b=None):
    y = x @ W.t()
    return y + b if b is not None else y


# ------------------------------------------------------------------------ depth-guided AdaIN
def dg_ada_channel(f, d, W, b):
    """DGAdaChannel.forward, ab_type 'a', a_type 'sigmoid' (agent_dg.py:1525-1547): sigmoid(a_fc(d)) * f."""
    return torch.sigmoid(linear(d, W, b)) * f


def calc_mean_std(feat, eps=1e-5):
    """model.py:1822-1830 (unbiased variance over the last dim, + eps, sqrt)."""
    var = feat.var(dim=-1, keepdim=True) + eps
    return feat.mean(dim=-1, keepdim=True), var.sqrt()


def adaptive_instance_normalization(content, style):
    """model.py:1832-1840."""
    sm, ss = calc_mean_std(style)
    cm, cs = calc_mean_std(content)
    return (content - cm) / cs * ss + sm


# ------------------------------------------------------------------------ attention heads
def softdot(h, ctx, W_in, W_out=None, mask=None, output_tilde=True, output_prob=True):
    """SoftDotAttention.forward (model.py:268-296). Softmax over dim 1 (nn.Softmax() on 2-D)."""
    target = linear(h, W_in)                              # [B, D]
    logit = torch.einsum("bnd,bd->bn", ctx, target)       # raw scores
    attn = logit
    if mask is not None:
        attn = attn.masked_fill(mask.bool(), -float("inf"))
        logit = attn                                      # masked_fill_ aliases `logit` in the reference
    p = torch.softmax(attn, dim=1)
    wctx = torch.einsum("bn,bnd->bd", p, ctx)
    out_attn = p if output_prob else logit
    if output_tilde:
        return torch.tanh(linear(torch.cat([wctx, h], 1), W_out)), out_attn
    return wctx, out_attn


def shift_softdot(h, ctx, W_in, W_shift, b_shift, kernel_size, output_prob=True):
    """ShiftSoftDotAttention.forward with output_tilde=False (model.py:318-353).

    The 3 elevation rows x 12 headings circular pad + grouped conv1d is restated as the circular
    correlation a'[r][j] = sum_k w_k a[r][(j + k - K//2) mod 12].
    """
    target = linear(h, W_in)
    logit = torch.einsum("bnd,bd->bn", ctx, target)
    a = torch.softmax(logit, dim=1)
    B = a.shape[0]
    w = torch.softmax(linear(h, W_shift, b_shift), dim=-1)   # [B, K]
    a3 = a.view(B, 3, 12)
    P = kernel_size // 2
    shifted = torch.zeros_like(a3)
    for k in range(kernel_size):
        shifted = shifted + w[:, k].view(B, 1, 1) * torch.roll(a3, shifts=-(k - P), dims=2)
    wctx = torch.einsum("bn,bnd->bd", shifted.reshape(B, 36), ctx)
    return wctx, (a if output_prob else logit)


def lstm_cell(x, h, c, W_ih, W_hh, b_ih, b_hh):
    """nn.LSTMCell (gate order i, f, g, o)."""
    g = linear(x, W_ih, b_ih) + linear(h, W_hh, b_hh)
    i, f, gg, o = g.chunk(4, 1)
    c1 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    return torch.sigmoid(o) * torch.tanh(c1), c1


# ------------------------------------------------------------------------ decoder / critic
def decoder_step(P, action, feature, cand_feat, prev_h1, c_0, ctx, ctx_mask, kernel_size=5, train=False,
                 dropout=None, featdropout=None, already_dropfeat=False):
    """BAttnDecoderLSTM.forward (model.py:472-574), use_shift, no pred_back/pred_pm.

    Returns (h_1, c_1, logit, h_tilde). The LSTM's previous hidden state is `prev_h1` (the caller
    passes the previous h_tilde, agent_dg.py:817-820); h_0 is unused by the reference.
    """
    dropout = DROP["dec"] if dropout is None else dropout
    featdropout = DROP["feat"] if featdropout is None else featdropout
    a_emb = torch.tanh(linear(action, P["embedding.0.weight"], P["embedding.0.bias"]))
    a_emb = _drop(a_emb, dropout, train)
    if not already_dropfeat and train:
        feature = torch.cat([_drop(feature[..., :-ANGLE], featdropout, train), feature[..., -ANGLE:]], -1)
    attn_feat, _ = shift_softdot(_drop(prev_h1, dropout, train), feature, P["feat_att_layer.linear_in.weight"],
                                 P["feat_att_layer.linear_shift.weight"], P["feat_att_layer.linear_shift.bias"],
                                 kernel_size)
    h_1, c_1 = lstm_cell(torch.cat([a_emb, attn_feat], 1), prev_h1, c_0, P["lstm.weight_ih"], P["lstm.weight_hh"],
                         P["lstm.bias_ih"], P["lstm.bias_hh"])
    h_tilde, _ = softdot(_drop(h_1, dropout, train), ctx, P["attention_layer.linear_in.weight"],
                         P["attention_layer.linear_out.weight"], mask=ctx_mask)
    h_tilde_drop = _drop(h_tilde, dropout, train)
    if not already_dropfeat and train:
        cand_feat = torch.cat([_drop(cand_feat[..., :-ANGLE], featdropout, train), cand_feat[..., -ANGLE:]], -1)
    _, logit = softdot(h_tilde_drop, cand_feat, P["candidate_att_layer.linear_in.weight"], output_tilde=False,
                       output_prob=False)
    return h_1, c_1, logit, h_tilde


def critic(P, state, train=False, dropout=None):
    """Critic.forward (model.py:970-982)."""
    dropout = DROP["dec"] if dropout is None else dropout
    x = torch.relu(linear(state, P["state2value.0.weight"], P["state2value.0.bias"]))
    x = _drop(x, dropout, train)
    return linear(x, P["state2value.3.weight"], P["state2value.3.bias"]).squeeze()


# ------------------------------------------------------------------------ BERT / LXRT
def gelu(x):
    """vilmodel.py:125-131 (erf form)."""
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def layer_norm(x, P, pre, eps=1e-12):
    return F.layer_norm(x, (x.shape[-1],), P[pre + ".weight"], P[pre + ".bias"], eps)


def mh_attention(P, pre, x, ctx, addmask, heads=12, train=False, p=None):
    """BertSelfAttention / BertOutAttention core (vilmodel.py:214-236, 481-506)."""
    p = DROP["bert"] if p is None else p
    q = linear(x, P[pre + ".query.weight"], P[pre + ".query.bias"])
    k = linear(ctx, P[pre + ".key.weight"], P[pre + ".key.bias"])
    v = linear(ctx, P[pre + ".value.weight"], P[pre + ".value.bias"])
    B, Lq, H = q.shape
    Lk = k.shape[1]
    dh = H // heads
    q = q.view(B, Lq, heads, dh).permute(0, 2, 1, 3)
    k = k.view(B, Lk, heads, dh).permute(0, 2, 1, 3)
    v = v.view(B, Lk, heads, dh).permute(0, 2, 1, 3)
    s = q @ k.transpose(-1, -2) / math.sqrt(dh)
    if addmask is not None:
        s = s + addmask[:, None, None, :]
    pr = _drop(torch.softmax(s, -1), p, train)
    return (pr @ v).permute(0, 2, 1, 3).reshape(B, Lq, H)


def self_output(P, pre, y, x, train=False, p=None):
    """BertSelfOutput / BertOutput: LayerNorm(dropout(dense(y)) + x) (vilmodel.py:239-250, 296-309)."""
    p = DROP["bert"] if p is None else p
    return layer_norm(_drop(linear(y, P[pre + ".dense.weight"], P[pre + ".dense.bias"]), p, train) + x, P,
                      pre + ".LayerNorm")


def bert_attention(P, pre, x, addmask, train=False):
    """BertAttention (vilmodel.py:253-280)."""
    return self_output(P, pre + ".output", mh_attention(P, pre + ".self", x, x, addmask, train=train), x, train)


def ffn(P, inter, out, x, train=False):
    """BertIntermediate + BertOutput (vilmodel.py:283-309)."""
    h = gelu(linear(x, P[inter + ".dense.weight"], P[inter + ".dense.bias"]))
    return self_output(P, out, h, x, train)


def bert_layer(P, pre, x, addmask, train=False):
    """BertLayer (vilmodel.py:312-325)."""
    a = bert_attention(P, pre + ".attention", x, addmask, train)
    return ffn(P, pre + ".intermediate", pre + ".output", a, train)


def lxrt_layer(P, pre, lang, lang_mask, visn, visn_mask, train=False):
    """LXRTXLayer.forward (vilmodel.py:1014-1064). One shared visual_attention for both directions."""
    xa = pre + ".visual_attention"
    l_att = self_output(P, xa + ".output", mh_attention(P, xa + ".att", lang, visn, visn_mask, train=train), lang, train)
    v_att = self_output(P, xa + ".output", mh_attention(P, xa + ".att", visn, lang, lang_mask, train=train), visn, train)
    l_att = bert_attention(P, pre + ".lang_self_att", l_att, lang_mask, train)
    v_att = bert_attention(P, pre + ".visn_self_att", v_att, visn_mask, train)
    l_out = ffn(P, pre + ".lang_inter", pre + ".lang_output", l_att, train)
    v_out = ffn(P, pre + ".visn_inter", pre + ".visn_output", v_att, train)
    return l_out, v_out


def dic_model(P, input_ids, attention_mask, img_feats, la_layers, vl_layers, train=False, lang_cache=None,
              update_lang_bert=False):
    """DicModel.forward (vilmodel.py:1327-1423) with keys prefixed 'bert.'. attention_mask: 1 = token.

    lang_cache: optional precomputed language-stack output (it does not depend on img_feats).
    Returns (sequence_output, pooled_output, visn_output, text_embeds).
    """
    B, L = input_ids.shape
    ext = (1.0 - attention_mask.float()) * -10000.0                      # [B, L]
    if lang_cache is None:
        e = (P["bert.embeddings.word_embeddings.weight"][input_ids]
             + P["bert.embeddings.position_embeddings.weight"][:L][None]
             + P["bert.embeddings.token_type_embeddings.weight"][0])
        x = _drop(layer_norm(e, P, "bert.embeddings.LayerNorm"), DROP["bert"], train)
        for i in range(la_layers):
            x = bert_layer(P, "bert.lalayer.%d" % i, x, ext, train)
    else:
        x = lang_cache
    if not update_lang_bert:                  # vilmodel.py:1377-1378 (README default: BERT not trained)
        x = x.detach()
    text = x
    v = linear(img_feats, P["bert.vision_encoder.visn_fc.weight"], P["bert.vision_encoder.visn_fc.bias"])
    v = _drop(layer_norm(v, P, "bert.vision_encoder.visn_layer_norm"), DROP["bert"], train)
    img_mask = torch.zeros(B, img_feats.shape[1])                        # (1 - 1) * -10000
    lang = text
    for i in range(vl_layers):
        lang, v = lxrt_layer(P, "bert.addlayer.%d" % i, lang, ext, v, img_mask, train)
    pooled = torch.tanh(linear(lang[:, 0], P["bert.pooler.dense.weight"], P["bert.pooler.dense.bias"]))
    return lang, pooled, v, text


def bilstm_packed(P, x, lengths, H):
    """Single-layer bidirectional nn.LSTM over pack_padded_sequence(x, lengths) (r2rmodel.py:2339-2343).

    Returns out [B, L, 2H] ([fwd, bwd], zeros past each length) and (h_n, c_n) [2, B, H].
    """
    B, L, _ = x.shape
    out = torch.zeros(B, L, 2 * H)
    hn = torch.zeros(2, B, H)
    cn = torch.zeros(2, B, H)
    lens = torch.as_tensor(lengths)
    for d, sfx in ((0, ""), (1, "_reverse")):
        Wih, Whh = P["lstm.weight_ih_l0" + sfx], P["lstm.weight_hh_l0" + sfx]
        bias = P["lstm.bias_ih_l0" + sfx] + P["lstm.bias_hh_l0" + sfx]
        xp = linear(x, Wih) + bias
        h = torch.zeros(B, H)
        c = torch.zeros(B, H)
        order = range(L) if d == 0 else range(L - 1, -1, -1)
        for t in order:
            act = (t < lens).float().unsqueeze(1)
            g = xp[:, t] + linear(h, Whh)
            i, f, gg, o = g.chunk(4, 1)
            c1 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h1 = torch.sigmoid(o) * torch.tanh(c1)
            c = act * c1 + (1 - act) * c
            h = act * h1 + (1 - act) * h
            out[:, t, d * H:(d + 1) * H] = act * h1
        hn[d], cn[d] = h, c
    return out, hn, cn


def reverse_valid(x, lengths):
    """r2rmodel.py:2326-2330: reverse the first lengths[b] positions of each row, zero the rest."""
    out = torch.zeros_like(x)
    for b, n in enumerate(lengths):
        n = int(n)
        out[b, :n] = x[b, :n].flip(0)
    return out


def dic_encoder(P, seq, mask, lengths, f_t_all, la_layers=9, vl_layers=3, H=1024, train=False, d_dropout=None,
                lang_cache=None, update_add_layer=False):
    """DicEncoder.forward (r2rmodel.py:2272-2365), reverse_input + top_lstm + bidirectional.

    mask: [B, L] bool, True at padding (agent_dg.py:276). Returns (ctx, decoder_init, c_t, mask, vision_out).
    """
    L = mask.shape[1]
    embeds, pooled, vis, text = dic_model(P, seq[:, :L], ~mask, f_t_all, la_layers, vl_layers, train, lang_cache)
    if not update_add_layer:                  # vilmodel.py:1408-1410, r2rmodel.py:2320-2321
        embeds, vis = embeds.detach(), vis.detach()
    embeds = reverse_valid(embeds, lengths)
    out, hn, cn = bilstm_packed(P, embeds, lengths, H)
    h_t = torch.cat([hn[1], hn[0]], 1)        # (enc_h_t[-1], enc_h_t[-2]) = (bwd, fwd)
    c_t = torch.cat([cn[1], cn[0]], 1)
    decoder_init = torch.tanh(linear(h_t, P["encoder_lstm2decoder_ht.weight"], P["encoder_lstm2decoder_ht.bias"]))
    c_t = linear(c_t, P["encoder_lstm2decoder_ct.weight"], P["encoder_lstm2decoder_ct.bias"])
    ctx = _drop(out, DROP["enc"] if d_dropout is None else d_dropout, train)
    return ctx, decoder_init, c_t, mask, vis


# ------------------------------------------------------------------------ rollout
def length2mask(length, size=None):
    """utils.length2mask (utils.py:503-508): True where index > len-1."""
    size = int(max(length)) if size is None else size
    return torch.arange(size).unsqueeze(0) > (torch.as_tensor(length) - 1).unsqueeze(1)


def sort_batch(obs):
    """Seq2SeqAgent._sort_batch (agent_dg.py:262-284)."""
    seq = np.array([ob["instr_encoding"] for ob in obs])
    lens = np.argmax(seq == 0, axis=1)
    lens[lens == 0] = seq.shape[1]
    seq_t = torch.from_numpy(seq)
    lens_t = torch.from_numpy(lens)
    lens_t, perm = lens_t.sort(0, True)
    sorted_seq = seq_t[perm]
    mask = (sorted_seq == 0)[:, :int(lens_t[0])]
    return sorted_seq.long(), mask.bool(), [int(x) for x in lens_t], [int(x) for x in perm]


def input_feat(obs):
    """get_input_feat (agent_dg.py:286-323)."""
    B = len(obs)
    a = torch.from_numpy(np.stack([np.array([math.sin(ob["heading"]), math.cos(ob["heading"]),
                                             math.sin(ob["elevation"]), math.cos(ob["elevation"])] * (ANGLE // 4),
                                            dtype=np.float32) for ob in obs]))
    f = torch.from_numpy(np.stack([ob["feature"] for ob in obs]).astype(np.float32))
    d = torch.from_numpy(np.stack([ob["dfeature"] for ob in obs]).astype(np.float32))
    leng = [len(ob["candidate"]) + 1 for ob in obs]
    cf = np.zeros((B, max(leng), FEAT + ANGLE), np.float32)
    cd = np.zeros_like(cf)
    for i, ob in enumerate(obs):
        for j, c in enumerate(ob["candidate"]):
            cf[i, j] = c["feature"]
            cd[i, j] = c["dfeature"]
    return a, f, d, torch.from_numpy(cf), torch.from_numpy(cd), leng


def teacher_action(obs, ended, ignoreid=-100):
    """agent_dg.py:325-344."""
    a = np.zeros(len(obs), dtype=np.int64)
    for i, ob in enumerate(obs):
        if ended[i]:
            a[i] = ignoreid
        else:
            for k, c in enumerate(ob["candidate"]):
                if c["viewpointId"] == ob["teacher"]:
                    a[i] = k
                    break
            else:
                assert ob["teacher"] == ob["viewpoint"]
                a[i] = len(ob["candidate"])
    return torch.from_numpy(a)


def make_equiv_action(env, a_t, perm_obs, perm_idx, traj=None):
    """agent_dg.py:358-391 (panoramic action -> discretized simulator actions)."""
    def take(i, sim, *a):
        sim.makeAction(*a)
        if traj is not None:
            traj[i].append(sim.getState().location.viewpointId)
    for i, idx in enumerate(perm_idx):
        action = a_t[i]
        if action != -1:
            sel = perm_obs[i]["candidate"][action]
            src, trg = perm_obs[i]["viewIndex"], sel["pointId"]
            sl, tl = src // 12, trg // 12
            sim = env.env.sims[idx]
            while sl < tl:
                take(i, sim, 0, 0, 1)
                sl += 1
            while sl > tl:
                take(i, sim, 0, 0, -1)
                sl -= 1
            while sim.getState().viewIndex != trg:
                take(i, sim, 0, 1, 0)
            assert sel["viewpointId"] == sim.getState().navigableLocations[sel["idx"]].viewpointId
            take(i, sim, sel["idx"], 0, 0)


class Weights:
    """Flat parameter dicts for the four reference modules (agent_dg.py:161-200)."""

    def __init__(self, enc, dec, critic, ada):
        self.enc, self.dec, self.critic, self.ada = enc, dec, critic, ada


def vl_rollout(W, env, feedback, *, la_layers=9, vl_layers=3, episode_len=35, kernel_size=5, train_ml=None,
               train_rl=False, train=False, gamma=0.9, obs=None, sample_fn=None, hoist_lang=False, record=None,
               update_add_layer=False):
    """Seq2SeqAgent.vl_rollout (agent_dg.py:633-1033) for the README config without speaker
    (consistent_drop off, so the decoder's own drop_env applies in train mode).

    Returns dict(loss, ml_loss, steps, traj, logits[t], h_t[t], ...). `sample_fn(probs) -> a_t`
    replaces Categorical sampling when given (deterministic tests).
    """
    if feedback in ("teacher", "argmax"):
        train_rl = False
    obs = np.array(env.reset()) if obs is None else np.array(obs)
    B = len(obs)
    seq, seq_mask, seq_lengths, perm_idx = sort_batch(obs)
    perm_obs = obs[perm_idx]
    traj = [[ob["viewpoint"]] for ob in perm_obs]
    last_dist = np.array([ob["distance"] for ob in perm_obs], np.float32)
    ended = np.array([False] * B)
    rewards, hidden_states, policy_log_probs, masks, entropys = [], [], [], [], []
    ml_loss = 0.0
    logits_rec, h_rec, a_rec = [], [], []
    lang_cache = None
    h_t = c_t = h1 = None
    ctx = None
    for t in range(episode_len):
        a_in, f_t, d_t, cf, cd, cleng = input_feat(perm_obs)
        df_t = f_t.clone()
        df_t[:, :, :-ANGLE] = dg_ada_channel(f_t[:, :, :-ANGLE], d_t[:, :, :-ANGLE], W.ada["a_fc.weight"],
                                             W.ada["a_fc.bias"])
        cf[:, :, :-ANGLE] = dg_ada_channel(cf[:, :, :-ANGLE].clone(), cd[:, :, :-ANGLE].clone(), W.ada["a_fc.weight"],
                                           W.ada["a_fc.bias"])
        if hoist_lang and lang_cache is None:
            L = seq_mask.shape[1]
            _, _, _, lang_cache = dic_model(W.enc, seq[:, :L], ~seq_mask, f_t, la_layers, 0, train)
        ctx, en_ht, en_ct, _, _ = dic_encoder(W.enc, seq, seq_mask, seq_lengths, f_t.clone(), la_layers, vl_layers,
                                              train=train, lang_cache=lang_cache if hoist_lang else None,
                                              update_add_layer=update_add_layer)
        if t == 0:
            h_t, c_t, logit, h1 = decoder_step(W.dec, a_in, df_t, cf, en_ht, en_ct, ctx, seq_mask, kernel_size, train)
        else:
            h_t, c_t, logit, h1 = decoder_step(W.dec, a_in, df_t, cf, h1, c_t, ctx, seq_mask, kernel_size, train)
        hidden_states.append(h_t)
        logits_rec.append(logit.detach().clone())      # raw (pre-mask) candidate logits
        h_rec.append((h_t.detach().clone(), c_t.detach().clone(), h1.detach().clone()))
        cmask = length2mask(cleng)
        logit = logit.masked_fill(cmask, -float("inf"))
        target = teacher_action(perm_obs, ended)
        ml_loss = ml_loss + F.cross_entropy(logit, target, ignore_index=-100, reduction="sum")
        if feedback == "teacher":
            a_t = target
        elif feedback == "argmax":
            a_t = logit.max(1)[1].detach()
            policy_log_probs.append(F.log_softmax(logit, 1).gather(1, a_t.unsqueeze(1)))
        else:
            probs = F.softmax(logit, 1)
            dist = torch.distributions.Categorical(probs)
            entropys.append(dist.entropy())
            a_t = (sample_fn(probs) if sample_fn is not None else dist.sample()).detach()
            policy_log_probs.append(dist.log_prob(a_t))
        cpu_a = a_t.numpy().copy()
        for i, nid in enumerate(cpu_a):
            if nid == cleng[i] - 1 or nid == -100:
                cpu_a[i] = -1
        a_rec.append(cpu_a.copy())
        make_equiv_action(env, cpu_a, perm_obs, perm_idx, traj)
        obs = np.array(env._get_obs())
        perm_obs = obs[perm_idx]
        dist_ = np.array([ob["distance"] for ob in perm_obs], np.float32)
        reward = np.zeros(B, np.float32)
        mask = np.ones(B, np.float32)
        for i in range(B):
            if ended[i]:
                reward[i] = 0.0
                mask[i] = 0.0
            elif cpu_a[i] == -1:
                reward[i] = 2.0 if dist_[i] < 3 else -2.0
            else:
                r = -(dist_[i] - last_dist[i])
                if r > 0:
                    reward[i] = 1
                elif r < 0:
                    reward[i] = -1
                else:
                    raise NameError("The action doesn't change the move")
        rewards.append(reward)
        masks.append(mask)
        last_dist[:] = dist_
        ended[:] = np.logical_or(ended, cpu_a == -1)
        if ended.all():
            break
    loss = 0.0
    rl_loss = None
    if train_rl:
        a_in, f_t, d_t, cf, cd, cleng = input_feat(perm_obs)
        last_h, _, _, _ = decoder_step(W.dec, a_in, f_t, cf, h1, c_t, ctx, seq_mask, kernel_size, train)
        last_value = critic(W.critic, last_h, train).detach()
        disc = np.zeros(B, np.float32)
        for i in range(B):
            if not ended[i]:
                disc[i] = last_value[i]
        rl_loss = 0.0
        total = 0
        for t in range(len(rewards) - 1, -1, -1):
            disc = disc * gamma + rewards[t]
            m = torch.from_numpy(masks[t])
            r = torch.from_numpy(disc.copy())
            v = critic(W.critic, hidden_states[t], train)
            a = (r - v).detach()
            rl_loss = rl_loss + (-policy_log_probs[t] * a * m).sum()
            rl_loss = rl_loss + (((r - v) ** 2) * m).sum() * 0.5
            if feedback == "sample":
                rl_loss = rl_loss + (-0.01 * entropys[t] * m).sum()
            total = total + np.sum(masks[t])
        rl_loss = rl_loss / total
        loss = loss + rl_loss
    if train_ml is not None:
        loss = loss + ml_loss * train_ml / B
    return dict(loss=loss, ml_loss=ml_loss, rl_loss=rl_loss, steps=len(rewards), logits=logits_rec, states=h_rec,
                actions=a_rec, perm_idx=perm_idx, seq_lengths=seq_lengths, traj=traj)


def state_dict_numpy(module):
    return {k: v.detach().cpu().clone() for k, v in module.state_dict().items()}
