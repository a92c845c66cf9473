"""Policy heads of r2r_src/model.py on the MI355X kernels: SoftDotAttention, ShiftSoftDotAttention,
BAttnDecoderLSTM, Critic and the mu/sigma AdaIN.

Parameters are held in the same nn.Linear / nn.LSTMCell containers as the reference, so state_dict keys
and shapes are identical; forward() never calls those containers — it runs the HIP
kernels through dasa_amd.functional. Removed by design (no caller observes them): the in-place dropout
on the caller's `feature` / `cand_feat` (model.py:508, 557) — the dropped copies are local here.
"""
import torch
import torch.nn as nn

from .. import functional as DF
from .. import ops
from .param import args


class SoftDotAttention(nn.Module):
    """model.py:253-296."""

    def __init__(self, query_dim, ctx_dim):
        super().__init__()
        self.linear_in = nn.Linear(query_dim, ctx_dim, bias=False)
        self.sm = nn.Softmax(dim=1)
        self.linear_out = nn.Linear(query_dim + ctx_dim, query_dim, bias=False)
        self.tanh = nn.Tanh()

    def forward(self, h, context, mask=None, output_tilde=True, output_prob=True):
        if output_tilde and output_prob:
            return DF.SoftDotTildeFn.apply(h, context, mask, self.linear_in.weight, self.linear_out.weight)
        if not output_tilde and not output_prob and mask is None:
            logit = DF.CandLogitFn.apply(h, context, self.linear_in.weight)
            q = ops.linear(h.detach(), self.linear_in.weight.detach())
            wctx = ops.softdot_fwd(q, context.detach(), None)[2]     # unused by the decoder (model.py:559)
            return wctx, logit
        # the other combinations (no README caller) on the same kernels: dasa_softdot_fwd / _bwd
        wctx, attn = DF.SoftDotFn.apply(h, context, mask, self.linear_in.weight, not output_prob)
        if output_tilde:
            return DF.linear(torch.cat((wctx, h), 1), self.linear_out.weight, None, "tanh"), attn
        return wctx, attn

    def logits(self, h, cand):
        """Raw candidate scores (output_tilde=False, output_prob=False) without the unused wctx."""
        return DF.CandLogitFn.apply(h, cand, self.linear_in.weight)


class ShiftSoftDotAttention(nn.Module):
    """model.py:300-353: soft attention over the 36 views followed by a learned K-tap circular shift
    along each of the 3 elevation rows."""

    def __init__(self, query_dim, ctx_dim, kernel_size=3):
        super().__init__()
        self.linear_in = nn.Linear(query_dim, ctx_dim, bias=False)
        self.linear_shift = nn.Linear(query_dim, kernel_size)
        self.sm = nn.Softmax(dim=1)
        self.linear_out = nn.Linear(query_dim + ctx_dim, query_dim, bias=False)
        self.tanh = nn.Tanh()
        self.kernel_size = kernel_size
        self.padding_size = kernel_size // 2

    def forward(self, h, context, mask=None, output_tilde=True, output_prob=True):
        if mask is not None:
            raise NotImplementedError("masked shift attention is not used by the reference decoder")
        if context.shape[1] != 36:
            raise ValueError("ShiftSoftDotAttention expects the 36-view panorama (3 x 12)")
        wctx, attn = DF.ShiftAttnFn.apply(h, context.contiguous(), self.linear_in.weight, self.linear_shift.weight,
                                          self.linear_shift.bias)
        if not output_prob:   # the raw scores (model.py:346-347), detached: no caller differentiates them
            q = ops.linear(h.detach(), self.linear_in.weight.detach())
            attn = ops.softdot_fwd(q, context.detach(), None, want_probs=False, want_wctx=False)[0]
        if output_tilde:
            return DF.linear(torch.cat((wctx, h), 1), self.linear_out.weight, None, "tanh"), attn
        return wctx, attn


class BAttnDecoderLSTM(nn.Module):
    """model.py:422-574 (use_shift / pred_back / decoder_consistent_drop supported; pred_pm is not)."""

    def __init__(self, embedding_size, hidden_size, dropout_ratio, feature_size=2048 + 4, pred_back=False):
        super().__init__()
        self.embedding_size = embedding_size
        self.feature_size = feature_size
        self.hidden_size = hidden_size
        self.embedding = nn.Sequential(nn.Linear(args.angle_feat_size, self.embedding_size), nn.Tanh())
        self.drop = nn.Dropout(p=dropout_ratio)
        self.drop_env = nn.Dropout(p=args.featdropout)
        self.lstm = nn.LSTMCell(embedding_size + feature_size, hidden_size)
        if args.use_shift:
            self.feat_att_layer = ShiftSoftDotAttention(hidden_size, feature_size, args.shift_kernel_size)
        else:
            self.feat_att_layer = SoftDotAttention(hidden_size, feature_size)
        self.attention_layer = SoftDotAttention(hidden_size, hidden_size * 2)
        self.candidate_att_layer = SoftDotAttention(hidden_size, feature_size)
        self.pred_back = pred_back
        if self.pred_back:
            self.back_candidate_att_layer = SoftDotAttention(hidden_size, feature_size)
        self.pred_pm = args.pred_pm
        if self.pred_pm:
            raise NotImplementedError("--pred_pm progress monitor is outside the DASA hot path")
        self.input_noise = None
        self.output_noise = None

    def init_noise(self, shape):
        dev = self.lstm.weight_hh.device
        self.input_noise = self.drop(torch.ones(shape, device=dev))
        self.output_noise = self.drop(torch.ones(shape, device=dev))

    def _drop_env_feat(self, feat, angle):
        """feat[..., :-angle] = drop_env(feat[..., :-angle]) (model.py:506-508, 556-557), out of place:
        the counter-RNG dropout kernel for an nn.Dropout, else the module itself (a caller's stand-in)."""
        if isinstance(self.drop_env, nn.Dropout):
            return DF.feat_drop(feat, self.drop_env.p, self.training, angle)
        return torch.cat((self.drop_env(feat[..., :-angle]), feat[..., -angle:]), -1)

    def forward(self, action, feature, cand_feat, h_0, prev_h1, c_0, ctx, ctx_mask=None, already_dropfeat=False):
        training = self.training
        p = self.drop.p
        angle = args.angle_feat_size
        aux_outputs = {}
        a_emb = DF.linear(action, self.embedding[0].weight, self.embedding[0].bias, "tanh")
        a_emb = DF.dropout(a_emb, p, training)
        if not already_dropfeat:
            feature = self._drop_env_feat(feature, angle)
        prev_h1_drop = DF.dropout(prev_h1, p, training)
        attn_feat, _ = self.feat_att_layer(prev_h1_drop, feature, output_tilde=False)
        h_1, c_1 = DF.LSTMCellFn.apply(a_emb, attn_feat, prev_h1, c_0, self.lstm.weight_ih, self.lstm.weight_hh,
                                       self.lstm.bias_ih, self.lstm.bias_hh)
        if args.decoder_consistent_drop:
            h_1_drop = h_1 * self.input_noise
        else:
            h_1_drop = DF.dropout(h_1, p, training)
        h_tilde, alpha = self.attention_layer(h_1_drop, ctx, ctx_mask)
        if args.decoder_consistent_drop:
            h_tilde_drop = h_tilde * self.output_noise
        else:
            h_tilde_drop = DF.dropout(h_tilde, p, training)
        if not already_dropfeat:
            cand_feat = self._drop_env_feat(cand_feat, angle)
        logit = self.candidate_att_layer.logits(h_tilde_drop, cand_feat)
        if self.pred_back:
            q = prev_h1 if args.back_input == "pre" else h_tilde_drop
            aux_outputs["back_logit"] = self.back_candidate_att_layer.logits(q, cand_feat)
        return h_1, c_1, logit, h_tilde, aux_outputs


class Critic(nn.Module):
    """model.py:970-982."""

    def __init__(self):
        super().__init__()
        self.dim = args.critic_dim
        self.state2value = nn.Sequential(nn.Linear(self.dim, self.dim), nn.ReLU(), nn.Dropout(args.dropout),
                                         nn.Linear(self.dim, 1))

    def forward(self, state):
        l0, drop, l3 = self.state2value[0], self.state2value[2], self.state2value[3]
        x = DF.linear(state, l0.weight, l0.bias, "relu")
        x = DF.dropout(x, drop.p, self.training)
        return DF.linear(x, l3.weight, l3.bias).squeeze()


def calc_mean_std(feat, eps=1e-5, dim=-1):
    """model.py:1822-1830 (returned for API parity; the fused kernel below does not need it)."""
    assert feat.dim() == 3
    var = feat.var(dim=dim, keepdim=True) + eps
    return feat.mean(dim=dim, keepdim=True), var.sqrt()


def adaptive_instance_normalization(content_feat, style_feat, out=None):
    """model.py:1832-1840, one wave per row (two wave-shuffle reductions per operand) on gfx950;
    differentiable in content and style (dasa_adain_musigma_bwd)."""
    assert content_feat.size() == style_feat.size()
    return DF.adain_musigma(content_feat, style_feat, out=out)


# ----------------------------------------------------------------------------- speaker (back-translation)
def _bilstm(lstm, x):
    """A single-layer bidirectional nn.LSTM over the full padded length (no packing: speaker.py feeds
    padded batches, model.py:1010 / 1025) on the persistent recurrence kernel."""
    B, T, _ = x.shape
    lens = torch.full((B,), T, dtype=torch.int32, device=x.device)
    out, _, _ = DF.BiLSTMFn.apply(x.contiguous(), lens, lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0,
                                  lstm.bias_hh_l0, lstm.weight_ih_l0_reverse, lstm.weight_hh_l0_reverse,
                                  lstm.bias_ih_l0_reverse, lstm.bias_hh_l0_reverse)
    return out


class SpeakerEncoder(nn.Module):
    """model.py:984-1032: bi-LSTM over the trajectory's action (candidate) features, SoftDot attention of
    each step over its 36-view panorama, a second bi-LSTM. Inference path (Speaker.infer_batch);
    training the speaker is outside the policy hot path."""

    def __init__(self, feature_size, hidden_size, dropout_ratio, bidirectional):
        super().__init__()
        self.num_directions = 2 if bidirectional else 1
        self.hidden_size = hidden_size
        self.num_layers = 1
        self.feature_size = feature_size
        if not bidirectional:
            raise NotImplementedError("the DASA speaker is bidirectional (param.py --bidir default True)")
        self.lstm = nn.LSTM(feature_size, self.hidden_size // self.num_directions, self.num_layers, batch_first=True,
                            bidirectional=bidirectional)
        self.drop = nn.Dropout(p=dropout_ratio)
        self.drop3 = nn.Dropout(p=args.featdropout)
        self.attention_layer = SoftDotAttention(self.hidden_size, feature_size)
        self.post_lstm = nn.LSTM(self.hidden_size, self.hidden_size // self.num_directions, self.num_layers,
                                 batch_first=True, bidirectional=bidirectional)

    def forward(self, action_embeds, feature, lengths, already_dropfeat=False):
        """action_embeds [B, T, F+A], feature [B, T, 36, F+A] -> ctx [B, T, hidden]."""
        training = self.training
        angle = args.angle_feat_size
        x = action_embeds
        if not already_dropfeat:
            x = DF.feat_drop(x, self.drop3.p, training, angle)
        ctx = DF.dropout(_bilstm(self.lstm, x), self.drop.p, training)
        B, T, _ = ctx.shape
        if not already_dropfeat:
            feature = DF.feat_drop(feature, self.drop3.p, training, angle)
        x, _ = self.attention_layer(ctx.contiguous().view(-1, self.hidden_size),
                                    feature.contiguous().view(B * T, -1, self.feature_size))
        x = DF.dropout(x.view(B, T, -1), self.drop.p, training)
        return DF.dropout(_bilstm(self.post_lstm, x), self.drop.p, training)


class SpeakerDecoder(nn.Module):
    """model.py:1034-1080: word embedding -> LSTM -> masked SoftDot attention over the encoder context ->
    vocabulary projection. Inference path (no autograd: infer_batch runs it under no_grad)."""

    def __init__(self, vocab_size, embedding_size, padding_idx, hidden_size, dropout_ratio):
        super().__init__()
        self.hidden_size = hidden_size
        self.embedding = torch.nn.Embedding(vocab_size, embedding_size, padding_idx)
        self.lstm = nn.LSTM(embedding_size, hidden_size, batch_first=True)
        self.drop = nn.Dropout(dropout_ratio)
        self.attention_layer = SoftDotAttention(hidden_size, hidden_size)
        self.projection = nn.Linear(hidden_size, vocab_size)
        self.baseline_projection = nn.Sequential(nn.Linear(hidden_size, 128), nn.ReLU(), nn.Dropout(dropout_ratio),
                                                 nn.Linear(128, 1))

    def forward(self, words, ctx, ctx_mask, h0, c0):
        """words [B, L] int64, ctx [B, T, H], ctx_mask [B, T] bool, h0 / c0 [1, B, H] ->
        (logit [B, L, V], h1 [1, B, H], c1 [1, B, H])."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("SpeakerDecoder runs the inference path only (call it under torch.no_grad())")
        B, L = words.shape
        H, E = self.hidden_size, self.embedding.weight.shape[1]
        training = self.training
        emb = torch.empty(B * L, E, dtype=torch.float32, device=ctx.device)
        ops.gather_rows(self.embedding.weight, words.reshape(-1).to(torch.int32), None, None, emb)
        emb = DF.dropout(emb.view(B, L, E), self.drop.p, training)
        lw = self.lstm
        h, c = h0.reshape(B, H).contiguous(), c0.reshape(B, H).contiguous()
        outs = []
        for t in range(L):                       # nn.LSTM over the L words (L = 1 while decoding)
            gates = ops.linear(emb[:, t], lw.weight_ih_l0, lw.bias_ih_l0)
            ops.linear(h, lw.weight_hh_l0, lw.bias_hh_l0, out=gates, beta=1.0)
            h, c, _ = ops.lstm_cell_fwd(gates, c)
            outs.append(h)
        x = outs[0].unsqueeze(1) if L == 1 else torch.stack(outs, 1)
        x = DF.dropout(x, self.drop.p, training)
        ctx_x = ctx if L == 1 else ctx.repeat_interleave(L, 0)
        mask_x = ctx_mask if L == 1 else ctx_mask.repeat_interleave(L, 0)
        x, _ = self.attention_layer(x.reshape(B * L, H), ctx_x.contiguous(), mask_x)
        x = DF.dropout(x.view(B, L, H), self.drop.p, training)
        logit = ops.linear(x, self.projection.weight, self.projection.bias)
        return logit, h.unsqueeze(0), c.unsqueeze(0)
