"""BERT / LXMERT blocks of r2r_src/vilmodel.py used by DicModel, on the MI355X kernels.

Same module tree and parameter names as the reference (so `bert.*` checkpoints load unchanged);
forward() runs fused HIP kernels: MFMA GEMMs with bias/GELU epilogues (dasa_gemm_f32), a fused
dropout+residual+LayerNorm (dasa_layernorm_fwd) and a per-(batch, head) LDS-resident masked
attention core (dasa_mha_fwd). Attention masks arrive in the reference's additive extended form
[B, 1, 1, L] (0 / -10000).
"""
import math
import os

import torch
import torch.nn as nn

from .. import functional as DF
from .. import graph
from .. import ops
from .param import args

BertLayerNorm = nn.LayerNorm   # vilmodel.py:141-145 (apex is bypassed there too)


def extended_mask(attention_mask):
    """The reference's additive attention mask ((1 - m) * -10000 as [B, 1, 1, L], vilmodel.py:1343-1347) for a
    0 / 1 token mask, built by a fill + select instead of torch's float subtract / multiply kernels: those
    carry packed-FP32 VALU (v_pk_*_f32), whose results the r06 reproducer shows corrupted on lanes 48-63
    while a bf16x6 GEMM of the concurrent language pipe starts on the same CU (profiles/r06/pk_repro/;
    DESIGN §4 r06). Same bits: -0.0 where m != 0 (0 * -10000), -10000.0 elsewhere."""
    m = attention_mask
    if m.is_floating_point():
        return ((1.0 - m.float()) * -10000.0).unsqueeze(1).unsqueeze(2)
    ext = torch.full(m.shape, -10000.0, dtype=torch.float32, device=m.device).masked_fill_(m != 0, -0.0)
    return ext.unsqueeze(1).unsqueeze(2)

class BertConfig:
    """bert-base-uncased hyper-parameters (the values BertConfig.from_pretrained('bert-base-uncased')
    yields, r2rmodel.py:2229), built locally: no network."""

    _BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02, layer_norm_eps=1e-12, output_attentions=False,
                 output_hidden_states=False)

    def __init__(self, **kw):
        for k, v in dict(self._BASE, **kw).items():
            setattr(self, k, v)

    @classmethod
    def from_pretrained(cls, name="bert-base-uncased", **kw):
        if "large" in str(name):
            kw = dict(dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096), **kw)
        return cls(**kw)


def gelu(x):
    """vilmodel.py:125-131 (exact erf form) on the device."""
    return ops.act_fwd(x, "gelu")


def _addmask(mask, B):
    """[B,1,1,L] additive -> [B, L] contiguous (or None)."""
    if mask is None:
        return None
    return mask.reshape(B, -1).contiguous().float()


def _lin(x, m, act=None):
    return DF.linear(x, m.weight, m.bias, act)


def _needs_grad(*ts):
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


def _attn_dtype(x, N, ctx=None):
    """Storage dtype of Q/K/V on a no-grad path: bf16 under ops.bf16_matmul with bf16 activations (the bf16
    attention core then runs), else None (fp32)."""
    ok = ops.bf16_acts_ok(x, N) and (ctx is None or ops.bf16_acts_ok(ctx, N))
    return torch.bfloat16 if ok and ops.bf16_attn_on() else None


def _fused_weights(owner, mods):
    """Concatenated [W_1; W_2; ...] / [b_1; ...] of several nn.Linear (one wide MFMA GEMM instead of
    several narrow ones), cached until any of the parameters changes (data_ptr or in-place version).
    Stream-safe: a use on another stream than the one that built the cache waits for the build."""
    params = [t for m in mods for t in (m.weight, m.bias)]
    key = tuple((t.data_ptr(), t._version) for t in params)
    cache = getattr(owner, "_fused_cache", None)
    cur = torch.cuda.current_stream()
    if cache is not None and cache[0] == key and torch.cuda.is_current_stream_capturing():
        return cache[1], cache[2]    # built by the pre-capture warm-up, which the capture stream follows
    if cache is None or cache[0] != key:
        with torch.no_grad():
            W = torch.cat([m.weight for m in mods], 0).contiguous()
            b = torch.cat([m.bias for m in mods], 0).contiguous()
        ev = torch.cuda.Event()
        ev.record(cur)
        cache = (key, W, b, ev, cur)
        owner._fused_cache = cache
    elif cur != cache[4]:
        cur.wait_event(cache[3])
        cache[1].record_stream(cur)
        cache[2].record_stream(cur)
    return cache[1], cache[2]


class BertEmbeddings(nn.Module):
    """vilmodel.py:147-176: word + position + token_type(0) -> LayerNorm -> dropout, one kernel."""

    def __init__(self, config):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size, padding_idx=0)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None, position_ids=None):
        if position_ids is not None or (token_type_ids is not None and bool((token_type_ids != 0).any())):
            raise NotImplementedError("explicit position ids / non-zero token types are not on the DASA path")
        p = self.dropout.p if self.training else 0.0
        return ops.bert_embed(input_ids, self.word_embeddings.weight, self.position_embeddings.weight,
                              self.token_type_embeddings.weight[0], self.LayerNorm.weight, self.LayerNorm.bias,
                              self.LayerNorm.eps, p, DF.new_seed() if p > 0 else 0)


class BertSelfAttention(nn.Module):
    """vilmodel.py:179-236."""

    def __init__(self, config):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError("hidden size not a multiple of heads")
        self.output_attentions = config.output_attentions
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = int(config.hidden_size / config.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.dropout = nn.Dropout(config.attention_probs_dropout_prob)

    def forward(self, hidden_states, attention_mask, head_mask=None):
        if head_mask is not None:
            raise NotImplementedError("head_mask")
        if _needs_grad(hidden_states, self.query.weight, self.key.weight, self.value.weight):
            q, k, v = _lin(hidden_states, self.query), _lin(hidden_states, self.key), _lin(hidden_states, self.value)
        else:   # one [M, 3H] GEMM; Q/K/V are row-strided views the attention kernel reads in place
            W, b = _fused_weights(self, (self.query, self.key, self.value))
            # configs[4]'s bf16 mode: Q/K/V stored bf16 for the bf16 attention core (ops.mha)
            qkv = ops.linear(hidden_states, W, b, out_dtype=_attn_dtype(hidden_states, W.shape[0]))
            Hs = self.all_head_size
            q, k, v = qkv[..., :Hs], qkv[..., Hs:2 * Hs], qkv[..., 2 * Hs:]
        ctx = DF.mha(q, k, v, _addmask(attention_mask, q.shape[0]), self.num_attention_heads,
                     1.0 / math.sqrt(self.attention_head_size), self.dropout.p, self.training)
        return (ctx,)


class BertSelfOutput(nn.Module):
    """vilmodel.py:239-250: LayerNorm(dropout(dense(h)) + input) — dropout+residual+LN fused."""

    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor):
        return DF.layer_norm(_lin(hidden_states, self.dense), self.LayerNorm.weight, self.LayerNorm.bias,
                             self.LayerNorm.eps, res=input_tensor, p=self.dropout.p, training=self.training)


class BertAttention(nn.Module):
    """vilmodel.py:253-280."""

    def __init__(self, config):
        super().__init__()
        self.self = BertSelfAttention(config)
        self.output = BertSelfOutput(config)

    def forward(self, input_tensor, attention_mask, head_mask=None):
        s = self.self(input_tensor, attention_mask, head_mask)
        return (self.output(s[0], input_tensor),) + s[1:]


class BertIntermediate(nn.Module):
    """vilmodel.py:283-293: GELU fused into the GEMM epilogue."""

    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.intermediate_size)
        if config.hidden_act != "gelu":
            raise NotImplementedError("only the gelu BERT configuration is on the DASA path")

    def forward(self, hidden_states):
        if not _needs_grad(hidden_states, self.dense.weight) and ops.bf16_acts_ok(hidden_states, self.dense.out_features):
            # bf16 matmul mode (configs[4]): the GELU output's one consumer is BertOutput's bf16 GEMM, which
            # rounds its A operand to bf16 anyway — store it rounded (half the bytes written and re-read)
            return ops.linear(hidden_states, self.dense.weight, self.dense.bias, act="gelu", out_dtype=torch.bfloat16)
        return _lin(hidden_states, self.dense, "gelu")


class BertOutput(nn.Module):
    """vilmodel.py:296-309."""

    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.intermediate_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor):
        return DF.layer_norm(_lin(hidden_states, self.dense), self.LayerNorm.weight, self.LayerNorm.bias,
                             self.LayerNorm.eps, res=input_tensor, p=self.dropout.p, training=self.training)


class BertLayer(nn.Module):
    """vilmodel.py:312-325."""

    def __init__(self, config):
        super().__init__()
        self.attention = BertAttention(config)
        self.intermediate = BertIntermediate(config)
        self.output = BertOutput(config)

    def forward(self, hidden_states, attention_mask, head_mask=None):
        a = self.attention(hidden_states, attention_mask, head_mask)
        return (self.output(self.intermediate(a[0]), a[0]),) + a[1:]


class BertPooler(nn.Module):
    """vilmodel.py:360-372."""

    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.activation = nn.Tanh()

    def forward(self, hidden_states):
        return _lin(hidden_states[:, 0], self.dense, "tanh")


class BertOutAttention(nn.Module):
    """vilmodel.py:455-506: attention of `hidden_states` (queries) over `context` (keys/values)."""

    def __init__(self, config, ctx_dim=None):
        super().__init__()
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = int(config.hidden_size / config.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        ctx_dim = config.hidden_size if ctx_dim is None else ctx_dim
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(ctx_dim, self.all_head_size)
        self.value = nn.Linear(ctx_dim, self.all_head_size)
        self.dropout = nn.Dropout(config.attention_probs_dropout_prob)

    def forward(self, hidden_states, context, attention_mask=None):
        nq = _needs_grad(hidden_states, self.query.weight)
        nkv = _needs_grad(context, self.key.weight, self.value.weight)
        # bf16 Q/K/V for the bf16 attention core in configs[4]'s bf16 mode (no-grad only)
        dt = None if (nq or nkv) else _attn_dtype(hidden_states, self.all_head_size, context)
        q = _lin(hidden_states, self.query) if nq else ops.linear(hidden_states, self.query.weight, self.query.bias,
                                                                   out_dtype=dt)
        if nkv:
            k, v = _lin(context, self.key), _lin(context, self.value)
        else:
            W, b = _fused_weights(self, (self.key, self.value))
            kv = ops.linear(context, W, b, out_dtype=dt)
            Hs = self.all_head_size
            k, v = kv[..., :Hs], kv[..., Hs:]
        return DF.mha(q, k, v, _addmask(attention_mask, q.shape[0]), self.num_attention_heads,
                      1.0 / math.sqrt(self.attention_head_size), self.dropout.p, self.training)


class BertXAttention(nn.Module):
    """vilmodel.py:443-452."""

    def __init__(self, config, ctx_dim=None):
        super().__init__()
        self.att = BertOutAttention(config, ctx_dim=ctx_dim)
        self.output = BertSelfOutput(config)

    def forward(self, input_tensor, ctx_tensor, ctx_att_mask=None):
        return self.output(self.att(input_tensor, ctx_tensor, ctx_att_mask), input_tensor)


_TWO_STREAMS = os.environ.get("DASA_LXRT_STREAMS", "1") != "0"
_SIDE = {}


def _side_stream(device):
    st = _SIDE.get(device.index)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _SIDE[device.index] = st
    return st


class LXRTXLayer(nn.Module):
    """vilmodel.py:1014-1064: cross attention (ONE shared visual_attention for both directions),
    then self attention and FFN on each stream."""

    def __init__(self, config):
        super().__init__()
        self.lang_self_att = BertAttention(config)
        self.lang_inter = BertIntermediate(config)
        self.lang_output = BertOutput(config)
        self.visn_self_att = BertAttention(config)
        self.visn_inter = BertIntermediate(config)
        self.visn_output = BertOutput(config)
        self.visual_attention = BertXAttention(config)

    def cross_att(self, lang_input, lang_attention_mask, visn_input, visn_attention_mask):
        lang_att = self.visual_attention(lang_input, visn_input, ctx_att_mask=visn_attention_mask)
        visn_att = self.visual_attention(visn_input, lang_input, ctx_att_mask=lang_attention_mask)
        return lang_att, visn_att

    def self_att(self, lang_input, lang_attention_mask, visn_input, visn_attention_mask):
        return self.lang_self_att(lang_input, lang_attention_mask), self.visn_self_att(visn_input, visn_attention_mask)

    def output_fc(self, lang_input, visn_input):
        lang = self.lang_output(self.lang_inter(lang_input), lang_input)
        visn = self.visn_output(self.visn_inter(visn_input), visn_input)
        return lang, visn

    def forward(self, lang_feats, lang_attention_mask, visn_feats, visn_attention_mask, want_visn=True):
        if not want_visn:
            # the caller drops this layer's vision output (the last layer when ctx_v is off: DicEncoder's
            # vision_outputs are unused, agent_dg.py:807): its vision branch has no consumer, so only the
            # language branch runs — the language output is the same either way
            la = self.visual_attention(lang_feats, visn_feats, ctx_att_mask=visn_attention_mask)
            la = self.lang_self_att(la, lang_attention_mask)[0]
            return self.lang_output(self.lang_inter(la), la), None
        if torch.is_grad_enabled() or not _TWO_STREAMS:
            la, va = self.cross_att(lang_feats, lang_attention_mask, visn_feats, visn_attention_mask)
            la, va = self.self_att(la, lang_attention_mask, va, visn_attention_mask)
            return self.output_fc(la[0], va[0])
        # No autograd (the detached train config and eval): after the cross attention reads both
        # inputs, the language and vision streams are independent, so the vision branch (36 rows per
        # sample) runs on a second HIP stream beside the language branch (80 rows): the two streams'
        # GEMM/attention grids share the CUs instead of each leaving part of the chip idle.
        main = torch.cuda.current_stream()
        side = _side_stream(lang_feats.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            va = self.visual_attention(visn_feats, lang_feats, ctx_att_mask=lang_attention_mask)
            va = self.visn_self_att(va, visn_attention_mask)[0]
            visn = self.visn_output(self.visn_inter(va), va)
        la = self.visual_attention(lang_feats, visn_feats, ctx_att_mask=visn_attention_mask)
        la = self.lang_self_att(la, lang_attention_mask)[0]
        lang = self.lang_output(self.lang_inter(la), la)
        main.wait_stream(side)
        if not torch.cuda.is_current_stream_capturing():
            visn.record_stream(main)
        return lang, visn


class VisionEncoder(nn.Module):
    """vilmodel.py:1067-1095: dropout(LayerNorm(visn_fc(f)))."""

    def __init__(self, vision_size, config):
        super().__init__()
        self.visn_fc = nn.Linear(vision_size, config.hidden_size)
        self.visn_layer_norm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, visn_input):
        x = _lin(visn_input, self.visn_fc)
        x = DF.layer_norm(x, self.visn_layer_norm.weight, self.visn_layer_norm.bias, self.visn_layer_norm.eps)
        return DF.dropout(x, self.dropout.p, self.training)


class DicModel(nn.Module):
    """vilmodel.py:1245-1423. `text_embeds` (extra, optional) short-circuits the language stack with a
    cached output — exact whenever the stack is not being trained, since it does not see the image."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embeddings = BertEmbeddings(config)
        self.pooler = BertPooler(config)
        self.img_dim = config.img_feature_dim
        self.img_feature_type = config.img_feature_type
        self.vl_layers = config.vl_layers
        self.la_layers = config.la_layers
        self.update_lang_bert = config.update_lang_bert
        self.update_add_layer = config.update_add_layer
        self.lalayer = nn.ModuleList([BertLayer(config) for _ in range(self.la_layers)])
        self.addlayer = nn.ModuleList([LXRTXLayer(config) for _ in range(self.vl_layers)])
        self.vision_encoder = VisionEncoder(self.config.img_feature_dim, self.config)
        self._graphs = None     # captured forward-only VL stacks (dasa_amd/graph.py)
        self._tgraphs = None    # captured TRAINING VL stacks with autograd (finetune: --d_update_add_layer)
        self._dummy = None      # a grad-requiring leaf that links such a region into the caller's graph
        if args.d_v_layers > 0:
            self.vlayer = nn.ModuleList([BertLayer(config) for _ in range(args.d_v_layers)])
        self.init_weights()

    def init_weights(self):
        std = getattr(self.config, "initializer_range", 0.02)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                m.weight.data.normal_(0.0, std)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.data.fill_(1.0)
                m.bias.data.zero_()

    def _vl_stack(self, text_embeds, ext, img_feats, want_visn=True):
        """VisionEncoder + the vl LXRT layers (vilmodel.py:1383-1406). want_visn=False: the last
        layer's vision branch is skipped and None returned for the vision output."""
        B, V = img_feats.shape[0], img_feats.shape[1]
        img_mask = torch.zeros(B, 1, 1, V, dtype=torch.float32, device=img_feats.device)
        lang = text_embeds
        visn = self.vision_encoder(img_feats)
        if args.d_v_layers > 0:
            for layer in self.vlayer:
                visn = layer(visn, img_mask)[0]
        last = len(self.addlayer) - 1
        for i, layer in enumerate(self.addlayer):
            lang, visn = layer(lang, ext, visn, img_mask, want_visn=want_visn or i < last)
        return lang, visn

    def _train_region_ok(self, text_embeds, img_feats):
        """The finetune configuration's VisionEncoder + LXRT stack (trained: --d_update_add_layer,
        vilmodel.py:1408-1410) replays as a captured region with autograd (graph.AutogradGraphs) — forward
        and backward one graph launch each instead of ~60 / ~100 host-issued launches per decision step,
        which bound the B = 2 finetune iteration — unless the profiler brackets every
        launch, an enclosing region is being captured, a module is hooked, or DASA_TRAIN_GRAPH=0."""
        mods = [self.vision_encoder, self.addlayer] + ([self.vlayer] if args.d_v_layers > 0 else [])
        # (the region detaches its inputs: only when neither the language stack nor the panorama trains)
        return (graph.ENABLED and img_feats.is_cuda and os.environ.get("DASA_TRAIN_GRAPH", "1") != "0"
                and not text_embeds.requires_grad and not img_feats.requires_grad
                and os.environ.get("DASA_TRAIN_GRAPH_VL", "1") != "0" and not graph.capturing()
                and not ops.prof.active()
                and all(not m._forward_hooks and not m._forward_pre_hooks and "forward" not in m.__dict__
                        for mm in mods for m in mm.modules())
                and (self._tgraphs is None or len(self._tgraphs.slots) < 1024))

    def _vl_train_region(self, text_embeds, ext, img_feats, want_visn):
        """_vl_stack as one captured training region (one slot per use within an iteration: the caller calls
        train_graphs_new_iteration() once every replayed region has had its backward). The language input is
        padded to --maxInput tokens (rounded up to 16) with the padding masked (-10000: zero attention weight),
        so one slot serves every batch; padded rows are computed and cut off. A zero-size leaf that requires
        grad links the region into the caller's graph (its other inputs are detached), so the region's
        parameters get their gradients when the caller's backward reaches it."""
        if self._tgraphs is None:
            mods = [self.vision_encoder, self.addlayer] + ([self.vlayer] if args.d_v_layers > 0 else [])
            self._tgraphs = graph.AutogradGraphs(mods, flat_key=True)
        dev = img_feats.device
        if self._dummy is None or self._dummy.device != dev:
            self._dummy = torch.zeros(0, device=dev, requires_grad=True)
        B, L, Hd = text_embeds.shape
        Lp = -(-max(L, args.maxInput) // 16) * 16

        def fn(t, e, f, _link):
            lang, visn = self._vl_stack(t, e, f, want_visn)
            return (lang, visn) if visn is not None else (lang,)
        key = ("vl", B, Lp, Hd, tuple(img_feats.shape[1:]), bool(want_visn), self.training)
        outs = self._tgraphs.run(key, fn, (text_embeds.detach(), ext, img_feats.detach(), self._dummy),
                                 pads={0: ((B, Lp, Hd), 0.0), 1: ((B, 1, 1, Lp), -10000.0)})
        lang = outs[0][:, :L]
        return lang, (outs[1] if len(outs) > 1 else None)

    def train_graphs_new_iteration(self):
        if self._tgraphs is not None:
            self._tgraphs.new_iteration()

    def language(self, input_ids, ext_mask):
        """Embeddings + the la_layers language BertLayers (vilmodel.py:1366-1372)."""
        x = self.embeddings(input_ids)
        for layer in self.lalayer:
            x = layer(x, ext_mask)[0]
        return x

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, position_ids=None, head_mask=None,
                img_feats=None, text_embeds=None, want_visn=True, want_pooled=True):
        """want_visn / want_pooled (extras, default on = the reference's outputs): False returns None for the
        vision output / pooled output and skips the work that only they need (the last LXRT layer's
        vision branch; the pooler). The language output is unchanged."""
        if head_mask is not None or position_ids is not None:
            raise NotImplementedError("head_mask / position_ids")
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        ext = extended_mask(attention_mask)
        if text_embeds is None:
            with torch.set_grad_enabled(torch.is_grad_enabled() and self.update_lang_bert):
                text_embeds = self.language(input_ids, ext)
        if not self.update_lang_bert:
            text_embeds = text_embeds.detach()
        visn_output = None
        if img_feats is not None:
            vl_grad = torch.is_grad_enabled() and self.update_add_layer
            if not vl_grad and graph.ENABLED and img_feats.is_cuda:
                # forward-only: one hipGraph replay per step (dasa_amd/graph.py)
                if self._graphs is None:
                    mods = [self.vision_encoder, self.addlayer] + ([self.vlayer] if args.d_v_layers > 0 else [])
                    self._graphs = graph.StepGraphs(mods)
                key = (tuple(text_embeds.shape), tuple(ext.shape), tuple(img_feats.shape), img_feats.stride(),
                       self.training, bool(want_visn))
                lang, visn = self._graphs.run(key, lambda t, e, f: self._vl_stack(t, e, f, want_visn),
                                              (text_embeds, ext, img_feats))
            elif vl_grad and self._train_region_ok(text_embeds, img_feats):
                lang, visn = self._vl_train_region(text_embeds, ext, img_feats, want_visn)
            else:
                with torch.set_grad_enabled(vl_grad):
                    lang, visn = self._vl_stack(text_embeds, ext, img_feats, want_visn)
            if not self.update_add_layer:
                lang = lang.detach()
                visn = visn.detach() if visn is not None else None
            sequence_output = lang
        else:
            sequence_output = text_embeds
        pooled_output = self.pooler(sequence_output) if want_pooled else None
        return sequence_output, pooled_output, visn_output if img_feats is None else visn
