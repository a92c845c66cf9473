"""Parameter schemas (state_dict key -> shape) of the reference modules on the hot path, restated from
their constructors so the oracle can build weight dicts without module objects. Pinned against the
schemas recorded from the reference itself in tests/golden/ops.npz (schema/*).

TEST INFRASTRUCTURE ONLY (see oracle/policy.py header).
"""
H, I, V, POS, TYPES = 768, 3072, 30522, 512, 2


def _lin(d, pre, out_f, in_f, bias=True):
    d[pre + ".weight"] = (out_f, in_f)
    if bias:
        d[pre + ".bias"] = (out_f,)


def _ln(d, pre, n=H):
    d[pre + ".weight"] = (n,)
    d[pre + ".bias"] = (n,)


def _bert_attention(d, pre):
    for n in ("query", "key", "value"):
        _lin(d, f"{pre}.self.{n}", H, H)
    _lin(d, pre + ".output.dense", H, H)
    _ln(d, pre + ".output.LayerNorm")


def encoder_schema(vl_layers=3, la_layers=9, img_dim=2176, enc_hidden=1024, dec_hidden=1024):
    """DicEncoder (r2rmodel.py:2204-2252) + DicModel (vilmodel.py:1275-1311)."""
    d = {}
    d["bert.embeddings.word_embeddings.weight"] = (V, H)
    d["bert.embeddings.position_embeddings.weight"] = (POS, H)
    d["bert.embeddings.token_type_embeddings.weight"] = (TYPES, H)
    _ln(d, "bert.embeddings.LayerNorm")
    _lin(d, "bert.pooler.dense", H, H)
    for i in range(la_layers):
        p = f"bert.lalayer.{i}"
        _bert_attention(d, p + ".attention")
        _lin(d, p + ".intermediate.dense", I, H)
        _lin(d, p + ".output.dense", H, I)
        _ln(d, p + ".output.LayerNorm")
    for i in range(vl_layers):
        p = f"bert.addlayer.{i}"
        for s in ("lang", "visn"):
            _bert_attention(d, f"{p}.{s}_self_att")
            _lin(d, f"{p}.{s}_inter.dense", I, H)
            _lin(d, f"{p}.{s}_output.dense", H, I)
            _ln(d, f"{p}.{s}_output.LayerNorm")
        for n in ("query", "key", "value"):
            _lin(d, f"{p}.visual_attention.att.{n}", H, H)
        _lin(d, f"{p}.visual_attention.output.dense", H, H)
        _ln(d, f"{p}.visual_attention.output.LayerNorm")
    _lin(d, "bert.vision_encoder.visn_fc", H, img_dim)
    _ln(d, "bert.vision_encoder.visn_layer_norm")
    for sfx in ("", "_reverse"):
        d["lstm.weight_ih_l0" + sfx] = (4 * enc_hidden, H)
        d["lstm.weight_hh_l0" + sfx] = (4 * enc_hidden, enc_hidden)
        d["lstm.bias_ih_l0" + sfx] = (4 * enc_hidden,)
        d["lstm.bias_hh_l0" + sfx] = (4 * enc_hidden,)
    for n in ("encoder2decoder_ht", "encoder2decoder_ct", "encoder_lstm2decoder_ht", "encoder_lstm2decoder_ct"):
        _lin(d, n, dec_hidden, 2 * enc_hidden)
    return d


def decoder_schema(aemb=64, hidden=1024, feat=2176, angle=128, kernel=5):
    """BAttnDecoderLSTM (model.py:425-466) with use_shift, no pred_back / pred_pm."""
    d = {}
    _lin(d, "embedding.0", aemb, angle)
    d["lstm.weight_ih"] = (4 * hidden, aemb + feat)
    d["lstm.weight_hh"] = (4 * hidden, hidden)
    d["lstm.bias_ih"] = (4 * hidden,)
    d["lstm.bias_hh"] = (4 * hidden,)
    _lin(d, "feat_att_layer.linear_in", feat, hidden, bias=False)
    _lin(d, "feat_att_layer.linear_shift", kernel, hidden)
    _lin(d, "feat_att_layer.linear_out", hidden, hidden + feat, bias=False)
    _lin(d, "attention_layer.linear_in", 2 * hidden, hidden, bias=False)
    _lin(d, "attention_layer.linear_out", hidden, 3 * hidden, bias=False)
    _lin(d, "candidate_att_layer.linear_in", feat, hidden, bias=False)
    _lin(d, "candidate_att_layer.linear_out", hidden, hidden + feat, bias=False)
    return d


def critic_schema(dim=1024):
    """Critic (model.py:970-979)."""
    d = {}
    _lin(d, "state2value.0", dim, dim)
    _lin(d, "state2value.3", 1, dim)
    return d


def ada_schema(channel=2048):
    """DGAdaChannel with ab_type 'a' (agent_dg.py:1516-1522)."""
    d = {}
    _lin(d, "a_fc", channel, channel)
    return d
