"""Speaker back-translation (dasa_amd/r2r/speaker.py on the HIP kernels) against the reference's
Speaker.infer_batch (speaker.py:265-350) run in the survey container (tests/golden/speaker.npz,
oracle/golden/make_golden.py speaker): encoder context, every decoding step's vocabulary logits and
LSTM state within 1e-4, identical argmax instructions. CPU: the module schema (state_dict keys and
shapes, the reference checkpoint layout) and the word Tokenizer."""
import json
import os

import numpy as np
import pytest
import torch

from tests import golden_inputs as GI
from tests.helpers import GOLDEN, close, golden


def _tok():
    from dasa_amd.r2r import utils
    return utils.Tokenizer(vocab=utils.read_vocab(os.path.join(GOLDEN, "train_vocab.txt")), encoding_length=80)


def test_tokenizer_matches_reference_vocab():
    G = golden("speaker")
    tok = _tok()
    assert tok.vocab_size() == int(G["spk/vocab_size"])
    assert tok.word_to_index["<BOS>"] == tok.vocab_size() - 1
    enc = tok.encode_sentence("Walk past the table, then stop.")
    assert enc[0] == tok.word_to_index["<BOS>"] and enc.shape == (80,)
    assert tok.decode_sentence(tok.shrink(list(enc))) == "walk past the table , then stop ."


def test_speaker_module_schema():
    G = golden("speaker")
    from dasa_amd.r2r import param
    param.readme_train([])
    from dasa_amd.r2r import model
    a = param.args
    enc = model.SpeakerEncoder(2048 + a.angle_feat_size, a.rnn_dim, a.dropout, bidirectional=a.bidir)
    dec = model.SpeakerDecoder(int(G["spk/vocab_size"]), a.wemb, 0, a.rnn_dim, a.dropout)
    for m, key in ((enc, "spk/schema_encoder"), (dec, "spk/schema_decoder")):
        want = json.loads(str(G[key]))
        assert {k: list(v.shape) for k, v in m.state_dict().items()} == want


@pytest.mark.gpu
def test_speaker_infer_batch_vs_reference(dev):
    G = golden("speaker")
    cfg = GI.SPEAKER
    from dasa_amd.r2r import param
    param.readme_train(["--maxDecode", str(cfg["max_decode"]), "--batchSize", str(cfg["batch"])])
    try:
        from dasa_amd.r2r import agent_dg, speaker
        from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
        import contextlib
        import io
        world = SynthWorld(cfg["viewpoints"], 0, cfg["graph_seed"])
        env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80, variable_len=True)
        with contextlib.redirect_stdout(io.StringIO()):
            listener = agent_dg.Seq2SeqAgent(env, "", None, 5, "Dic")
        spk = speaker.Speaker(env, listener, _tok())
        init_params(spk.encoder, cfg["seed_enc"])
        init_params(spk.decoder, cfg["seed_dec"])
        rec = {"ctx": None, "logits": [], "h": []}
        enc_fwd, dec_fwd = spk.encoder.forward, spk.decoder.forward

        def enc_wrap(*a, **k):
            r = enc_fwd(*a, **k)
            rec["ctx"] = r.detach().cpu().clone()
            return r

        def dec_wrap(*a, **k):
            r = dec_fwd(*a, **k)
            rec["logits"].append(r[0].detach().cpu().clone())
            rec["h"].append(r[1].detach().cpu().clone())
            return r
        spk.encoder.forward, spk.decoder.forward = enc_wrap, dec_wrap
        env.reset()
        insts = spk.infer_batch()
        close(rec["ctx"], G["spk/ctx"], 1e-4, "speaker ctx")
        assert len(rec["logits"]) == int(G["spk/steps"])
        for t, (lg, h) in enumerate(zip(rec["logits"], rec["h"])):
            close(lg, G[f"spk/logit/{t}"], 1e-4, f"speaker logit {t}")
            close(h, G[f"spk/h/{t}"], 1e-4, f"speaker h {t}")
        assert np.array_equal(np.asarray(insts), G["spk/insts"])
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])


@pytest.mark.gpu
def test_speaker_featdropmask_and_sampling(dev):
    """The shared env-drop mask path (speaker.py:293-295, ops.colscale on the RGB columns): an all-ones
    mask reproduces the unmasked instructions and a zero mask changes the context; sampled decoding
    yields vocabulary ids with <PAD> after each row's <EOS>."""
    cfg = GI.SPEAKER
    from dasa_amd.r2r import param
    param.readme_train(["--maxDecode", str(cfg["max_decode"]), "--batchSize", str(cfg["batch"])])
    try:
        from dasa_amd.r2r import agent_dg, speaker
        from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
        import contextlib
        import io
        world = SynthWorld(cfg["viewpoints"], 0, cfg["graph_seed"])

        def make():
            env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80,
                                variable_len=True)
            with contextlib.redirect_stdout(io.StringIO()):
                listener = agent_dg.Seq2SeqAgent(env, "", None, 5, "Dic")
            spk = speaker.Speaker(env, listener, _tok())
            init_params(spk.encoder, cfg["seed_enc"])
            init_params(spk.decoder, cfg["seed_dec"])
            env.reset()
            return spk
        base = make().infer_batch()
        ones = make().infer_batch(featdropmask=torch.ones(2048, device=dev))
        assert np.array_equal(base, ones)
        ctxs = []
        for m in (torch.ones(2048, device=dev), torch.zeros(2048, device=dev)):
            spk = make()
            fwd = spk.encoder.forward
            spk.encoder.forward = lambda *a, _f=fwd, **k: (ctxs.append(_f(*a, **k)), ctxs[-1])[1]
            spk.infer_batch(featdropmask=m)
        assert not torch.allclose(ctxs[0], ctxs[1])
        spk = make()
        w2i = spk.tok.word_to_index
        insts = spk.infer_batch(sampling=True)
        assert insts.dtype.kind in "iu" and insts.min() >= 0 and insts.max() < spk.tok.vocab_size()
        assert not (insts == w2i["<UNK>"]).any()
        for row in insts:
            eos = np.nonzero(row == w2i["<EOS>"])[0]
            if len(eos):
                assert (row[eos[0] + 1:] == w2i["<PAD>"]).all()
    finally:
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
