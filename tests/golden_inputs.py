"""Seeded inputs shared by oracle/golden/make_golden.py (which ran the reference on them) and the
tests (which re-create them). Fixtures store only outputs; inputs and weights regenerate from seeds.
"""
import numpy as np
import torch

# weight seeds per reference module (agent_dg.py:161-200)
SEED_ENC, SEED_DEC, SEED_CRITIC, SEED_ADA = 1, 2, 3, 4
CFG1 = dict(batch=2, vl_layers=1, la_layers=9, max_action=5, instr_len=80, kernel=5)
# cfg4 (finetune, --d_update_add_layer True): the LXRT stack and VisionEncoder are trained; per-rank B=2.
# Two cross layers so the backward crosses a layer boundary; fewer steps keep the CPU reference short.
CFG4 = dict(batch=2, vl_layers=2, la_layers=9, max_action=4, instr_len=80, kernel=5)
# cfg2 (the bench configuration: B=20, vl=3): a full 35-step argmax eval rollout, and one training
# iteration (teacher + argmax-'sampled' rollout, backward) at maxAction 5 with dropout 0.
CFG2 = dict(batch=20, vl_layers=3, la_layers=9, max_action=35, train_max_action=5, instr_len=80, kernel=5,
            viewpoints=32, graph_seed=5, eval_seed=21, train_seed=22)
# cfg5 numerics at a CPU-affordable batch: vl=6, B=4, a 6-step teacher-forced eval rollout (fp32
# golden; the GPU compares its fp32 and its bf16-operand rollouts against it).
CFG5 = dict(batch=4, vl_layers=6, la_layers=9, max_action=6, instr_len=80, kernel=5, viewpoints=16, graph_seed=3,
            seed=23)
# configs[4] at its own batch (r05): B=256, vl=6, a 2-step teacher-forced eval rollout (fp32 golden), so
# the B >= 128 kernel forms — whole-row attention incl. the N = 80 SoftDot, the bf16x6 plans at 256-row
# batches, the bi-LSTM's 192-row tiles — are compared with the reference itself, not with the product.
CFG5_B256 = dict(batch=256, vl_layers=6, la_layers=9, max_action=2, instr_len=80, kernel=5, viewpoints=64,
                 graph_seed=3, seed=31)


def _u(rng, *shape):
    return torch.from_numpy(rng.random(shape, dtype=np.float32))


def _n(rng, *shape, scale=1.0):
    return torch.from_numpy((rng.standard_normal(shape, dtype=np.float32) * scale).astype(np.float32))


def ada_inputs():
    rng = np.random.default_rng(100)
    return _u(rng, 2, 10, 2048), _u(rng, 2, 10, 2048), _n(rng, 2, 10, 2048)


def adain_inputs():
    rng = np.random.default_rng(101)
    return _u(rng, 2, 10, 2048), _u(rng, 2, 10, 2048)


def adain_grad_weights():
    return _n(np.random.default_rng(102), 2, 10, 2048)


def shift_inputs(K):
    rng = np.random.default_rng(102 + K)
    return _n(rng, 3, 1024, scale=0.5), _u(rng, 3, 36, 2176), _n(rng, 3, 2176)


def softdot_inputs():
    rng = np.random.default_rng(110)
    h = _n(rng, 3, 1024, scale=0.5)
    ctx = _n(rng, 3, 12, 2048)
    mask = torch.zeros(3, 12, dtype=torch.bool)
    mask[1, 7:] = True
    mask[2, 3:] = True
    cand = _u(rng, 3, 6, 2176)
    return h, ctx, mask, cand, _n(rng, 3, 1024), _n(rng, 3, 6)


def decoder_inputs():
    rng = np.random.default_rng(120)
    B = 3
    action = _n(rng, B, 128)
    feature = _u(rng, B, 36, 2176)
    cand = _u(rng, B, 6, 2176)
    h0 = _n(rng, B, 1024, scale=0.3)
    prev_h1 = torch.tanh(_n(rng, B, 1024))
    c0 = _n(rng, B, 1024, scale=0.3)
    ctx = _n(rng, B, 12, 2048, scale=0.2)
    mask = torch.zeros(B, 12, dtype=torch.bool)
    mask[2, 9:] = True
    return action, feature, cand, h0, prev_h1, c0, ctx, mask


def critic_inputs():
    rng = np.random.default_rng(130)
    return _n(rng, 4, 1024)


def lxrt_inputs():
    rng = np.random.default_rng(140)
    lang = _n(rng, 2, 12, 768)
    visn = _n(rng, 2, 36, 768)
    lang_mask = torch.zeros(2, 12)
    lang_mask[1, 8:] = -10000.0
    return lang, lang_mask, visn, torch.zeros(2, 36)


def encoder_inputs():
    """DicEncoder at B=3, L=12, lengths 12/9/5 (sorted descending like _sort_batch)."""
    rng = np.random.default_rng(150)
    B, L = 3, 12
    lengths = [12, 9, 5]
    seq = np.zeros((B, L), dtype=np.int64)
    for i, n in enumerate(lengths):
        seq[i, 0] = 101
        seq[i, 1:n - 1] = rng.integers(1000, 30000, size=n - 2)
        seq[i, n - 1] = 102
    seq = torch.from_numpy(seq)
    mask = seq == 0
    f = _u(rng, B, 36, 2176)
    return seq, mask, lengths, f


def io_tables():
    """Tiny real-format feature tables (utils.py:272-312 TSV, env.py:22-29 depth .npy pair)."""
    rng = np.random.default_rng(160)
    img = {f"scan{s}_vp{v:02d}": rng.random((36, 2048), dtype=np.float32) for s, v in (("A", 0), ("A", 1), ("B", 7))}
    keys = np.array([["scanA", "vp00"], ["scanB", "vp07"], ["scanC", "vp03"]])
    vals = rng.random((3, 36, 2048), dtype=np.float32)
    return img, keys, vals

# Speaker back-translation (speaker.py:265-350) at the auglistener batch: B=6 goal episodes (the teacher
# path ends), weights seeded, eval mode, argmax decoding, maxDecode 12.
SPEAKER = dict(batch=6, viewpoints=16, graph_seed=3, env_seed=41, max_decode=12, seed_enc=61, seed_dec=62)


# ---- forced actions for the sampled rollout (the fused policy head at rollout level) ---------------
# Categorical.sample is replaced, in the reference run, by a seeded table: at sampled step t row b takes
# candidate floor(u[t, b] * n_b), n_b = the row's valid candidates (the nonzero probabilities); the
# product passes the same actions to dasa_policy_head_fwd in mode FORCED (Seq2SeqAgent.force_action_fn).
FORCED_SEED = 31


def forced_table(steps, batch, seed=FORCED_SEED):
    return np.random.default_rng(seed).random((steps, batch))


def forced_actions(table, t, lens, no_stop=False):
    """Row b takes candidate floor(u[t, b] * n_b); with no_stop the draw is over the navigable
    candidates only (n_b - 1 of them; the stop entry is the last, agent_dg.py:305-306), so a
    'wander' episode runs every one of its maxAction steps."""
    lens = np.asarray(lens, np.int64)
    if no_stop:
        n = np.maximum(lens - 1, 1)
        return np.minimum((table[t] * n).astype(np.int64), n - 1)
    return np.minimum((table[t] * lens).astype(np.int64), lens - 1)


def reference_forced_sample(table, utils_mod, no_stop=False):
    """A Categorical.sample replacement for the reference run: the t-th call returns the table's step t,
    over the candidate counts the step passed to utils.length2mask (agent_dg.py:834, right before the
    draw; counting probs > 0 instead would miss candidates whose probability underflows). Returns
    (sample, install, uninstall): install() also wraps utils_mod.length2mask to record the counts."""
    state = {"t": 0, "lens": None}
    orig = utils_mod.length2mask

    def length2mask(length, size=None):
        state["lens"] = [int(x) for x in length]
        return orig(length, size) if size is not None else orig(length)

    def sample(self, *a, **k):
        out = torch.from_numpy(forced_actions(table, state["t"], state["lens"], no_stop))
        state["t"] += 1
        return out

    def install():
        utils_mod.length2mask = length2mask

    def uninstall():
        utils_mod.length2mask = orig
    return sample, install, uninstall


# ---- the aug half of the auglistener iteration (speaker + shared env-drop mask) -------------------
# accumulate_gradient('sample', speaker=...) at B=4, vl=3: the speaker back-translates each rollout's
# teacher path, the listener re-tokenises it, and both rollouts run with the shared env-drop noise
# (agent_dg.py:656-677, 731-736, 780-785, 946-952). Every dropout is p=0 except the env-drop mask,
# which is a fixed seeded mask (FixedEnvDrop) in both runs.
# The speaker's seeded weights are scaled by spk_scale: at the 0.02 init every row decodes the same word
# over and over; x10 gives row-dependent instructions (distinct listener token sequences per row).
CFG_AUG = dict(batch=4, vl_layers=3, la_layers=9, max_action=4, viewpoints=16, graph_seed=3, env_seed=43,
               max_decode=12, seed_enc=61, seed_dec=62, mask_seed=44, featdropout=0.4, spk_scale=10.0)


def scale_params(module, s):
    with torch.no_grad():
        for p in module.parameters():
            p.mul_(s)
    return module


def env_drop_mask(seed=CFG_AUG["mask_seed"], p=CFG_AUG["featdropout"], n=2048):
    keep = np.random.default_rng(seed).random(n) >= p
    return torch.from_numpy((keep / (1.0 - p)).astype(np.float32))


class FixedEnvDrop(torch.nn.Module):
    """decoder.drop_env replaced by a fixed mask: drop_env(ones(2048)) is the shared noise vector."""

    def __init__(self, mask):
        super().__init__()
        self.register_buffer("mask", mask.clone())

    def forward(self, x):
        return x * self.mask.to(x.device)


class WordHashBTokenizer:
    """The listener's tokenizer in the aug loop is utils.BTokenizer (utils.py:581-616, bert-base-uncased
    WordPiece, a name-based download unavailable offline). This stand-in keeps BTokenizer's contract —
    [CLS]=101 + one id per word + [SEP]=102, padded with pad_token_id 0 to encoding_length, an over-long
    encoding cut with [SEP] last — with word ids from a CRC of the word; both runs use it."""

    class _T:
        pad_token_id = 0
        sep_token_id = 102

    def __init__(self, encoding_length=80):
        self.tokenizer = self._T()
        self.encoding_length = encoding_length

    def encode_sentence(self, sentence, seps=None):
        import re
        import zlib
        words = [w for w in re.split(r"\s+", sentence.strip().lower()) if w]
        enc = [101] + [1000 + zlib.crc32(w.encode()) % 29000 for w in words] + [102]
        if len(enc) < self.encoding_length:
            enc += [0] * (self.encoding_length - len(enc))
        if len(enc) > self.encoding_length:
            enc[self.encoding_length - 1] = 102
        return np.array(enc[:self.encoding_length])


# ---- optim_step after a training iteration (clip 40 + RMSprop + LambdaLR, agent_dg.py:1389-1405) ---
CFG_OPTIM = dict(batch=2, vl_layers=1, la_layers=9, max_action=5, instr_len=80, iters=2, env_seed=8)

# ---- cfg4 at its README configuration (README.md:104-116: vl=3, B=2, maxAction 35 -> 6 steps here) --
CFG4R = dict(batch=2, vl_layers=3, la_layers=9, max_action=6, instr_len=80, env_seed=10)

# ---- the headline iteration at its real length (BASELINE configs[1], the bench workload) -------------
# accumulate_gradient('sample') at B=20, vl=3, maxAction 35 on 'wander' episodes (the teacher never
# stops: 35 teacher steps) with the sampled draws from a no-stop forced table (35 sampled steps), dropout
# 0: the timed path end to end — 8-step teacher chunks (the language pipe and the persistent bi-LSTM at
# 160 rows), the fused policy head in TEACHER and FORCED modes, the batched BPTT over all 70 encoder calls
# and the deferred weight gradients with K = T*B.
CFG2_FULL = dict(batch=20, vl_layers=3, la_layers=9, max_action=35, instr_len=80, viewpoints=32, graph_seed=5,
                 env_seed=24, forced_seed=33)

# ---- cfg4 at its README length (r05): the finetune iteration the bench's cfg4 leg runs (README.md:104-116:
# --d_update_add_layer True, vl 3, B 2, maxAction 35) on 'wander' episodes with no-stop forced draws, so
# 35 teacher + 35 sampled steps run: the 70-step bi-LSTM BPTT at B = 2 and the LXRT / MHA backward at full
# length, every gradient, every decoder call's logits; dropout 0.
CFG4_FULL = dict(batch=2, vl_layers=3, la_layers=9, max_action=35, instr_len=80, viewpoints=32, graph_seed=5,
                 env_seed=44, forced_seed=45)

# ---- --pretrain_model_name (agent_dg.py:165-188): a DicAddActionPreTrain checkpoint directory -------
# whose config.json says vl_layers=2 while the command line says d_vl_layers=3 (the checkpoint decides)
CFG_PRE = dict(batch=2, vl_layers_ckpt=2, la_layers=9, max_action=5, instr_len=80, env_seed=12, seed_bert=71)
