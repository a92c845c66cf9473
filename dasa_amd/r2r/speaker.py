"""Speaker of r2r_src/speaker.py (the back-translation model of the auglistener loop, SURVEY.md §8(f)
rank 3) on the MI355X kernels: SpeakerEncoder / SpeakerDecoder (dasa_amd.r2r.model) run the persistent
bi-LSTM, SoftDot attention, LSTM-cell and GEMM kernels of the policy path.

`infer_batch` follows speaker.py:265-350 (walk the env along the teacher path collecting panorama and
action features, encode, decode word by word, one host sync per word as the reference's `.cpu()`).
Deliberate differences, none observable by the agent: it runs under torch.no_grad() (the reference
builds an autograd graph it never uses); `np.bool` (gone from numpy 2) is `bool`; the word copy is an
explicit host copy (the reference's CPU-aliasing hazard); with an env that offers
`device_input_feat` the features are gathered on the device. Training the speaker (train /
teacher_forcing / beam search) is not part of the policy path and is not provided.
"""
import os

import numpy as np
import torch

from .. import ops
from . import model
from . import utils
from .param import args


class Speaker:
    env_actions = {
        "left": (0, -1, 0), "right": (0, 1, 0), "up": (0, 0, 1), "down": (0, 0, -1),
        "forward": (1, 0, 0), "<end>": (0, 0, 0), "<start>": (0, 0, 0), "<ignore>": (0, 0, 0),
    }

    def __init__(self, env, listener, tok):
        self.env = env
        self.feature_size = env.feature_size if env is not None else 2048
        self.tok = tok
        self.tok.finalize()
        self.listener = listener
        dev = listener.device if listener is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.encoder = model.SpeakerEncoder(self.feature_size + args.angle_feat_size, args.rnn_dim, args.dropout,
                                            bidirectional=args.bidir).to(dev)
        self.decoder = model.SpeakerDecoder(self.tok.vocab_size(), args.wemb, self.tok.word_to_index["<PAD>"],
                                            args.rnn_dim, args.dropout).to(dev)
        self.encoder_optimizer = args.optimizer(self.encoder.parameters(), lr=args.lr)
        self.decoder_optimizer = args.optimizer(self.decoder.parameters(), lr=args.lr)

    # ------------------------------------------------------------------ trajectory features
    def _teacher_action(self, obs, ended):
        """speaker.py:133-152 (host array; the reference copies it up and back down)."""
        a = np.zeros(len(obs), dtype=np.int64)
        for i, ob in enumerate(obs):
            if ended[i]:
                a[i] = args.ignoreid
            else:
                for k, candidate in enumerate(ob["candidate"]):
                    if candidate["viewpointId"] == ob["teacher"]:
                        a[i] = k
                        break
                else:
                    assert ob["teacher"] == ob["viewpoint"]
                    a[i] = len(ob["candidate"])
        return a

    def _step_features(self, obs, actions):
        """The panorama [B, 36, F+A] (listener._feature_variable) and the taken candidate's feature
        [B, F+A] (zero for stop / ended, speaker.py:154-162) of one step."""
        B = len(obs)
        if hasattr(self.env, "device_input_feat"):
            _, f_t, _, cf, _, _ = self.env.device_input_feat(obs, self.device)
            idx = torch.as_tensor(np.where(actions < 0, 0, actions), device=self.device)
            can = cf[torch.arange(B, device=self.device), idx]
            keep = torch.as_tensor((actions >= 0).astype(np.float32), device=self.device).unsqueeze(1)
            return f_t, can * keep
        f_t = self.listener._feature_variable(obs)
        can = np.zeros((B, self.feature_size + args.angle_feat_size), np.float32)
        for i, (ob, act) in enumerate(zip(obs, actions)):
            if act != -1:
                can[i] = ob["candidate"][act]["feature"]
        return f_t, torch.from_numpy(can).to(self.device)

    def make_equiv_action(self, a_t, perm_obs, perm_idx=None, traj=None):
        """speaker.py:98-131 (the listener's implementation: same action sequence)."""
        if self.listener is not None:
            return self.listener.make_equiv_action(a_t, perm_obs, perm_idx, traj)
        raise RuntimeError("Speaker.make_equiv_action needs the listener's simulator binding")

    def from_shortest_path(self, viewpoints=None, get_first_feat=False):
        """speaker.py:164-199: features along the teacher path until every agent stops."""
        obs = self.env._get_obs()
        B = len(obs)
        ended = np.array([False] * B)
        length = np.zeros(B, np.int64)
        img_feats, can_feats = [], []
        first_feat = None
        if get_first_feat:
            ff = np.zeros((B, self.feature_size + args.angle_feat_size), np.float32)
            for i, ob in enumerate(obs):
                ff[i, -args.angle_feat_size:] = utils.angle_feature(ob["heading"], ob["elevation"])
            first_feat = torch.from_numpy(ff).to(self.device)
        while not ended.all():
            if viewpoints is not None:
                for i, ob in enumerate(obs):
                    viewpoints[i].append(ob["viewpoint"])
            teacher_action = self._teacher_action(obs, ended)
            for i, act in enumerate(teacher_action):
                if act < 0 or act == len(obs[i]["candidate"]):
                    teacher_action[i] = -1
            f_t, can = self._step_features(obs, teacher_action)
            img_feats.append(f_t)
            can_feats.append(can)
            self.make_equiv_action(teacher_action, obs)
            length += (1 - ended)
            ended[:] = np.logical_or(ended, teacher_action == -1)
            obs = self.env._get_obs()
        img_feats = torch.stack(img_feats, 1).contiguous()
        can_feats = torch.stack(can_feats, 1).contiguous()
        if get_first_feat:
            return (img_feats, can_feats, first_feat), length
        return (img_feats, can_feats), length

    # ------------------------------------------------------------------ decoding
    def infer_batch(self, sampling=False, train=False, featdropmask=None):
        """speaker.py:265-350. Returns insts np [B, len] (argmax, or Categorical samples with
        sampling=True; the train-mode log-prob / hidden / entropy returns are not provided)."""
        if train and sampling:
            raise NotImplementedError("speaker training (sampling with gradients) is outside the policy path")
        for m in (self.encoder, self.decoder):
            m.train() if train else m.eval()
        with torch.no_grad():
            obs = self.env._get_obs()
            B = len(obs)
            viewpoints_list = [list() for _ in range(B)]
            (img_feats, can_feats), lengths = self.from_shortest_path(viewpoints=viewpoints_list)
            if featdropmask is not None:      # the shared env-drop mask on the RGB columns (speaker.py:293-295)
                A = args.angle_feat_size
                img_feats, can_feats = img_feats.clone(), can_feats.clone()
                ops.colscale(img_feats[..., :-A], featdropmask, img_feats[..., :-A])
                ops.colscale(can_feats[..., :-A], featdropmask, can_feats[..., :-A])
            ctx = self.encoder(can_feats, img_feats, lengths, already_dropfeat=(featdropmask is not None))
            ctx_mask = utils.length2mask(lengths, device=self.device)
            w2i = self.tok.word_to_index
            words = []
            h_t = torch.zeros(1, B, args.rnn_dim, device=self.device)
            c_t = torch.zeros(1, B, args.rnn_dim, device=self.device)
            ended = np.zeros(B, bool)
            word = torch.full((B, 1), w2i["<BOS>"], dtype=torch.int64, device=self.device)
            for _ in range(args.maxDecode):
                logits, h_t, c_t = self.decoder(word, ctx, ctx_mask, h_t, c_t)
                logits = logits.view(B, -1)
                logits[:, w2i["<UNK>"]] = -float("inf")            # no <UNK> in inference
                if sampling:
                    word = torch.distributions.Categorical(logits=logits).sample()
                else:
                    word = logits.argmax(1)
                cpu_word = word.cpu().numpy().copy()
                cpu_word[ended] = w2i["<PAD>"]
                words.append(cpu_word)
                word = word.view(-1, 1)
                ended = np.logical_or(ended, cpu_word == w2i["<EOS>"])
                if ended.all():
                    break
        return np.stack(words, 1)

    # ------------------------------------------------------------------ checkpoints
    def save(self, epoch, path):
        """speaker.py:352-366 schema: {'encoder'|'decoder': {'epoch', 'state_dict', 'optimizer'}}."""
        the_dir, _ = os.path.split(path)
        if the_dir:
            os.makedirs(the_dir, exist_ok=True)
        states = {}
        for name, m, opt in (("encoder", self.encoder, self.encoder_optimizer),
                             ("decoder", self.decoder, self.decoder_optimizer)):
            states[name] = {"epoch": epoch + 1, "state_dict": m.state_dict(), "optimizer": opt.state_dict()}
        torch.save(states, path)

    def load(self, path):
        """speaker.py:368-388 (safe loader: weights_only=True)."""
        print("Load the speaker's state dict from %s" % path)
        states = torch.load(path, map_location=self.device, weights_only=True)
        for name, m, opt in (("encoder", self.encoder, self.encoder_optimizer),
                             ("decoder", self.decoder, self.decoder_optimizer)):
            state = m.state_dict()
            state.update(states[name]["state_dict"])
            m.load_state_dict(state)
            if args.loadOptim:
                opt.load_state_dict(states[name]["optimizer"])
        return states["encoder"]["epoch"] - 1
