"""Seq2SeqAgent / DGAdaChannel of r2r_src/agent_dg.py on the MI355X kernels.

Same constructor, methods, attributes, `logs` keys and checkpoint schema as the reference
(agent_dg.py:102-1510), so r2r_src/train.py drives it unchanged. The per-step policy math runs in
libdasa_hip.so; the host loop keeps the reference's semantics (per-row env stepping, rewards, A2C).
Deliberate differences, none observable by train.py:
  * `.item()` logging syncs are deferred to the end of the rollout (same values, same order);
  * if the env offers `device_input_feat(perm_obs)` the panorama blocks are gathered on the device
    instead of numpy-assembled and copied (identical tensors);
  * eval rollouts compute the (input-independent, detached) 9-layer language stack once per batch;
  * data-parallel training: optim_step() all-reduces gradients over the default process group.
"""
import json
import math
import os
import random
import sys
from collections import defaultdict

import numpy as np
import torch
import torch.nn as nn

from .. import functional as DF
from .. import graph
from .. import ops
from .. import prof
from . import model
from . import utils
from .param import args
from .r2rmodel import DicEncoder

FEATURE_SIZE = 2048
FEATURE_ALL_SIZE = 2176


def _device():
    return torch.device("cuda", torch.cuda.current_device())


class BaseAgent(object):
    """agent_dg.py:31-100."""

    def __init__(self, env, results_path):
        self.env = env
        self.results_path = results_path
        random.seed(1)
        self.results = {}
        self.losses = []

    def write_results(self):
        output = [{"instr_id": k, "trajectory": v} for k, v in self.results.items()]
        with open(self.results_path, "w") as f:
            json.dump(output, f)

    def get_results(self):
        return [{"instr_id": k, "trajectory": v} for k, v in self.results.items()]

    def rollout(self, **kwargs):
        raise NotImplementedError

    @staticmethod
    def get_agent(name):
        return globals()[name + "Agent"]

    def test(self, iters=None, **kwargs):
        args.is_test = True
        self.env.reset_epoch(shuffle=(iters is not None))
        self.losses = []
        self.results = {}
        looped = False
        self.loss = 0
        if iters is not None:
            for _ in range(iters):
                for traj in self.vl_rollout(**kwargs):
                    self.loss = 0
                    self.results[traj["instr_id"]] = traj["path"]
        else:
            while True:
                for traj in self.vl_rollout(**kwargs):
                    if traj["instr_id"] in self.results:
                        looped = True
                    else:
                        self.loss = 0
                        self.results[traj["instr_id"]] = traj["path"]
                if looped:
                    break
        args.is_test = False


class DGAdaChannel(nn.Module):
    """agent_dg.py:1513-1547: a = sigmoid(a_fc(d)) (ab_type 'a'), out = a * f (+ b_fc(d) for 'ab'/'b').
    ab_type 'a' + a_type 'sigmoid' (the README configuration) is one fused GEMM + gate epilogue."""

    def __init__(self, channel, eps=1e-6):
        super().__init__()
        if args.ab_type in ["ab", "a"]:
            self.a_fc = nn.Linear(channel, channel)
        if args.ab_type in ["ab", "b"]:
            self.b_fc = nn.Linear(channel, channel)
        self.eps = eps

    def fused_ok(self):
        return args.ab_type == "a" and args.a_type == "sigmoid"

    def forward(self, f_t, d_t):
        if self.fused_ok():
            s = DF.linear(d_t, self.a_fc.weight, self.a_fc.bias, "sigmoid")
            return s * f_t
        a, b = 1, 0
        if args.ab_type in ["ab", "a"]:
            a = DF.linear(d_t, self.a_fc.weight, self.a_fc.bias)
        if args.ab_type in ["ab", "b"]:
            b = DF.linear(d_t, self.b_fc.weight, self.b_fc.bias)
        if args.a_type == "sigmoid":
            a = torch.sigmoid(a)
        elif args.a_type == "gumbel_sigmoid":
            raise NotImplementedError("gumbel_sigmoid AdaIN is not in any DASA configuration")
        return a * f_t + b

    def feature(self, f_full, d_full, noise=None):
        """df = f_full with its RGB columns replaced by forward(f, d) (* noise): one fused kernel chain."""
        if self.fused_ok():
            return DF.ada_feature(f_full, d_full, self.a_fc.weight, self.a_fc.bias, noise, args.angle_feat_size)
        out = f_full.clone()
        out[..., :-args.angle_feat_size] = self.forward(f_full[..., :-args.angle_feat_size],
                                                        d_full[..., :-args.angle_feat_size])
        if noise is not None:
            out[..., :-args.angle_feat_size] *= noise
        return out


# the pretraining heads of r2rpretrain_class.py:106-147 / :150-199 that a `.bert` hand-off drops
PRETRAIN_HEADS = {"DicAddActionPreTrain": ("next_action.", "mlmhead."),
                  "DicPMActionPreTrain": ("next_action.", "mlmhead.", "critic.")}


def _legacy_key(k):
    """pytorch_transformers' from_pretrained renames TF-style LayerNorm keys (gamma/beta)."""
    return k.replace("gamma", "weight") if "gamma" in k else (k.replace("beta", "bias") if "beta" in k else k)


def load_pretrained_bert(path, model_type="DicAddActionPreTrain"):
    """The DicModel of a pretrained checkpoint (agent_dg.py:165-188), loaded with the safe loader.

    * DicAddActionPreTrain (the README flag): `path` is a from_pretrained directory — config.json gives
      the architecture (vl_layers, la_layers, hidden sizes), pytorch_model.bin the weights.
    * DicPMActionPreTrain: `path` is a torch.save({'state_dict': ...}) file; the architecture is
      bert-base with the command line's d_vl_layers / d_la_layers (agent_dg.py:166-177).
    Stricter than pytorch_transformers' non-strict load: every DicModel key must be present, and every
    other key must belong to the model type's pretraining heads (PRETRAIN_HEADS); anything else raises
    instead of leaving randomly initialised layers behind silently."""
    from .vilmodel import BertConfig, DicModel
    from .._lib import DasaError
    if model_type not in PRETRAIN_HEADS:
        raise DasaError("--pretrain_model_type %r is not a DASA pretraining model" % model_type)
    if model_type == "DicPMActionPreTrain":
        cfg = BertConfig.from_pretrained("bert-base-uncased")
        cfg.img_feature_dim, cfg.img_feature_type = 2048 + args.angle_feat_size, ""
        cfg.update_lang_bert = cfg.update_add_layer = True
        cfg.vl_layers, cfg.la_layers, cfg.action_space = args.d_vl_layers, args.d_la_layers, 36
        states = torch.load(path, map_location="cpu", weights_only=True)
        if not isinstance(states, dict) or "state_dict" not in states:
            raise DasaError("%s: a DicPMActionPreTrain checkpoint is {'state_dict': ...}" % path)
        sd = states["state_dict"]
    else:
        if not os.path.isdir(path):
            raise DasaError("%s: a DicAddActionPreTrain checkpoint is a directory (config.json + "
                            "pytorch_model.bin)" % path)
        with open(os.path.join(path, "config.json")) as f:
            cfg = BertConfig(**json.load(f))
        sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
    for need in ("img_feature_dim", "vl_layers", "la_layers"):
        if not hasattr(cfg, need):
            raise DasaError("%s: the checkpoint config has no %r" % (path, need))
    if not hasattr(cfg, "img_feature_type"):
        cfg.img_feature_type = ""
    for flag in ("update_lang_bert", "update_add_layer"):
        if not hasattr(cfg, flag):
            setattr(cfg, flag, True)
    bert = DicModel(cfg)
    heads = PRETRAIN_HEADS[model_type]
    bert_sd, stray = {}, []
    for k, v in sd.items():
        k = _legacy_key(k)
        if k.startswith("bert."):
            bert_sd[k[len("bert."):]] = v
        elif not k.startswith(heads):
            stray.append(k)
    want = set(bert.state_dict())
    missing, unexpected = sorted(want - set(bert_sd)), sorted(set(bert_sd) - want)
    if stray or missing or unexpected:
        raise DasaError("%s: not a %s checkpoint of this architecture (keys outside bert.* and the heads %s: "
                        "%s; missing: %s; unexpected: %s)" % (path, model_type, heads, stray[:5], missing[:5],
                                                              unexpected[:5]))
    bert.load_state_dict(bert_sd, strict=True)
    return bert


MAX_CANDIDATES = 255   # navigable viewpoints per observation (+ the stop row = 256 = the HIP kernels' C limit)


def _check_candidates(obs):
    """The candidate attention and the policy head take C <= 256 rows per decision (include/dasa_hip.h:
    dasa_softdot_fwd N <= 256, dasa_policy_head_fwd C <= 256; R2R viewpoints have at most a few dozen
    navigable neighbours). The reference's masked_fill + CrossEntropy + Categorical take any count, so a
    larger candidate list is refused here, where the observation is read, with the limit named."""
    n = max((len(ob["candidate"]) for ob in obs), default=0)
    if n > MAX_CANDIDATES:
        raise NotImplementedError(f"an observation has {n} navigable candidates; the MI355X path takes at most "
                                  f"{MAX_CANDIDATES} (+ stop) per decision step")


class Seq2SeqAgent(BaseAgent):
    """agent_dg.py:102-1510 (encoder_type 'Dic' — the DASA configuration)."""

    env_actions = {
        "left": (0, -1, 0), "right": (0, 1, 0), "up": (0, 0, 1), "down": (0, 0, -1),
        "forward": (1, 0, 0), "<end>": (0, 0, 0), "<start>": (0, 0, 0), "<ignore>": (0, 0, 0),
    }

    def __init__(self, env, results_path, tok, episode_len=20, encoder_type="EncoderLSTM"):
        super().__init__(env, results_path)
        self.tok = tok
        self.episode_len = episode_len
        self.feature_size = self.env.feature_size
        self.encoder_type = encoder_type
        self.device = _device()
        if encoder_type in ("EncoderLSTM", "DicEncoder", "CEncoder"):
            raise NotImplementedError("encoder_type %r is not the DASA (Dic) agent" % encoder_type)
        self.encoder = DicEncoder(FEATURE_ALL_SIZE, args.d_enc_hidden_size, args.d_hidden_size, args.d_dropout_ratio,
                                  args.d_bidirectional, args.d_transformer_update, args.d_bert_n_layers,
                                  args.d_reverse_input, args.d_top_lstm, args.d_vl_layers, args.d_la_layers,
                                  args.d_bert_type, update_add_layer=args.d_update_add_layer).to(self.device)
        if args.pretrain_model_name is not None:
            self._load_pretrained_bert(args.pretrain_model_name)
        self.decoder = model.BAttnDecoderLSTM(args.aemb, args.d_hidden_size, args.dropout,
                                              feature_size=self.feature_size + args.angle_feat_size,
                                              pred_back=args.pred_back).to(self.device)
        self.critic = model.Critic().to(self.device)
        if args.adaIn_type in ("channel", "rgb_channel"):
            self.adaIn = DGAdaChannel(args.feature_size).to(self.device)
        elif args.adaIn_type in ("default", "none"):
            self.adaIn = None
        else:
            raise NotImplementedError("adaIn_type %r is outside the DASA configurations" % args.adaIn_type)

        self.encoder_optimizer = args.optimizer(self.encoder.parameters(), lr=args.lr, weight_decay=args.weight_decay)
        self.decoder_optimizer = args.optimizer(self.decoder.parameters(), lr=args.lr, weight_decay=args.weight_decay)
        self.critic_optimizer = args.optimizer(self.critic.parameters(), lr=args.lr, weight_decay=args.weight_decay)

        def lr_lambda(it):   # agent_dg.py:219-227
            if args.warm_steps > 0 and it < args.warm_steps:
                return (1.0 + it) / args.warm_steps
            if it < args.decay_start:
                return 1.0
            return args.lr_decay ** ((it - args.decay_start) // args.decay_intervals)

        if args.use_lr_scheduler:
            self.decoder_lr_scheduler = torch.optim.lr_scheduler.LambdaLR(self.decoder_optimizer, lr_lambda)
            self.critic_lr_scheduler = torch.optim.lr_scheduler.LambdaLR(self.critic_optimizer, lr_lambda)
        else:
            self.decoder_lr_scheduler = None
            self.critic_lr_scheduler = None
        if args.adaIn_type not in ("default", "none"):
            self.adaIn_optimizer = args.optimizer(self.adaIn.parameters(), lr=args.lr)
            self.adaIn_lr_scheduler = torch.optim.lr_scheduler.LambdaLR(self.adaIn_optimizer, lr_lambda)
            self.models = (self.encoder, self.decoder, self.critic, self.adaIn)
            self.optimizers = (self.encoder_optimizer, self.decoder_optimizer, self.critic_optimizer,
                               self.adaIn_optimizer)
        else:
            self.models = (self.encoder, self.decoder, self.critic)
            self.optimizers = (self.encoder_optimizer, self.decoder_optimizer, self.critic_optimizer)
        self.losses = []
        self.criterion = nn.CrossEntropyLoss(ignore_index=args.ignoreid, reduction="sum")
        self.logs = defaultdict(list)
        self.sample_fn = None        # test hook: "argmax" replaces the sampled rollout's Categorical draw by the argmax
        # test hook: (step, candidate lengths) -> int64 [B] actions replacing the draw of the sampled
        # rollout while the one-kernel policy head stays on (dasa_policy_head_fwd mode FORCED)
        self.force_action_fn = None
        self._step_graphs = None     # captured forward-only decision steps (_graph_step)
        self._train_graphs = None    # captured training decoder steps (_decode, graph.AutogradGraphs)
        self.grad_sync = None        # data-parallel hook set by dasa_amd.dp

    def _load_pretrained_bert(self, path):
        """--pretrain_model_name (agent_dg.py:165-188): the encoder's DicModel becomes the pretrained
        model's `.bert` — its depth (vl_layers / la_layers) is the checkpoint's, not the command line's —
        then dropout and the update flags are reset from args as the reference does."""
        bert = load_pretrained_bert(path, args.pretrain_model_type)
        self.encoder.bert = bert.to(self.device)
        self.encoder.drop = nn.Dropout(p=args.d_dropout_ratio)
        self.encoder.bert.update_lang_bert = self.encoder.bert.config.update_lang_bert = args.d_transformer_update
        self.encoder.bert.update_add_layer = self.encoder.bert.config.update_add_layer = args.d_update_add_layer

    # ------------------------------------------------------------------ observation -> tensors
    def _sort_batch(self, obs):
        """agent_dg.py:262-284."""
        seq_tensor = np.array([ob["instr_encoding"] for ob in obs])
        seq_lengths = np.argmax(seq_tensor == utils.padding_idx, axis=1)
        seq_lengths[seq_lengths == 0] = seq_tensor.shape[1]
        seq_tensor = torch.from_numpy(seq_tensor)
        seq_lengths = torch.from_numpy(seq_lengths)
        seq_lengths, perm_idx = seq_lengths.sort(0, True)
        sorted_tensor = seq_tensor[perm_idx]
        mask = (sorted_tensor == utils.padding_idx)[:, :seq_lengths[0]]
        progresses = torch.Tensor([ob["progress"] for ob in obs])[perm_idx].float().to(self.device)
        return (sorted_tensor.long().to(self.device), mask.bool().to(self.device), list(seq_lengths),
                list(perm_idx), progresses)

    def _fused_head(self, logit):  # noqa: D401
        """Every decision step's loss / action stage is the one-kernel policy head (dasa_policy_head_fwd,
        C <= 256 candidates); --submit's visited candidates and the back-prediction head (--pred_back) are
        fed to it as an extra mask / a second teacher-mode call."""
        if logit.shape[1] > 256:
            raise NotImplementedError("more than 256 candidates per viewpoint")
        return True

    def _head_mode(self):
        """The policy head's mode for this rollout's feedback (agent_dg.py:862-886): teacher, argmax,
        sample (a Categorical draw on the device RNG), forced (force_action_fn: a caller's action table)
        or sample_argmax (sample_fn == "argmax": Categorical semantics with the draw replaced by the
        argmax, the golden fixtures' sampled rollouts)."""
        fb = self.feedback
        if fb == "sample":
            if self.force_action_fn is not None:
                return "forced"
            if self.sample_fn is None:
                return "sample"
            if self.sample_fn == "argmax":
                return "sample_argmax"
            raise NotImplementedError("sample_fn: None or 'argmax' (the policy head draws on the device)")
        if fb in ("teacher", "argmax"):
            return fb
        sys.exit("Invalid feedback option")

    def _visited_mask(self, perm_obs, visited, C):
        """--submit (agent_dg.py:852-858): a candidate whose viewpoint the agent already visited is masked
        like a padding candidate; updates `visited` with this step's viewpoints."""
        m = np.zeros((len(perm_obs), C), dtype=bool)
        for i, ob in enumerate(perm_obs):
            visited[i].add(ob["viewpoint"])
            for c_id, c in enumerate(ob["candidate"]):
                if c["viewpointId"] in visited[i]:
                    m[i, c_id] = True
        return self._to_dev(m)

    def _lens_dev(self, leng):
        return self._to_dev(np.asarray(leng, dtype=np.int32))

    def _to_dev(self, arr):
        return torch.from_numpy(arr).pin_memory().to(self.device, non_blocking=True)

    def _feature_variable(self, obs):
        features = np.empty((len(obs), args.views, self.feature_size + args.angle_feat_size), dtype=np.float32)
        for i, ob in enumerate(obs):
            features[i] = ob["feature"]
        return self._to_dev(features)

    def _dfeature_variable(self, obs):
        dfeatures = np.empty((len(obs), args.views, self.feature_size + args.angle_feat_size), dtype=np.float32)
        for i, ob in enumerate(obs):
            dfeatures[i] = ob["dfeature"]
        return self._to_dev(dfeatures)

    def _candidate_variable(self, obs):
        candidate_leng = [len(ob["candidate"]) + 1 for ob in obs]
        cf = np.zeros((len(obs), max(candidate_leng), self.feature_size + args.angle_feat_size), dtype=np.float32)
        cd = np.zeros_like(cf)
        for i, ob in enumerate(obs):
            for j, c in enumerate(ob["candidate"]):
                cf[i, j] = c["feature"]
                cd[i, j] = c["dfeature"]
        return self._to_dev(cf), self._to_dev(cd), candidate_leng

    def get_input_feat(self, obs):
        """agent_dg.py:313-323; device-side gather when the env provides one."""
        _check_candidates(obs)
        if hasattr(self.env, "device_input_feat"):
            return self.env.device_input_feat(obs, self.device)
        input_a_t = np.zeros((len(obs), args.angle_feat_size), np.float32)
        for i, ob in enumerate(obs):
            input_a_t[i] = utils.angle_feature(ob["heading"], ob["elevation"])
        input_a_t = self._to_dev(input_a_t)
        f_t = self._feature_variable(obs)
        d_t = self._dfeature_variable(obs)
        cf, cd, leng = self._candidate_variable(obs)
        return input_a_t, f_t, d_t, cf, cd, leng

    def _teacher_action(self, obs, ended):
        return self._to_dev(self._teacher_action_np(obs, ended))

    def _teacher_action_np(self, obs, ended):
        """agent_dg.py:325-344 on the host (the device copy is made without a sync)."""
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

    def _back_teacher_action(self, obs, ended):
        a = np.zeros(len(obs), dtype=np.int64)
        for i, ob in enumerate(obs):
            for k, candidate in enumerate(ob["candidate"]):
                if candidate["viewpointId"] == ob["back_teacher"]:
                    a[i] = k
                    break
            else:
                assert ob["back_teacher"] == ob["viewpoint"]
                a[i] = len(ob["candidate"])
        return torch.from_numpy(a).to(self.device)

    def make_equiv_action(self, a_t, perm_obs, perm_idx=None, traj=None):
        """agent_dg.py:358-391. Simulators exposing quick_state() (the synthetic MatterSim stand-in)
        are polled without building a SimState per turn; same actions, same trajectory."""
        sims = self.env.env.sims

        def take_action(i, sim, name):
            if type(name) is int:
                sim.makeAction(name, 0, 0)
            else:
                sim.makeAction(*self.env_actions[name])
            if traj is not None:
                if hasattr(sim, "quick_state"):
                    traj[i]["path"].append(sim.quick_state()[:3])
                else:
                    state = sim.getState()
                    traj[i]["path"].append((state.location.viewpointId, state.heading, state.elevation))

        def view_index(sim):
            return sim.quick_state()[3] if hasattr(sim, "quick_state") else sim.getState().viewIndex
        if perm_idx is None:
            perm_idx = range(len(perm_obs))
        for i, idx in enumerate(perm_idx):
            action = a_t[i]
            if action != -1:
                sim = sims[idx]
                select_candidate = perm_obs[i]["candidate"][action]
                if hasattr(sim, "equiv_action"):     # the same action sequence, one call per agent
                    assert select_candidate["viewpointId"] == sim.navigable_id(select_candidate["idx"])
                    sim.equiv_action(select_candidate["pointId"], select_candidate["idx"],
                                     traj[i]["path"] if traj is not None else None)
                    continue
                src_point = perm_obs[i]["viewIndex"]
                trg_point = select_candidate["pointId"]
                src_level = src_point // 12
                trg_level = trg_point // 12
                while src_level < trg_level:
                    take_action(i, sim, "up")
                    src_level += 1
                while src_level > trg_level:
                    take_action(i, sim, "down")
                    src_level -= 1
                while view_index(sim) != trg_point:
                    take_action(i, sim, "right")
                nav_id = (sim.navigable_id(select_candidate["idx"]) if hasattr(sim, "navigable_id") else
                          sim.getState().navigableLocations[select_candidate["idx"]].viewpointId)
                assert select_candidate["viewpointId"] == nav_id
                take_action(i, sim, select_candidate["idx"])

    # ------------------------------------------------------------------ the rollout
    def _noise_mult(self, x, noise):
        """x[..., :-angle] *= noise, out of place (shared env-drop mask, agent_dg.py:731-736, 780-785)."""
        out = torch.empty_like(x)
        ops.colscale(x[..., :-args.angle_feat_size], noise, out[..., :-args.angle_feat_size])
        ops.copy2d(x[..., -args.angle_feat_size:], out[..., -args.angle_feat_size:])
        return out

    def _batch_teacher_ok(self):
        """Teacher-forced rollouts are encoded for all steps at once unless a per-step host decision
        needs the policy (--submit's visited masks) or it is switched off (DASA_TEACHER_BATCH=0)."""
        return not args.submit and os.environ.get("DASA_TEACHER_BATCH", "1") != "0"

    def _step_reward(self, perm_obs, cpu_a_t, ended, last_dist):
        """agent_dg.py:900-925: reward / mask of one step; updates last_dist in place."""
        batch_size = len(perm_obs)
        dist = np.zeros(batch_size, np.float32)
        reward = np.zeros(batch_size, np.float32)
        mask = np.ones(batch_size, np.float32)
        for i, ob in enumerate(perm_obs):
            dist[i] = ob["distance"]
            if ended[i]:
                reward[i] = 0.0
                mask[i] = 0.0
            else:
                action_idx = cpu_a_t[i]
                if action_idx == -1:
                    reward[i] = 2.0 if dist[i] < 3 else -2.0
                else:
                    reward[i] = -(dist[i] - last_dist[i])
                    if reward[i] > 0:
                        reward[i] = 1
                    elif reward[i] < 0:
                        reward[i] = -1
                    else:
                        raise NameError("The action doesn't change the move")
        last_dist[:] = dist
        return reward, mask

    def _teacher_plan(self, perm_obs, perm_idx, ended, last_dist, traj, n_steps):
        """Steps the env through up to n_steps teacher-forced steps ahead of the policy work (the
        reference interleaves the same env calls with the decoder, agent_dg.py:832-936; the teacher
        action depends only on the observation and `ended`, :325-344). Returns one record per step
        (observations, teacher targets, ended-before-step, reward, mask) and the final observations;
        `ended`, `last_dist` and `traj` are advanced in place exactly as the step loop advances them.
        Stops early when every row has ended."""
        plan = []
        for _ in range(n_steps):
            if ended.all():
                break
            target_np = self._teacher_action_np(perm_obs, ended)
            rec = {"obs": perm_obs, "target_np": target_np, "ended": ended.copy()}
            cpu_a_t = target_np.copy()
            for i, next_id in enumerate(cpu_a_t):
                if next_id == len(perm_obs[i]["candidate"]) or next_id == args.ignoreid:
                    cpu_a_t[i] = -1
            self.make_equiv_action(cpu_a_t, perm_obs, perm_idx, traj)
            obs = np.array(self.env._get_obs())
            perm_obs = obs[perm_idx]
            rec["reward"], rec["mask"] = self._step_reward(perm_obs, cpu_a_t, ended, last_dist)
            plan.append(rec)
            ended[:] = np.logical_or(ended, (cpu_a_t == -1))
            if ended.all():
                break
        return plan, perm_obs

    def _step_inputs(self, obs_steps):
        """get_input_feat for several steps, stacked along the batch (step-major); the candidates of
        all steps as flat rows [R, F] with cinfo[t] = (first row, C_t, candidate lengths)."""
        if hasattr(self.env, "device_input_feat_steps"):
            return self.env.device_input_feat_steps(obs_steps, self.device)
        parts = [self.get_input_feat(o) for o in obs_steps]
        cinfo, row = [], 0
        for p in parts:
            cinfo.append((row, p[3].shape[1], p[5]))
            row += p[3].shape[0] * p[3].shape[1]
        cat = (lambda ts: ts[0] if len(ts) == 1 else torch.cat(ts, 0))
        return (cat([p[0] for p in parts]), cat([p[1] for p in parts]), cat([p[2] for p in parts]),
                cat([p[3].reshape(-1, p[3].shape[-1]) for p in parts]),
                cat([p[4].reshape(-1, p[4].shape[-1]) for p in parts]), cinfo)

    def _graph_step_ok(self, t, consistent_drop, noise, speaker):
        """A forward-only argmax decision step (eval rollouts) whose whole device work — AdaIN, the
        encoder (VisionEncoder + LXRT + bi-LSTM + init projections), the decoder and the policy head —
        replays as ONE captured hipGraph (dasa_amd/graph.py), keyed by the candidate count: every step
        after the first of a rollout, once the rollout's language stack is cached."""
        enc = self.encoder
        return (graph.ENABLED and t > 0 and self.feedback == "argmax" and not torch.is_grad_enabled()
                and not enc.training and not self.decoder.training and speaker is None
                and not (consistent_drop and noise is not None) and not args.submit and not args.pred_back
                and self.sample_fn is None and os.environ.get("DASA_STEP_GRAPH", "1") != "0"
                and enc._lang_cache_on and enc._lang_cache is not None and not prof.active()
                # a caller that wraps or hooks the modules observes every per-step call: run eagerly
                and all("forward" not in m.__dict__ and not m._forward_hooks and not m._forward_pre_hooks
                        for m in (enc, self.decoder, self.adaIn)))

    def _graph_step(self, perm_obs, target, h_t, h1, c_t, seq, seq_mask, lens_dev, ctx_mask):
        """agent_dg.py:725-886 for one argmax step as a graph replay. The observation gather (host index
        arrays -> dasa_gather_rows) stays outside the graph; the replay reads the gathered blocks, the
        recurrent state, the rollout's cached language stack and the step's host-built candidate lengths
        / teacher targets from its static buffers. Returns (candidate lengths, (h_t, c_t, logit, h1,
        ce, log-prob of the action, action))."""
        inputs = self._step_inputs([perm_obs])
        a, f, d, cf, cd, cinfo = inputs
        _, C, leng = cinfo[0]
        B = a.shape[0]
        cand_lens = self._lens_dev(leng)
        text = self.encoder._lang_cache[1]
        if self._step_graphs is None:
            self._step_graphs = graph.StepGraphs([self.encoder, self.decoder, self.adaIn])

        def step(a, f, d, cf, cd, seq, seq_mask, lens_dev, h_t, h1, c_t, ctx_mask, cand_lens, target, text):
            self.encoder._text_in = text
            try:
                (e,) = self._encode_steps(None, seq, seq_mask, lens_dev, None, False,
                                          inputs=(a, f, d, cf, cd, [(0, C, leng)]))
            finally:
                self.encoder._text_in = None
            h_t2, c_t2, logit, h1_2, _ = self.decoder(e["a"], e["df"], e["cand"], h_t, h1, c_t, e["ctx"], ctx_mask,
                                                      already_dropfeat=False)
            ce, _, lpa, a_dev = DF.policy_head(logit, cand_lens, target, "argmax")
            return h_t2, c_t2, logit, h1_2, ce, lpa, a_dev
        ops._exclusive(self.device)
        outs = self._step_graphs.run((B, C, seq.shape[1]), step, (a, f, d, cf, cd, seq, seq_mask, lens_dev, h_t, h1,
                                                                  c_t, ctx_mask, cand_lens, target, text))
        return leng, outs

    def _train_graph_ok(self):
        """A training decoder step (decoder + one-kernel policy head, with autograd) replays as a captured
        graph (graph.AutogradGraphs) unless a per-step host decision or a caller-visible module hook
        needs the eager calls, the profiler brackets every launch, or it is switched off
        (DASA_TRAIN_GRAPH=0)."""
        dec = self.decoder
        return (graph.ENABLED and os.environ.get("DASA_TRAIN_GRAPH", "1") != "0" and torch.is_grad_enabled()
                and dec.training and not prof.active() and not graph.capturing()
                and not args.decoder_consistent_drop and not args.pred_back and not args.submit
                and isinstance(dec.drop_env, nn.Dropout)
                and "forward" not in dec.__dict__ and not dec._forward_hooks and not dec._forward_pre_hooks
                and (self._train_graphs is None or len(self._train_graphs.slots) < 1024))

    def _decode(self, t, mode, e, h0, prev_h1, c0, ctx_mask, cand_lens, target, forced, dropfeat, extra_mask=None,
                back_target=None):
        """agent_dg.py:811-886 for one step: BAttnDecoderLSTM + the one-kernel policy head (mask, CE,
        action, entropy / log-prob). Training steps replay a captured graph keyed by the step index;
        the candidate block is zero-padded and the instruction context padded to --maxInput tokens with
        the padding masked (_slot_pads): the head masks padded candidates and the
        instruction attention gives masked tokens weight 0, so every valid logit, loss and gradient is
        unchanged while few shapes (slots) arise. Otherwise eager, with --submit's extra mask and the
        --pred_back CE (a second teacher-mode head call on the back logits, agent_dg.py:872-876).
        Returns (h_t, c_t, logit, h1, ce, entropy, log-prob of the action, action, back CE or None)."""
        dec = self.decoder

        def step(a, df, cand, h0, prev_h1, c0, ctx, ctx_mask, cand_lens, target, forced):
            h_t, c_t, logit, h1, _ = dec(a, df, cand, h0, prev_h1, c0, ctx, ctx_mask, already_dropfeat=dropfeat)
            ce, ent, lpa, act = DF.policy_head(logit, cand_lens, target, mode, forced=forced)
            return h_t, c_t, logit, h1, ce, ent, lpa, act
        if extra_mask is not None or args.pred_back or not self._train_graph_ok():
            h_t, c_t, logit, h1, aux = dec(e["a"], e["df"], e["cand"], h0, prev_h1, c0, e["ctx"], ctx_mask,
                                           already_dropfeat=dropfeat)
            if extra_mask is not None:
                logit = logit.masked_fill(extra_mask, -float("inf"))
            ce, ent, lpa, act = DF.policy_head(logit, cand_lens, target, mode, forced=forced)
            back = None
            if args.pred_back:
                bl = aux["back_logit"]
                if extra_mask is not None:
                    bl = bl.masked_fill(extra_mask, -float("inf"))
                back = DF.policy_head(bl, cand_lens, back_target, "teacher")[0]
            return h_t, c_t, logit, h1, ce, ent, lpa, act, back
        inputs = (e["a"], e["df"], e["cand"], h0, prev_h1, c0, e["ctx"], ctx_mask, cand_lens, target, forced)
        if self._train_graphs is None:
            # every module any captured region reads (teacher-forcing decoder steps AND the AdaIN + decoder
            # regions of _adain_decode), so a re-assigned parameter of either re-captures
            self._train_graphs = graph.AutogradGraphs([self.decoder, self.adaIn])
        B, C, F = e["cand"].shape
        L, H2 = e["ctx"].shape[1:]
        Cp, Lp = self._slot_pads(C, L)
        key = ("dec", mode, t, B, Cp, Lp, H2, bool(dropfeat))
        out = self._train_graphs.run(key, step, inputs, pads={2: ((B, Cp, F), 0), 6: ((B, Lp, H2), 0),
                                                              7: ((B, Lp), True)})
        return out[:2] + (out[2][:, :C],) + out[3:] + (None,)

    @staticmethod
    def _slot_pads(C, L):
        """Padded candidate / instruction extents of a captured training step: candidates to 16, 32, 64, ...
        and the instruction context to the longest instruction the encoder admits (--maxInput, rounded
        up to 16), so a slot serves every batch of its step index — at small B the batch's longest
        instruction and candidate count vary from batch to batch, and per-extent slots would re-capture
        for most steps. Padded tokens are masked, padded candidates lie past every row's length."""
        Cp = 16
        while Cp < C:
            Cp *= 2
        Lp = -(-max(L, args.maxInput) // 16) * 16
        return Cp, Lp

    def _step_region_ok(self, consistent_drop, noise):
        """The per-step loop's AdaIN joins the captured decoder region (_adain_decode) in the README
        configuration: the channel AdaIN as one fused gate, no --ctx_v, and the shared env-drop noise
        (aug half) only after AdaIN (agent_dg.py:764-785)."""
        use_noise = consistent_drop and noise is not None
        return (self._train_graph_ok() and args.adaIn_type == "channel" and self.adaIn.fused_ok() and not args.ctx_v
                and (not use_noise or args.env_drop_stage == "after_adain"))

    def _adain_decode(self, t, mode, inputs, seq, seq_mask, lens_dev, noise, consistent_drop, h_t, h1, c_t, ctx_mask,
                      target, forced_fn):
        """One decision step of the per-step loop (agent_dg.py:725-886) with AdaIN, the decoder and the
        policy head as ONE captured training region: the observation gather and the DicEncoder (its
        language stack comes from the side-stream pipe, the bi-LSTM needs the whole chip) run eagerly
        around it. Same values as _encode_steps + _decode. Returns (leng, ctx, h_t, c_t, logit, h1, ce,
        entropy, log-prob, action)."""
        a, f, d, cf, cd, cinfo = inputs
        _, C, leng = cinfo[0]
        B = a.shape[0]
        use_noise = consistent_drop and noise is not None
        img = self._noise_mult(f, noise) if (use_noise and args.use_dropout_vision) else f   # agent_dg.py:780-797
        ctx, en_ht, en_ct, _, _ = self.encoder(seq, mask=seq_mask, lengths=lens_dev, f_t_all=img, want_vision=False)
        h0, c0, prev = (en_ht, en_ct, en_ht) if t == 0 else (h_t, c_t, h1)
        forced = forced_fn(leng) if forced_fn is not None else None
        cand_lens = self._lens_dev(leng)
        dec, ada, depth_drop = self.decoder, self.adaIn, args.depth_drop

        def step(a, f, d, cf, cd, noise, h0, prev_h1, c0, ctx, ctx_mask, cand_lens, target, forced):
            df = ada.feature(f, d, noise if (noise is not None and depth_drop) else None)
            cand = ada.feature(cf, cd, noise)
            h_t, c_t, logit, h1, _ = dec(a, df, cand, h0, prev_h1, c0, ctx, ctx_mask, already_dropfeat=consistent_drop)
            ce, ent, lpa, act = DF.policy_head(logit, cand_lens, target, mode, forced=forced)
            return h_t, c_t, logit, h1, ce, ent, lpa, act
        cf3, cd3 = cf.view(B, C, -1), cd.view(B, C, -1)
        step_in = (a, f, d, cf3, cd3, noise if use_noise else None, h0, prev, c0, ctx, ctx_mask, cand_lens, target,
                   forced)
        if self._train_graphs is None:
            self._train_graphs = graph.AutogradGraphs([self.decoder, self.adaIn])
        F = cf3.shape[2]
        L, H2 = ctx.shape[1:]
        Cp, Lp = self._slot_pads(C, L)
        key = ("step", mode, t, B, Cp, Lp, H2, bool(consistent_drop), bool(use_noise))
        out = self._train_graphs.run(key, step, step_in, pads={3: ((B, Cp, F), 0), 4: ((B, Cp, F), 0),
                                                               9: ((B, Lp, H2), 0), 10: ((B, Lp), True)})
        return (leng, ctx) + out[:2] + (out[2][:, :C],) + out[3:]

    def _encode_steps(self, obs_steps, seq, seq_mask, lens_dev, noise, consistent_drop, inputs=None):
        """Feature stage of the step loop (agent_dg.py:725-805): features -> env drop -> AdaIN ->
        DicEncoder, for one or several steps' observations at once (every op in it is per row, so
        stacking T steps along the batch computes each step's values; dropout draws stay independent
        per row and step). Returns per step: angle input, AdaIN'd panorama, AdaIN'd candidates,
        candidate lengths, ctx and the encoder's decoder-init states."""
        angle = args.angle_feat_size
        if inputs is None:
            inputs = self._step_inputs(obs_steps)
        input_a_t, f_t, d_t, candidate_feat, candidate_dfeat, cinfo = inputs
        T = len(cinfo)
        B = input_a_t.shape[0] // T
        stage = args.env_drop_stage
        use_noise = consistent_drop and noise is not None
        all_img_feats = f_t                  # the raw panorama (agent_dg.py:730)
        df_t = f_t                           # df_t = f_t.clone() (agent_dg.py:728), copied lazily below
        if use_noise and stage == "before_adain":     # agent_dg.py:731-736
            candidate_feat = self._noise_mult(candidate_feat, noise)
            f_t = self._noise_mult(f_t, noise)
            if args.depth_drop:
                candidate_dfeat = self._noise_mult(candidate_dfeat, noise)
                df_t = f_t
        after = use_noise and stage == "after_adain"
        if args.adaIn_type in ("channel", "rgb_channel"):            # agent_dg.py:748-768
            style_v = f_t if args.adaIn_type == "rgb_channel" else d_t
            style_c = candidate_feat if args.adaIn_type == "rgb_channel" else candidate_dfeat
            # df_t's angle columns are df_t's own (== f_t's); its RGB columns are replaced
            df_t = self.adaIn.feature(f_t, style_v, noise if (after and args.depth_drop) else None)
            candidate_feat = self.adaIn.feature(candidate_feat, style_c, noise if after else None)
            if after:
                f_t = self._noise_mult(f_t, noise)
        elif args.adaIn_type == "default":                             # agent_dg.py:774-777
            f_t = f_t.clone()
            model.adaptive_instance_normalization(f_t[..., :-angle], d_t[..., :-angle], out=f_t[..., :-angle])
            candidate_feat = candidate_feat.clone()
            model.adaptive_instance_normalization(candidate_feat[..., :-angle], candidate_dfeat[..., :-angle],
                                                  out=candidate_feat[..., :-angle])
            if after:                                                  # agent_dg.py:780-785
                candidate_feat = self._noise_mult(candidate_feat, noise)
                f_t = self._noise_mult(f_t, noise)
                if args.depth_drop:
                    df_t = self._noise_mult(df_t, noise)
        elif after:
            candidate_feat = self._noise_mult(candidate_feat, noise)
            f_t = self._noise_mult(f_t, noise)
            if args.depth_drop:
                df_t = self._noise_mult(df_t, noise)
        img = f_t if args.use_dropout_vision else all_img_feats
        wv = bool(args.ctx_v)   # vision_outputs are consumed only with --ctx_v (agent_dg.py:807-808)
        if T == 1:
            ctx, en_ht, en_ct, _, ctx_v = self.encoder(seq, mask=seq_mask, lengths=lens_dev, f_t_all=img,
                                                       want_vision=wv)
        else:
            ctx, en_ht, en_ct, _, ctx_v = self.encoder(seq.repeat(T, 1), mask=seq_mask.repeat(T, 1),
                                                       lengths=lens_dev.repeat(T), f_t_all=img, want_vision=wv)
        if args.ctx_v:
            df_t = df_t + ctx_v
        out = []
        for t in range(T):
            sl = slice(t * B, (t + 1) * B)
            off, C, leng = cinfo[t]
            out.append({"a": input_a_t[sl], "df": df_t[sl], "cand": candidate_feat[off:off + B * C].view(B, C, -1),
                        "leng": leng, "ctx": ctx[sl], "en_ht": en_ht[sl], "en_ct": en_ct[sl]})
        return out

    def vl_rollout(self, train_ml=None, train_rl=True, reset=True, speaker=None):
        """agent_dg.py:633-1033."""
        if self.feedback == "teacher" or self.feedback == "argmax":
            train_rl = False
        obs = np.array(self.env.reset()) if reset else np.array(self.env._get_obs())
        batch_size = len(obs)
        noise = None
        if speaker is not None:
            noise = self.decoder.drop_env(torch.ones(self.feature_size, device=self.device))
            batch = self.env.batch.copy()
            speaker.env = self.env
            insts = speaker.infer_batch(featdropmask=noise)
            inst_lengths = np.argmax(insts == self.tok.tokenizer.pad_token_id, axis=1)
            inst_lengths[inst_lengths == 0] = insts.shape[1]
            for i, (datum, inst) in enumerate(zip(batch, insts)):
                inst = inst[:inst_lengths[i]]
                if inst[-1] == speaker.tok.word_to_index["<EOS>"]:
                    inst = inst[:-1]
                datum.pop("instructions")
                datum.pop("instr_encoding")
                datum["instructions"] = speaker.tok.decode_sentence(inst)
                datum["instr_encoding"] = self.tok.encode_sentence(datum["instructions"])
            obs = np.array(self.env.reset(batch))
        elif args.consistent_drop:
            noise = self.decoder.drop_env(torch.ones(self.feature_size, device=self.device))

        seq, seq_mask, seq_lengths, perm_idx, progresses = self._sort_batch(obs)
        perm_obs = obs[perm_idx]
        ctx_mask = seq_mask
        lens_dev = torch.as_tensor([int(x) for x in seq_lengths], dtype=torch.int32).to(self.device)
        if not args.include_vision:
            raise NotImplementedError("include_vision=False is not the DASA configuration")

        last_dist = np.zeros(batch_size, np.float32)
        for i, ob in enumerate(perm_obs):
            last_dist[i] = ob["distance"]
        traj = [{"instr_id": ob["instr_id"], "path": [(ob["viewpoint"], ob["heading"], ob["elevation"])]}
                for ob in perm_obs]
        visited = [set() for _ in perm_obs]
        ended = np.array([False] * batch_size)
        rewards, hidden_states, policy_log_probs, masks, entropys = [], [], [], [], []
        deferred = defaultdict(list)     # logs whose .item() is taken after the loop
        ml_loss = 0.0
        # per-step loss terms, summed once after the loop on the library's kernels (DF.sum_terms): a torch
        # scalar add per step ran its packed-FP32 kernel beside the language pipe's GEMMs
        forth_terms, back_terms, ent_terms = [], [], []
        consistent_drop = args.consistent_drop or (speaker is not None)
        if args.decoder_consistent_drop:
            self.decoder.init_noise((seq.shape[0], args.d_enc_hidden_size))
        enc_args = (seq, seq_mask, lens_dev, noise, consistent_drop)
        h_t = c_t = h1 = ctx = None
        if self.feedback == "teacher" and self._batch_teacher_ok():
            # Teacher forcing: the actions (and so every observation of the episode) do not depend
            # on the policy, so the env is stepped first and the encoder runs once for all steps.
            # Chunked: the host steps the env for chunk k+1 while the GPU encodes and decodes chunk k.
            # The env is stepped one chunk ahead: chunk k+1 is planned on the host right after chunk
            # k's encoder is enqueued, while the GPU runs it (the first chunk is half-size so the GPU
            # starts early).
            self.encoder.cache_language(not self.encoder.training, steps=0, rows=batch_size)
            chunk = max(1, int(os.environ.get("DASA_TEACHER_CHUNK", "8")))
            t = 0
            plan = []
            if not ended.all():
                plan, perm_obs = self._teacher_plan(perm_obs, perm_idx, ended, last_dist, traj,
                                                    min(max(1, chunk // 2), self.episode_len))
            while plan:
                enc = self._encode_steps([s["obs"] for s in plan], *enc_args)
                targets = self._to_dev(np.stack([s["target_np"] for s in plan]))
                t_next = t + len(plan)
                nxt = []
                if t_next < self.episode_len and not ended.all():
                    nxt, perm_obs = self._teacher_plan(perm_obs, perm_idx, ended, last_dist, traj,
                                                       min(chunk, self.episode_len - t_next))
                for i, (s, e) in enumerate(zip(plan, enc)):
                    self._fused_head(e["cand"][:, :, 0])
                    h0, c0 = (e["en_ht"], e["en_ct"]) if t == 0 else (h_t, c_t)
                    back_target = self._back_teacher_action(s["obs"], s["ended"]) if args.pred_back else None
                    h_t, c_t, logit, h1, ce, _, _, _, back = self._decode(
                        t, "teacher", e, h0, h0 if t == 0 else h1, c0, ctx_mask, self._lens_dev(e["leng"]),
                        targets[i], None, consistent_drop, None, back_target)
                    forth_terms.append(ce)
                    if back is not None:
                        back_terms.append(back)
                    t += 1
                    ctx = e["ctx"]
                    hidden_states.append(h_t)
                    rewards.append(s["reward"])
                    masks.append(s["mask"])
                plan = nxt
        else:
            self.encoder.cache_language(not self.encoder.training, steps=self.episode_len, rows=batch_size)
            for t in range(self.episode_len):
                # host-side inputs of the step's loss/action stage, copied up front without a sync (the
                # reference builds them after the decoder with blocking copies; same values)
                target_np = self._teacher_action_np(perm_obs, ended)
                target = self._to_dev(target_np)
                if self._graph_step_ok(t, consistent_drop, noise, speaker):
                    candidate_leng, (h_t, c_t, logit, h1, ce, lpa, a_t) = self._graph_step(
                        perm_obs, target, h_t, h1, c_t, *enc_args[:3], ctx_mask)
                    hidden_states.append(h_t)
                    forth_terms.append(ce)
                    policy_log_probs.append(lpa.unsqueeze(1))
                    cpu_a_t = a_t.cpu().numpy().copy()      # the step's one device->host sync
                    for i, next_id in enumerate(cpu_a_t):
                        if next_id == (candidate_leng[i] - 1) or next_id == args.ignoreid:
                            cpu_a_t[i] = -1
                    self.make_equiv_action(cpu_a_t, perm_obs, perm_idx, traj)
                    obs = np.array(self.env._get_obs())
                    perm_obs = obs[perm_idx]
                    reward, mask = self._step_reward(perm_obs, cpu_a_t, ended, last_dist)
                    rewards.append(reward)
                    masks.append(mask)
                    ended[:] = np.logical_or(ended, (cpu_a_t == -1))
                    if ended.all():
                        break
                    continue
                mode = self._head_mode()
                forced_fn = None
                if mode == "forced":
                    forced_fn = (lambda leng, t=t: self._to_dev(
                        np.asarray(self.force_action_fn(t, list(leng)), np.int64)))
                back = None
                if self._step_region_ok(consistent_drop, noise):
                    # AdaIN + decoder + one-kernel policy head replayed as one captured training region
                    candidate_leng, ctx, h_t, c_t, logit, h1, ce, ent, lpa, a_dev = self._adain_decode(
                        t, mode, self._step_inputs([perm_obs]), *enc_args, h_t, h1, c_t, ctx_mask, target, forced_fn)
                else:
                    (e,) = self._encode_steps([perm_obs], *enc_args)
                    candidate_leng, ctx = e["leng"], e["ctx"]
                    self._fused_head(e["cand"][:, :, 0])
                    h0, c0 = (e["en_ht"], e["en_ct"]) if t == 0 else (h_t, c_t)
                    extra = self._visited_mask(perm_obs, visited, e["cand"].shape[1]) if args.submit else None
                    back_target = self._back_teacher_action(perm_obs, ended) if args.pred_back else None
                    h_t, c_t, logit, h1, ce, ent, lpa, a_dev, back = self._decode(
                        t, mode, e, h0, h0 if t == 0 else h1, c0, ctx_mask, self._lens_dev(candidate_leng), target,
                        forced_fn(candidate_leng) if forced_fn is not None else None, consistent_drop, extra,
                        back_target)
                hidden_states.append(h_t)
                forth_terms.append(ce)          # mask + CE + action + entropy / log-prob: one kernel (policy.hip)
                if back is not None:
                    back_terms.append(back)
                if self.feedback == "argmax":
                    a_t = a_dev
                    policy_log_probs.append(lpa.unsqueeze(1))
                elif self.feedback == "sample":
                    ent_terms.append(ent.detach())
                    entropys.append(ent)
                    a_t = a_dev
                    policy_log_probs.append(lpa)
                else:
                    a_t = target
                if self.feedback == "teacher":
                    cpu_a_t = target_np.copy()           # a_t is target: its host copy, no device round trip
                else:
                    cpu_a_t = a_t.cpu().numpy().copy()  # the step's one device->host sync
                for i, next_id in enumerate(cpu_a_t):
                    if next_id == (candidate_leng[i] - 1) or next_id == args.ignoreid:
                        cpu_a_t[i] = -1
                self.make_equiv_action(cpu_a_t, perm_obs, perm_idx, traj)
                obs = np.array(self.env._get_obs())
                perm_obs = obs[perm_idx]
                reward, mask = self._step_reward(perm_obs, cpu_a_t, ended, last_dist)
                rewards.append(reward)
                masks.append(mask)
                ended[:] = np.logical_or(ended, (cpu_a_t == -1))
                if ended.all():
                    break

        if train_rl:
            input_a_t, f_t, d_t, candidate_feat, candidate_dfeat, candidate_leng = self.get_input_feat(perm_obs)
            # (the reference also builds this step's teacher target and candidate mask, agent_dg.py:945-950;
            # nothing reads them)
            if speaker is not None:
                candidate_feat = self._noise_mult(candidate_feat, noise)
                f_t = self._noise_mult(f_t, noise)
            last_h_, _, _, _, _ = self.decoder(input_a_t, f_t, candidate_feat, h_t, h1, c_t, ctx, ctx_mask,
                                               speaker is not None)
            last_value__ = self.critic(last_h_).detach().view(-1).cpu().numpy()
            discount_reward = np.zeros(batch_size, np.float32)
            for i in range(batch_size):
                if not ended[i]:
                    discount_reward[i] = last_value__[i]
            # agent_dg.py:955-993 for all steps at once: the discounted returns are accumulated on the
            # host (same recursion), the critic runs once over the [T*B, 1024] stack of step states
            # (its dropout draws stay independent per element), and the per-step loss terms are
            # vectors over T summed in the reference's (reverse-step) order.
            length = len(rewards)
            R = np.zeros((length, batch_size), np.float32)
            for t in range(length - 1, -1, -1):
                discount_reward = discount_reward * args.gamma + rewards[t]
                R[t] = discount_reward
            Mk = np.stack(masks).astype(np.float32)
            rm = self._to_dev(np.stack((R, Mk)))
            r_, mask_ = rm[0], rm[1]
            H = torch.stack(hidden_states)
            v_ = self.critic(H.view(length * batch_size, -1)).view(length, batch_size)
            a_ = (r_ - v_).detach()
            lp = torch.stack([p.view(-1) for p in policy_log_probs])
            sq = ((r_ - v_) ** 2) * mask_
            terms = (-lp * a_ * mask_).sum(1) + sq.sum(1) * 0.5
            if self.feedback == "sample":
                terms = terms + (-0.01 * torch.stack(entropys) * mask_).sum(1)
            rl_loss = terms.flip(0).sum()
            deferred["critic_loss"].extend(sq.sum(1).detach().flip(0).unbind(0))
            total = float(Mk.sum())
            self.logs["total"].append(total)
            if args.normalize_loss == "total":
                rl_loss /= total
            elif args.normalize_loss == "batch":
                rl_loss /= batch_size
            else:
                assert args.normalize_loss == "none"
            self.loss += rl_loss
            deferred["normalized_rl_loss"].append(rl_loss.detach())

        if ent_terms:      # the per-step entropy logs (agent_dg.py:916): row sums of the [T, B] stack, one GEMM
            deferred["entropy"] = list(DF.row_sums(torch.stack(ent_terms)).unbind(0)) + deferred["entropy"]
        total_forth_loss = DF.sum_terms(forth_terms) if forth_terms else 0.0
        total_back_loss = DF.sum_terms(back_terms) if back_terms else 0.0
        ml_loss += total_forth_loss
        deferred["forth_loss"].append(total_forth_loss.detach())
        if args.pred_back:
            ml_loss += args.back_weight * total_back_loss
            deferred["back_loss"].append(args.back_weight * total_back_loss.detach())
        self.logs["viewsteps/{}".format(self.feedback)].append(len(rewards))
        if train_ml is not None:
            self.loss += ml_loss * train_ml / batch_size
            deferred["normalized_supervised_loss"].append((ml_loss * train_ml / batch_size).detach())
        deferred["ml_loss"].append(ml_loss.detach())
        # flush the deferred scalars with one host sync, in the reference's key order
        keys = [k for k in ("entropy", "critic_loss", "total", "normalized_rl_loss", "forth_loss", "back_loss",
                            "normalized_supervised_loss", "ml_loss") if k in deferred]
        flat = [v for k in keys for v in deferred[k]]
        if flat:
            vals = torch.stack([v.float().reshape(()) for v in flat]).cpu().tolist()
            i = 0
            for k in keys:
                for _ in deferred[k]:
                    self.logs[k].append(vals[i])
                    i += 1
        ops.check_device_errors()     # a persistent-kernel failure since the last check raises here
        if type(self.loss) is int:
            self.losses.append(0.0)
        else:
            self.losses.append(float(self.loss.item()) / self.episode_len)
        self.last_rollout_steps = len(rewards)
        return traj

    # ------------------------------------------------------------------ training API
    def test(self, use_dropout=False, feedback="argmax", allow_cheat=False, iters=None):
        self.feedback = feedback
        for m in (self.encoder, self.decoder, self.critic):
            m.train() if use_dropout else m.eval()
        with torch.no_grad():
            super().test(iters)

    def zero_grad(self):
        self.loss = 0.0
        self.losses = []
        if self._train_graphs is not None:
            self._train_graphs.new_iteration()
        self.encoder.bert.train_graphs_new_iteration()
        for m, opt in zip(self.models, self.optimizers):
            m.train()
            opt.zero_grad()

    def accumulate_gradient(self, feedback="teacher", **kwargs):
        """agent_dg.py:1347-1384."""
        if args.schedule_ratio == -1:
            if feedback == "teacher":
                self.feedback = "teacher"
                self.vl_rollout(train_ml=args.teacher_weight, train_rl=False, **kwargs)
            elif feedback == "sample":
                self.feedback = "teacher"
                self.vl_rollout(train_ml=args.ml_weight, train_rl=False, **kwargs)
                self.feedback = "sample"
                self.vl_rollout(train_ml=None, train_rl=True, **kwargs)
            else:
                assert False
        else:
            feedback = random.choices(["sample", "teacher"], [args.schedule_ratio, 1 - args.schedule_ratio], k=1)[0]
            if feedback == "teacher":
                self.feedback = "teacher"
                self.vl_rollout(train_ml=args.teacher_weight, train_rl=False, **kwargs)
            else:
                self.feedback = "sample"
                self.vl_rollout(train_ml=None, train_rl=True, **kwargs)

    def optim_step(self, **kwargs):
        """agent_dg.py:1389-1405 (+ data-parallel gradient all-reduce before clipping)."""
        # the encoder's per-step bi-LSTM BPTTs and the per-step decoder / critic weight gradients run
        # batched after the backward pass (dasa_amd/functional.py). When the bi-LSTM's input trains (the
        # language stack updates: --d_update_add_layer / --d_transformer_update, cfg4's finetune) its input
        # gradients come from the batched recurrence too and the backward continues from there, so the
        # first pass keeps its graph for that second one
        bert = self.encoder.bert
        dx = bool(getattr(bert, "update_add_layer", False) or getattr(bert, "update_lang_bert", False))
        dx = dx and os.environ.get("DASA_BPTT_DX", "0") == "1"       # off by default: measured slower (DESIGN r05)
        with DF.defer_bilstm_backward(input_grads=dx), DF.defer_weight_grads():
            self.loss.backward(retain_graph=dx)
            DF.flush_bilstm_backward()
        DF.flush_weight_grads()
        if self._train_graphs is not None:
            self._train_graphs.new_iteration()     # every replayed step has had its backward
        self.encoder.bert.train_graphs_new_iteration()
        # every kernel with a bounded inter-workgroup barrier (persistent bi-LSTM BPTT, D-split attention
        # backward) NaN-poisons its outputs and sets an error bit when the barrier times out: read the
        # error word (one host sync) before the gradients reach grad_sync, clipping and the optimizers;
        # the data-parallel mask all-reduce is enqueued first, so that one sync covers its host read too
        prep = getattr(self.grad_sync, "prepare", None)
        if prep is not None:
            prep()
        ops.check_device_errors()
        if self.grad_sync is not None:
            self.grad_sync()
        torch.nn.utils.clip_grad_norm_(self.encoder.parameters(), 40.0)
        torch.nn.utils.clip_grad_norm_(self.decoder.parameters(), 40.0)
        self.encoder_optimizer.step()
        self.decoder_optimizer.step()
        self.critic_optimizer.step()
        if args.adaIn_type not in ("default", "none"):
            self.adaIn_optimizer.step()
        if args.use_lr_scheduler:
            self.decoder_lr_scheduler.step()
            self.critic_lr_scheduler.step()
            if args.adaIn_type not in ("default", "none"):
                self.adaIn_lr_scheduler.step()

    def train(self, n_iters, feedback="teacher", **kwargs):
        """agent_dg.py:1407-1464."""
        self.feedback = feedback
        for m in (self.encoder, self.decoder, self.critic):
            m.train()
        self.losses = []
        for _ in range(1, n_iters + 1):
            self.encoder_optimizer.zero_grad()
            self.decoder_optimizer.zero_grad()
            self.critic_optimizer.zero_grad()
            self.loss = 0
            if args.schedule_ratio == -1:
                if feedback == "teacher":
                    self.feedback = "teacher"
                    self.vl_rollout(train_ml=args.teacher_weight, train_rl=False, **kwargs)
                elif feedback == "sample":
                    if args.ml_weight != 0:
                        self.feedback = "teacher"
                        self.vl_rollout(train_ml=args.ml_weight, train_rl=False, **kwargs)
                    self.feedback = "sample"
                    self.vl_rollout(train_ml=None, train_rl=True, **kwargs)
                else:
                    assert False
            else:
                fb = random.choices(["sample", "teacher"], [args.schedule_ratio, 1 - args.schedule_ratio], k=1)[0]
                self.feedback = fb
                self.vl_rollout(train_ml=args.teacher_weight if fb == "teacher" else None, train_rl=fb == "sample",
                                **kwargs)
            self.optim_step()

    def save(self, epoch, path):
        """agent_dg.py:1466-1487 (same checkpoint schema)."""
        the_dir, _ = os.path.split(path)
        if the_dir:
            os.makedirs(the_dir, exist_ok=True)
        states = {}
        items = [("encoder", self.encoder, self.encoder_optimizer), ("decoder", self.decoder, self.decoder_optimizer),
                 ("critic", self.critic, self.critic_optimizer)]
        if args.adaIn_type not in ("default", "none"):
            items.append(("adaIn", self.adaIn, self.adaIn_optimizer))
        for name, m, opt in items:
            states[name] = {"epoch": epoch + 1, "state_dict": m.state_dict(), "optimizer": opt.state_dict()}
        torch.save(states, path)

    def load(self, path):
        """agent_dg.py:1489-1510."""
        states = torch.load(path, map_location=self.device, weights_only=True)

        def recover_state(name, m, opt):
            state = m.state_dict()
            if set(state.keys()) != set(states[name]["state_dict"].keys()):
                print("NOTICE: DIFFERENT KEYS IN THE LISTEREN")
            state.update(states[name]["state_dict"])
            m.load_state_dict(state)
            if args.loadOptim:
                opt.load_state_dict(states[name]["optimizer"])
        items = [("encoder", self.encoder, self.encoder_optimizer), ("decoder", self.decoder, self.decoder_optimizer),
                 ("critic", self.critic, self.critic_optimizer)]
        if args.adaIn_type not in ("default", "none"):
            items.append(("adaIn", self.adaIn, self.adaIn_optimizer))
        for it in items:
            recover_state(*it)
        return states["encoder"]["epoch"] - 1
