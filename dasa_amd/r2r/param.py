"""The global `args` namespace of the reference (r2r_src/param.py:18-215), restated as a flag table.

Same flag names, destinations and defaults, so train.py and the policy modules read the same
attributes. Differences by design:
  * importing this module does NOT parse sys.argv (the reference parses at import, param.py:214);
    `parse(argv)` does, and dasa_amd.launch calls it for drop-in runs of train.py;
  * no snap/<name> directory is created at import (param.py:252-256) — `parse(..., make_dirs=True)` does.
`README_TRAIN_FLAGS` is the README "train" command line (README.md:82-96) without data/speaker paths.
"""
import argparse
import os

import torch


def _str2boolish(v):
    # the reference declares these `type=bool`: any non-empty string is True (param.py:101,109-125)
    return bool(v)


# (flag, dest, type, default); type 'const' = store_const True
_FLAGS = [
    ("--iters", None, int, 100000), ("--name", None, str, "default"), ("--train", None, str, "speaker"),
    ("--maxInput", None, int, 80), ("--maxDecode", None, int, 120), ("--maxAction", None, int, 20),
    ("--batchSize", None, int, 64), ("--ignoreid", None, int, -100), ("--feature_size", None, int, 2048),
    ("--loadOptim", None, "const", False), ("--speaker", None, str, None), ("--listener", None, str, None),
    ("--load", None, str, None), ("--aug", None, str, None), ("--pred_back", "pred_back", "const", False),
    ("--back_input", "back_input", str, "pre"), ("--use_action_seq", "use_action_seq", "const", False),
    ("--pred_pm", "pred_pm", "const", False), ("--pm_type", "pm_type", str, "att"),
    ("--zeroInit", "zero_init", "const", False), ("--mlWeight", "ml_weight", float, 0.05),
    ("--mlWeight_org", "ml_weight_org", float, 0.2), ("--mlWeight_aug", "ml_weight_aug", float, 0.6),
    ("--teacherWeight", "teacher_weight", float, 1.0), ("--accumulateGrad", "accumulate_grad", "const", False),
    ("--features", None, str, "imagenet"), ("--dfeatures", None, str, "imagenet"),
    ("--featdropout", None, float, 0.3), ("--selfTrain", "self_train", "const", False),
    ("--candidates", None, int, 1), ("--paramSearch", "param_search", "const", False),
    ("--submit", None, "const", False), ("--beam", None, "const", False), ("--alpha", None, float, 0.5),
    ("--optim", None, str, "rms"), ("--lr", None, float, 0.0001), ("--decay", "weight_decay", float, 0.0),
    ("--dropout", None, float, 0.5), ("--feedback", None, str, "sample"), ("--teacher", None, str, "final"),
    ("--epsilon", None, float, 0.1), ("--use_lr_scheduler", "use_lr_scheduler", "const", False),
    ("--rnnDim", "rnn_dim", int, 512), ("--critic_dim", "critic_dim", int, 512), ("--wemb", None, int, 256),
    ("--aemb", None, int, 64), ("--proj", None, int, 512), ("--fast", "fast_train", "const", False),
    ("--valid", None, "const", False), ("--candidate", "candidate_mask", "const", False),
    ("--bidir", None, bool, True), ("--encode", None, str, "word"), ("--subout", "sub_out", str, "tanh"),
    ("--attn", None, str, "soft"), ("--angleFeatSize", "angle_feat_size", int, 4),
    ("--philly", None, bool, False), ("--update_bert", None, bool, False),
    ("--include_vision", None, bool, False), ("--use_dropout_vision", None, bool, False),
    ("--encoderType", None, str, "EncoderLSTM"), ("--schedule_ratio", None, float, -1),
    ("--d_hidden_size", "d_hidden_size", int, 1024), ("--d_ctx_size", "d_ctx_size", int, 2048),
    ("--d_enc_hidden_size", "d_enc_hidden_size", int, 768), ("--d_dropout_ratio", "d_dropout_ratio", float, 0.4),
    ("--d_bidirectional", "d_bidirectional", bool, True), ("--d_transformer_update", "d_transformer_update", bool, False),
    ("--d_update_add_layer", "d_update_add_layer", bool, False), ("--d_bert_n_layers", "d_bert_n_layers", int, 1),
    ("--d_reverse_input", "d_reverse_input", bool, True), ("--d_top_lstm", "d_top_lstm", bool, True),
    ("--d_vl_layers", "d_vl_layers", int, 4), ("--d_la_layers", "d_la_layers", int, 9),
    ("--d_v_layers", "d_v_layers", int, 0), ("--d_bert_type", "d_bert_type", str, "small"),
    ("--pretrain_model_name", "pretrain_model_name", str, None),
    ("--pretrain_model_type", None, str, "DicAddActionPreTrain"), ("--log_every", None, int, 100),
    ("--warm_steps", None, int, 1000), ("--decay_start", None, int, 4000), ("--decay_intervals", None, int, 2000),
    ("--lr_decay", None, float, 0.2), ("--val_every", None, int, 1000), ("--save_every", None, int, 5000),
    ("--is_test", None, bool, False), ("--gamma", None, float, 0.9), ("--normalize", "normalize_loss", str, "total"),
    ("--mini", None, "const", False), ("--agent_type", "agent_type", str, "default"),
    ("--backward_inrollout", None, "const", False), ("--layer", "LAYER", int, 2),
    ("--word_mask_rate", None, float, 0.15), ("--tasks", None, str, "lmask"), ("--lmask_weight", None, float, 1.0),
    ("--action_weight", None, float, 1.0), ("--pm_weight", None, float, 1.0), ("--back_weight", None, float, 1.0),
    ("--depth_index_file", None, str, "data/viewpointIds.npy"),
    ("--depth_value_file", None, str, "data/ResNet-152-imagenet-depth.npy"),
    ("--adaIn_type", None, str, "none"), ("--ab_type", None, str, "ab"), ("--a_type", None, str, None),
    ("--decoder_type", None, str, "advanced"), ("--env_drop_stage", None, str, "after_adain"),
    ("--depth_drop", None, "const", False), ("--use_shift", None, "const", False),
    ("--shift_kernel_size", None, int, 3), ("--consistent_drop", None, "const", False),
    ("--decoder_consistent_drop", None, "const", False), ("--ctx_v", None, "const", False),
    # not a reference flag: compute the detached language stack once per rollout in train
    # mode too (one dropout draw per rollout instead of one per step). Off = the reference's per-step
    # recompute; no gradient changes either way (vilmodel.py:1377-1378 detaches the stack).
    ("--hoist_language", None, "const", False),
]

README_TRAIN_FLAGS = [
    "--agent_type", "dg", "--adaIn_type", "channel", "--attn", "soft", "--train", "auglistener",
    "--mlWeight_org", "0.4", "--mlWeight_aug", "1.2", "--ab_type", "a", "--a_type", "sigmoid",
    "--d_vl_layers", "3", "--env_drop_stage", "after_adain", "--depth_drop", "--use_shift",
    "--shift_kernel_size", "5", "--warm_steps", "1000", "--decay_intervals", "2000", "--decay_start", "4000",
    "--lr_decay", "0.2", "--log_every", "100", "--val_every", "2000", "--use_lr_scheduler",
    "--angleFeatSize", "128", "--accumulateGrad", "--featdropout", "0.4", "--feedback", "sample",
    "--subout", "max", "--optim", "rms", "--lr", "0.0001", "--iters", "20000", "--maxAction", "35",
    "--encoderType", "Dic", "--batchSize", "20", "--include_vision", "True", "--use_dropout_vision", "True",
    "--d_enc_hidden_size", "1024", "--critic_dim", "1024", "--name", "dasa_amd",
]


# README "finetune" command line (README.md:104-116) without data / speaker / load paths: the train
# flags with --d_update_add_layer True, lr 2e-6, batch 2 and no --use_lr_scheduler
README_FINETUNE_FLAGS = [f for f in README_TRAIN_FLAGS if f != "--use_lr_scheduler"]
for _flag, _val in (("--lr", "0.000002"), ("--batchSize", "2"), ("--iters", "30000"), ("--val_every", "1000")):
    README_FINETUNE_FLAGS[README_FINETUNE_FLAGS.index(_flag) + 1] = _val
README_FINETUNE_FLAGS += ["--d_update_add_layer", "True"]


def make_parser():
    p = argparse.ArgumentParser(description="DASA agent_dg (MI355X build)")
    for flag, dest, typ, default in _FLAGS:
        kw = {} if dest is None else {"dest": dest}
        if typ == "const":
            p.add_argument(flag, action="store_const", default=default, const=True, **kw)
        elif typ is bool:
            p.add_argument(flag, type=_str2boolish, default=default, **kw)
        else:
            p.add_argument(flag, type=typ, default=default, **kw)
    return p


_OPTIMIZERS = {"rms": torch.optim.RMSprop, "adam": torch.optim.Adam, "sgd": torch.optim.SGD}


def _finish(ns, make_dirs=False):
    if ns.optim not in _OPTIMIZERS:
        raise ValueError("unknown --optim %r" % ns.optim)
    ns.optimizer = _OPTIMIZERS[ns.optim]
    ns.TRAIN_VOCAB = "tasks/R2R/data/train_vocab.txt"
    ns.TRAINVAL_VOCAB = "tasks/R2R/data/trainval_vocab.txt"
    ns.IMAGENET_FEATURES = "img_features/ResNet-152-imagenet.tsv"
    ns.CANDIDATE_FEATURES = "img_features/ResNet-152-candidate.tsv"
    ns.features_fast = "img_features/ResNet-152-imagenet-fast.tsv"
    ns.log_dir = "snap/%s" % ns.name
    ns.views = 36
    if make_dirs:
        os.makedirs(ns.log_dir, exist_ok=True)
    return ns


args = _finish(make_parser().parse_args([]))


def parse(argv, make_dirs=False):
    """Re-parse `argv` into the shared `args` object (in place, so importers keep their reference)."""
    ns = _finish(make_parser().parse_args(list(argv)), make_dirs)
    args.__dict__.clear()
    args.__dict__.update(vars(ns))
    return args


def readme_train(extra=()):
    """args for the README training configuration (optionally overridden by `extra` flags)."""
    return parse(README_TRAIN_FLAGS + list(extra))


def readme_finetune(extra=()):
    """args for the README finetune configuration (configs[3] per rank)."""
    return parse(README_FINETUNE_FLAGS + list(extra))
