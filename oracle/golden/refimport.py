"""Import the reference r2r_src policy modules in THIS container (CPU, fp32) behind offline shims.

Test infrastructure only: used by make_golden.py to produce tests/golden fixtures. Never imported by
dasa_amd, bench.py or anything that runs on the GPU box (/root/reference does not exist there).
"""
import os
import sys
import tempfile

REF_SRC = "/root/reference/r2r_src"
SHIMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shims")

# README "train" flags (README.md:82-96) minus the data/speaker/pretrained paths, plus cfg1 sizes.
README_TRAIN_FLAGS = [
    "--agent_type", "dg", "--adaIn_type", "channel", "--attn", "soft", "--train", "auglistener",
    "--mlWeight_org", "0.4", "--mlWeight_aug", "1.2", "--ab_type", "a", "--a_type", "sigmoid",
    "--d_vl_layers", "3", "--env_drop_stage", "after_adain", "--depth_drop", "--use_shift",
    "--shift_kernel_size", "5", "--warm_steps", "1000", "--decay_intervals", "2000", "--decay_start", "4000",
    "--lr_decay", "0.2", "--log_every", "100", "--val_every", "2000", "--use_lr_scheduler",
    "--angleFeatSize", "128", "--accumulateGrad", "--featdropout", "0.4", "--feedback", "sample",
    "--subout", "max", "--optim", "rms", "--lr", "0.0001", "--iters", "20000", "--maxAction", "35",
    "--encoderType", "Dic", "--batchSize", "20", "--include_vision", "True", "--use_dropout_vision", "True",
    "--d_enc_hidden_size", "1024", "--critic_dim", "1024", "--name", "golden",
]

_MODS = None


def import_reference(extra_argv=()):
    """Returns a namespace with the reference modules (param, utils, model, vilmodel, r2rmodel, agent_dg)."""
    global _MODS
    if _MODS is not None:
        return _MODS
    if not os.path.isdir(REF_SRC):
        raise RuntimeError("reference source not present (golden generation runs only in the survey container)")
    import torch
    sys.dont_write_bytecode = True
    sys.path[:0] = [SHIMS, REF_SRC]
    os.chdir(tempfile.mkdtemp(prefix="dasa_golden_"))   # param.py creates snap/<name> in the CWD
    argv_saved = sys.argv
    sys.argv = ["train.py"] + README_TRAIN_FLAGS + list(extra_argv)
    # device plumbing: the reference calls .cuda() everywhere; run it on the CPU.
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.Tensor.cuda = lambda self, *a, **k: self
    _cpu = torch.Tensor.cpu
    # a real D2H copy never aliases; without this agent_dg.py:890-893 corrupts a_t on CPU
    torch.Tensor.cpu = lambda self, *a, **k: _cpu(self, *a, **k).clone()
    import io, contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        import param  # noqa: F401
        import utils
        import model
        import vilmodel
        import r2rmodel
        import agent_dg
    sys.argv = argv_saved

    class NS:
        pass
    ns = NS()
    ns.param, ns.utils, ns.model, ns.vilmodel, ns.r2rmodel, ns.agent_dg = param, utils, model, vilmodel, r2rmodel, agent_dg
    ns.args = param.args
    _MODS = ns
    return ns
