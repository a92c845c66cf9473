"""Drop-in launcher: run the reference's r2r_src/train.py unchanged on the MI355X policy.

    python -m dasa_amd.launch /path/to/DASA/r2r_src/train.py --agent_type dg --adaIn_type channel ...

train.py does `from param import args`, `from agent_dg import Seq2SeqAgent`, and its helpers import
`model`, `vilmodel`, `r2rmodel`. This launcher binds those module names to dasa_amd.r2r (whose
classes, signatures, state_dict keys and args flags match the reference), parses the command line
into the shared `args` like param.py does at import, and executes train.py as __main__. In the
listener modes (the speaker only back-translates through `infer_batch`) the speaker module and its
model classes are ours as well; `--train speaker` / `validspeaker` / `all` train or validate the
speaker (train, valid, teacher_forcing, beam_search), which is outside the policy path, so there the
reference's `speaker` module and `model.SpeakerEncoder/SpeakerDecoder` are used unchanged. Everything
else (env, utils, eval, tokenizers, MatterSim) is the reference's own code. Names the policy modules do
not define (e.g. the alternative decoders) resolve to the reference's definitions, loaded under a
private module name.
"""
import importlib.util
import os
import runpy
import sys
import types


def _load_reference(name, path):
    spec = importlib.util.spec_from_file_location("_dasa_ref_" + name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


# train.py modes whose speaker only runs infer_batch (train.py:165-171, agent_dg.py:656-677)
SPEAKER_INFER_MODES = ("listener", "validlistener", "auglistener")
SPEAKER_NAMES = ("SpeakerEncoder", "SpeakerDecoder")


def _proxy(ours, ref_dir, name, exclude=()):
    """Module `name`: our definitions (minus `exclude`), falling back to the reference module for
    anything else."""
    px = types.ModuleType(name)
    px.__dict__.update({k: v for k, v in vars(ours).items() if not k.startswith("__") and k not in exclude})
    ref_path = os.path.join(ref_dir, name + ".py")
    state = {}

    def __getattr__(attr):
        if "ref" not in state:
            if not os.path.exists(ref_path):
                raise AttributeError(attr)
            state["ref"] = _load_reference(name, ref_path)
        return getattr(state["ref"], attr)
    px.__getattr__ = __getattr__
    px.__file__ = ours.__file__
    return px


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    script = os.path.abspath(argv[0])
    ref_dir = os.path.dirname(script)
    sys.argv = [script] + argv[1:]
    sys.path.insert(0, ref_dir)
    from dasa_amd.r2r import param
    param.parse(sys.argv[1:], make_dirs=True)
    sys.modules["param"] = param
    from dasa_amd.r2r import agent_dg, model, r2rmodel, speaker, vilmodel
    ours_speaker = param.args.train in SPEAKER_INFER_MODES
    binds = [("model", model), ("vilmodel", vilmodel), ("r2rmodel", r2rmodel), ("agent_dg", agent_dg)]
    if ours_speaker:
        binds.append(("speaker", speaker))
    for name, ours in binds:
        excl = SPEAKER_NAMES if (name == "model" and not ours_speaker) else ()
        sys.modules[name] = _proxy(ours, ref_dir, name, excl)
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
