"""__graft_entry__.smoke(): one small policy rollout (cfg1 shape: B=2, vl=1, 5 steps, eval/argmax)
on cuda:0 through libdasa_hip.so, checked against the CPU oracle (test infrastructure)."""
import contextlib
import io

import torch


def run_smoke():
    assert torch.cuda.is_available(), "smoke() needs the MI355X"
    from dasa_amd import _lib
    _lib.lib()
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    from dasa_amd.synth import SynthR2RBatch, SynthWorld, init_params
    from oracle import policy as O
    from tests import golden_inputs as GI
    from tests.helpers import oracle_weights

    world = SynthWorld(16, 0, 3)
    env = SynthR2RBatch(world, 2, seed=7, mode="goal", instr_len=80, variable_len=True)
    with contextlib.redirect_stdout(io.StringIO()):
        ag = Seq2SeqAgent(env, "", None, 5, "Dic")
    for m, s in ((ag.encoder, GI.SEED_ENC), (ag.decoder, GI.SEED_DEC), (ag.critic, GI.SEED_CRITIC),
                 (ag.adaIn, GI.SEED_ADA)):
        init_params(m, s)
        m.eval()
    logits = []
    fwd = ag.decoder.forward

    def wrap(*a, **k):
        r = fwd(*a, **k)
        logits.append(r[2].detach().float().cpu())
        return r
    ag.decoder.forward = wrap
    ag.loss = 0
    ag.feedback = "argmax"
    with torch.no_grad():
        ag.vl_rollout(train_ml=None, train_rl=False, reset=True)
    env_ref = SynthR2RBatch(world, 2, seed=7, mode="goal", instr_len=80, variable_len=True)
    with torch.no_grad():
        ref = O.vl_rollout(oracle_weights(1), env_ref, "argmax", la_layers=9, vl_layers=1, episode_len=5)
    assert len(logits) == ref["steps"], (len(logits), ref["steps"])
    err = max((a - b).abs().max().item() for a, b in zip(logits, ref["logits"]))
    assert err < 1e-4, f"smoke: logits differ from the oracle by {err:.3e}"
    print(f"[smoke] {len(logits)} steps on {torch.cuda.get_device_name(0)}; max |logit - oracle| = {err:.2e}")
