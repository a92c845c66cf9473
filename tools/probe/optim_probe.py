"""Two cfg1 training iterations (forced draws, dropout 0) with optim_step: per-iteration losses / logs
and, after step 0, per-parameter norms of the parameter and of its change. Runs the product on the GPU
(default) or, with --reference in the survey container, the reference itself (CPU)."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np
import torch

from dasa_amd.synth import SynthR2RBatch, SynthWorld
from tests import golden_inputs as GI


def run(agent, cfg, sample_patch):
    out = {"it": []}
    mods = (("encoder", agent.encoder), ("decoder", agent.decoder), ("critic", agent.critic), ("adaIn", agent.adaIn))
    for it in range(2):
        table = GI.forced_table(cfg["max_action"], cfg["batch"], seed=GI.FORCED_SEED + it)
        sample_patch(agent, table)
        before = {f"{n}.{k}": p.detach().double().cpu().clone() for n, m in mods for k, p in m.named_parameters()}
        agent.zero_grad()
        agent.accumulate_gradient("sample")
        rec = {"loss": agent.loss.item(), "logs": {k: [float(x) for x in v[-6:]] for k, v in agent.logs.items()}}
        agent.optim_step()
        rec["delta"] = {}
        for n, m in mods:
            for k, p in m.named_parameters():
                d = p.detach().double().cpu() - before[f"{n}.{k}"]
                if d.abs().max() > 0:
                    rec["delta"][f"{n}.{k}"] = [float(d.norm()), float(p.detach().double().norm())]
        out["it"].append(rec)
    return out


def main():
    cfg = GI.CFG_OPTIM
    ref = "--reference" in sys.argv
    if ref:
        from oracle.golden.refimport import import_reference
        from oracle.golden import make_golden as MG
        R = import_reference()
        A = R.args
        A.d_vl_layers, A.batchSize, A.maxAction, A.views = cfg["vl_layers"], cfg["batch"], cfg["max_action"], 36
        A.ml_weight = A.ml_weight_org
        world = SynthWorld(16, 0, 3)
        env = SynthR2RBatch(world, cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80, variable_len=True)
        agent = MG.make_agent(R, env, cfg["max_action"])
        MG._zero_dropout(agent)

        def patch(ag, table):
            sample, install, _ = GI.reference_forced_sample(table, R.utils)
            install()
            torch.distributions.Categorical.sample = sample
    else:
        from dasa_amd.r2r import param
        param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
        param.args.ml_weight = param.args.ml_weight_org
        from tests.test_train_parity_gpu import _agent, _zero_dropout, _force
        from dasa_amd.r2r import agent_dg, model, r2rmodel, vilmodel
        Rm = (param, agent_dg, model, r2rmodel, vilmodel)
        env = SynthR2RBatch(SynthWorld(16, 0, 3), cfg["batch"], seed=cfg["env_seed"], mode="goal", instr_len=80,
                            variable_len=True)
        agent = _agent(Rm, env, cfg["max_action"])
        _zero_dropout(agent)

        def patch(ag, table):
            _force(ag, table)
    out = run(agent, cfg, patch)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
