"""--pretrain_model_name hand-off (agent_dg.py:165-188) on the host: dasa_amd.r2r.agent_dg.
load_pretrained_bert reads the checkpoint layouts the reference loads (a DicAddActionPreTrain
from_pretrained directory whose config.json fixes the VL depth; a DicPMActionPreTrain {'state_dict'}
file) and refuses anything else instead of loading it non-strictly. The layout (config + head keys) is
the one the reference wrote in tests/golden/pretrain.npz (oracle/golden/make_golden.py pretrain); the
GPU parity of the loaded model is tests/test_train_parity_gpu.py::test_pretrained_bert_handoff_vs_reference."""
import json

import pytest
import torch

from dasa_amd.synth import init_params
from tests import golden_inputs as GI
from tests.helpers import golden


@pytest.fixture(scope="module")
def mods():
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "3"])
    from dasa_amd.r2r import agent_dg, vilmodel
    return param, agent_dg, vilmodel


def _write(path, vilmodel, drop=None, extra=None):
    from tests.test_train_parity_gpu import write_pretrain_dir
    sd = write_pretrain_dir(str(path), vilmodel)
    if drop or extra:
        if drop:
            del sd[drop]
        if extra:
            sd[extra] = torch.zeros(3)
        torch.save(sd, str(path / "pytorch_model.bin"))
    return sd


def test_checkpoint_dir_decides_depth_and_weights(mods, tmp_path):
    _, agent_dg, vilmodel = mods
    sd = _write(tmp_path, vilmodel)
    bert = agent_dg.load_pretrained_bert(str(tmp_path), "DicAddActionPreTrain")
    assert len(bert.addlayer) == GI.CFG_PRE["vl_layers_ckpt"] == 2 and len(bert.lalayer) == 9
    for k, v in bert.state_dict().items():
        assert torch.equal(v, sd["bert." + k]), k
    heads = json.loads(str(golden("pretrain")["pre/head_schema"]))
    assert heads and all(k.startswith(("next_action.", "mlmhead.")) for k in heads)


def test_tf_style_layernorm_names_load(mods, tmp_path):
    """pytorch_transformers renames gamma / beta LayerNorm keys on load; so does the hand-off."""
    _, agent_dg, vilmodel = mods
    sd = _write(tmp_path, vilmodel)
    k = "bert.embeddings.LayerNorm.weight"
    sd["bert.embeddings.LayerNorm.gamma"] = sd.pop(k)
    torch.save(sd, str(tmp_path / "pytorch_model.bin"))
    bert = agent_dg.load_pretrained_bert(str(tmp_path))
    assert torch.equal(bert.embeddings.LayerNorm.weight, sd["bert.embeddings.LayerNorm.gamma"])


@pytest.mark.parametrize("bad", ["stray", "missing", "prefix"])
def test_bad_checkpoint_raises(mods, tmp_path, bad):
    from dasa_amd._lib import DasaError
    _, agent_dg, vilmodel = mods
    if bad == "stray":
        _write(tmp_path, vilmodel, extra="classifier.weight")          # not a DicAddActionPreTrain head
    elif bad == "missing":
        _write(tmp_path, vilmodel, drop="bert.addlayer.1.visn_output.dense.weight")
    else:      # a DicModel saved without the `bert.` prefix: every key is stray
        sd = _write(tmp_path, vilmodel)
        torch.save({k[len("bert."):]: v for k, v in sd.items() if k.startswith("bert.")},
                   str(tmp_path / "pytorch_model.bin"))
    with pytest.raises(DasaError):
        agent_dg.load_pretrained_bert(str(tmp_path), "DicAddActionPreTrain")


def test_pm_checkpoint_file_uses_command_line_depth(mods, tmp_path):
    """DicPMActionPreTrain (agent_dg.py:166-177): a {'state_dict': ...} file; bert-base with
    d_vl_layers / d_la_layers from args; its progress-monitor `critic.*` head is dropped too."""
    param, agent_dg, vilmodel = mods
    cfg = vilmodel.BertConfig(img_feature_dim=2176, img_feature_type="", update_lang_bert=True, update_add_layer=True,
                              vl_layers=param.args.d_vl_layers, la_layers=param.args.d_la_layers)
    bert = init_params(vilmodel.DicModel(cfg), 5)
    sd = {"bert." + k: v for k, v in bert.state_dict().items()}
    sd["critic.0.weight"] = torch.zeros(1, 80 + 768)
    sd["next_action.linear.weight"] = torch.zeros(36, 768)
    f = tmp_path / "pm.pt"
    torch.save({"state_dict": sd}, str(f))
    got = agent_dg.load_pretrained_bert(str(f), "DicPMActionPreTrain")
    assert len(got.addlayer) == param.args.d_vl_layers == 3
    assert all(torch.equal(v, sd["bert." + k]) for k, v in got.state_dict().items())
    with pytest.raises(Exception):
        agent_dg.load_pretrained_bert(str(f), "DicAddActionPreTrain")     # a file is not a from_pretrained dir
