"""Offline stand-in for pytorch_transformers (absent, unpinned): only what r2r_src imports.

BertConfig carries bert-base-uncased hyper-parameters built locally (the name-based download in
BertConfig.from_pretrained cannot run offline). BertPreTrainedModel supplies `config` and the
standard BERT init (normal(0, initializer_range) for Linear/Embedding, zero bias, LN = 1/0); the
golden generator overwrites every weight with seeded values afterwards anyway.
"""
import copy
import json
import os

import torch
from torch import nn

_BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
             intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
             attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
             initializer_range=0.02, layer_norm_eps=1e-12, output_attentions=False,
             output_hidden_states=False, torchscript=False, num_labels=2)
_LARGE = dict(_BASE, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)


class BertConfig:
    def __init__(self, **kw):
        for k, v in _BASE.items():
            setattr(self, k, v)
        for k, v in kw.items():
            setattr(self, k, v)

    @classmethod
    def from_pretrained(cls, name, **kw):
        base = _LARGE if "large" in str(name) else _BASE
        return cls(**dict(base, **kw))

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n"

    @classmethod
    def from_json_file(cls, path):
        with open(path) as f:
            return cls(**json.load(f))

    def __repr__(self):
        return "BertConfig(%r)" % (self.__dict__,)


class BertPreTrainedModel(nn.Module):
    config_class = BertConfig
    base_model_prefix = "bert"

    def __init__(self, config, *inputs, **kwargs):
        super().__init__()
        self.config = config

    def _init_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(mean=0.0, std=self.config.initializer_range)
        elif isinstance(module, nn.LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def init_weights(self):
        self.apply(self._init_weights)

    def _tie_or_clone_weights(self, first_module, second_module):
        """pytorch_transformers 1.x: the output embedding shares the input embedding's weight."""
        first_module.weight = second_module.weight

    @classmethod
    def from_pretrained(cls, path, *a, **k):
        """pytorch_transformers 1.x PreTrainedModel.from_pretrained restated for a LOCAL directory (the
        name-based hub download is unavailable offline): config.json -> cls(config) -> non-strict load
        of pytorch_model.bin (base_model_prefix handling; missing / unexpected keys are reported, not
        raised) -> tie_weights -> eval()."""
        if not os.path.isdir(path):
            raise RuntimeError("pretrained checkpoints are unavailable offline (only a local directory loads)")
        config = cls.config_class.from_json_file(os.path.join(path, "config.json"))
        model = cls(config)
        state_dict = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
        renames = {}
        for key in state_dict:      # TF-style LayerNorm names
            if "gamma" in key:
                renames[key] = key.replace("gamma", "weight")
            if "beta" in key:
                renames[key] = key.replace("beta", "bias")
        for old, new in renames.items():
            state_dict[new] = state_dict.pop(old)
        missing, unexpected, errors = [], [], []
        metadata = getattr(state_dict, "_metadata", None)
        state_dict = state_dict.copy()
        if metadata is not None:
            state_dict._metadata = metadata

        def load(module, prefix=""):
            local_metadata = {} if metadata is None else metadata.get(prefix[:-1], {})
            module._load_from_state_dict(state_dict, prefix, local_metadata, True, missing, unexpected, errors)
            for name, child in module._modules.items():
                if child is not None:
                    load(child, prefix + name + ".")
        start_prefix = ""
        model_to_load = model
        if not hasattr(model, cls.base_model_prefix) and any(s.startswith(cls.base_model_prefix) for s in state_dict):
            start_prefix = cls.base_model_prefix + "."
        if hasattr(model, cls.base_model_prefix) and not any(s.startswith(cls.base_model_prefix) for s in state_dict):
            model_to_load = getattr(model, cls.base_model_prefix)
        load(model_to_load, prefix=start_prefix)
        if errors:
            raise RuntimeError("Error(s) in loading state_dict for %s:\n\t%s" % (cls.__name__, "\n\t".join(errors)))
        model.load_report = {"missing": missing, "unexpected": unexpected}
        if hasattr(model, "tie_weights"):
            model.tie_weights()
        model.eval()
        return model
