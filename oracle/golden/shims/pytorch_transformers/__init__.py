"""Offline stand-in for pytorch_transformers (absent, unpinned): only what r2r_src imports.

BertConfig carries bert-base-uncased hyper-parameters built locally (the name-based download in
BertConfig.from_pretrained cannot run offline). BertPreTrainedModel supplies `config` and the
standard BERT init (normal(0, initializer_range) for Linear/Embedding, zero bias, LN = 1/0); the
golden generator overwrites every weight with seeded values afterwards anyway.
"""
import copy

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

    @classmethod
    def from_pretrained(cls, *a, **k):
        raise RuntimeError("pretrained checkpoints are unavailable offline")
