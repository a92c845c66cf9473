"""pytorch_transformers.modeling_bert.BertOnlyMLMHead (the masked-LM pretraining head that
r2rpretrain_class.py builds), restated from its published architecture: transform (dense H->H, gelu,
LayerNorm eps 1e-12) then a decoder H->vocab without bias plus a separate bias vector. Only its
state_dict layout matters here (--pretrain_model_name drops the head when it takes `.bert`)."""
import math

import torch
from torch import nn


def _gelu(x):
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


class BertPredictionHeadTransform(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)

    def forward(self, x):
        return self.LayerNorm(_gelu(self.dense(x)))


class BertLMPredictionHead(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.transform = BertPredictionHeadTransform(config)
        self.decoder = nn.Linear(config.hidden_size, config.vocab_size, bias=False)
        self.bias = nn.Parameter(torch.zeros(config.vocab_size))

    def forward(self, x):
        return self.decoder(self.transform(x)) + self.bias


class BertOnlyMLMHead(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.predictions = BertLMPredictionHead(config)

    def forward(self, sequence_output):
        return self.predictions(sequence_output)
