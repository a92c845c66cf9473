"""Stub: r2rpretrain_class.py imports BertOnlyMLMHead (pretraining head, off the hot path)."""
from torch import nn


class BertOnlyMLMHead(nn.Module):
    def __init__(self, config):
        super().__init__()
        raise RuntimeError("BertOnlyMLMHead is not available offline")
