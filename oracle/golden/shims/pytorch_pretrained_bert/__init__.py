"""Stub: r2rmodel.py imports these names; the hot path never instantiates them."""


class BertModel:
    pass


class OpenAIGPTModel:
    pass
