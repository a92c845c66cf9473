"""Diagnosis: cfg2_full [record_logits] after a given precondition (r04: it failed only after the
train-graph tests). python tools/diag_order.py <seed|graph|none>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_train_parity_gpu as T  # noqa: E402


class _MP:
    def setenv(self, k, v):
        os.environ[k] = v


def main():
    what = sys.argv[1]
    dev = torch.device("cuda:0")
    if what == "seed":
        torch.manual_seed(3)
    elif what == "graph":
        from tests import test_train_graph_gpu as G
        G.test_train_graph_matches_eager(dev, _MP())
        os.environ.pop("DASA_TRAIN_GRAPH", None)
    elif what == "graph_eager":
        from tests import test_train_graph_gpu as G
        os.environ["DASA_TRAIN_GRAPH"] = "0"
        torch.manual_seed(3)
        ag = G._agent(700)
        for it in range(2):
            G._iteration(ag, it)
        del ag
        os.environ.pop("DASA_TRAIN_GRAPH", None)
    gen = T.R._get_wrapped_function()(dev)
    R = next(gen)
    try:
        T.test_cfg2_full_length_iteration(R, dev, True)
        print(what, "PASS", flush=True)
    except AssertionError as e:
        print(what, "FAIL", str(e)[:200], flush=True)


if __name__ == "__main__":
    main()
