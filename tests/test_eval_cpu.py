"""Evaluation.score (dasa_amd/r2r/eval.py) against the reference's own Evaluation (eval.py:17-108) on
the reference's connectivity graphs of three scans (copies in tests/golden/connectivity) for the
synthetic items / trajectories recorded in tests/golden/eval.npz (oracle/golden/make_golden.py eval):
every per-item score and the summary (nav error, oracle error, SR, oracle SR, SPL) within 1e-9."""
import json
import os

import numpy as np

from dasa_amd.r2r.eval import Evaluation
from tests.helpers import GOLDEN, golden


def test_evaluation_matches_reference():
    G = golden("eval")
    items = json.loads(str(G["eval/items"]))
    results = json.loads(str(G["eval/results"]))
    want_summary = json.loads(str(G["eval/summary"]))
    want_scores = json.loads(str(G["eval/scores"]))
    ev = Evaluation(["val_seen"], None, None, items=items, conn_dir=os.path.join(GOLDEN, "connectivity"))
    summary, scores = ev.score(results)
    assert set(summary) == set(want_summary)
    for k, v in want_summary.items():
        assert abs(float(summary[k]) - v) < 1e-9, (k, summary[k], v)
    assert set(scores) == set(want_scores)
    for k, v in want_scores.items():
        np.testing.assert_allclose(np.array(scores[k], np.float64), np.array(v), rtol=0, atol=1e-9, err_msg=k)
