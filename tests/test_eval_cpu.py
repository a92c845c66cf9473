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


def test_unreachable_viewpoint_raises():
    """Two components (a-b, c-d): the reference's networkx distance dict has no a->c entry and raises
    KeyError (eval.py:47-52); the restatement raises too instead of scoring an infinite distance."""
    import pytest
    from dasa_amd.r2r.eval import NavGraph

    def vp(name, x, conn):
        pose = [0.0] * 16
        pose[3] = x
        return {"image_id": name, "pose": pose, "included": True, "unobstructed": conn}
    g = NavGraph([vp("a", 0.0, [False, True, False, False]), vp("b", 1.0, [True, False, False, False]),
                  vp("c", 5.0, [False, False, False, True]), vp("d", 7.0, [False, False, True, False])])
    assert g.distance("a", "b") == 1.0 and g.distance("c", "d") == 2.0
    with pytest.raises(KeyError):
        g.distance("a", "c")
