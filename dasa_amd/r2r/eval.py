"""Evaluation of agent trajectories (r2r_src/eval.py:17-108, utils.load_nav_graphs utils.py:26-57),
restated for the drop-in package: navigation error, oracle error, success
rate, oracle success rate and SPL with the reference's 3 m margin.

The reference builds a networkx graph per scan and runs all-pairs Dijkstra in Python; here each scan's
connectivity becomes a sparse matrix over its included viewpoints and scipy's compiled Dijkstra fills a
dense distance matrix (same edge set and euclidean weights; shortest-path lengths equal to fp64
rounding). Host-side metric code: nothing of it is on the policy step.
"""
import json
import os
from collections import defaultdict

import numpy as np


class NavGraph:
    """One scan's navigation graph: included viewpoints with an unobstructed edge, euclidean edge
    weights from the pose translation (utils.py:29-33), all-pairs shortest-path lengths."""

    def __init__(self, data):
        def pos(item):
            return np.array([item["pose"][3], item["pose"][7], item["pose"][11]], np.float64)
        edges = []
        nodes = {}
        for i, item in enumerate(data):
            if not item["included"]:
                continue
            for j, conn in enumerate(item["unobstructed"]):
                if conn and data[j]["included"]:
                    assert data[j]["unobstructed"][i], "Graph should be undirected"
                    for vid in (item["image_id"], data[j]["image_id"]):
                        nodes.setdefault(vid, len(nodes))
                    edges.append((item["image_id"], data[j]["image_id"],
                                  float(np.sqrt(((pos(item) - pos(data[j])) ** 2).sum()))))
        self.ids = list(nodes)
        self.index = nodes
        n = len(nodes)
        from scipy.sparse import coo_matrix
        from scipy.sparse.csgraph import dijkstra
        und = {}                   # each undirected edge once (it is listed from both ends)
        for a, b, x in edges:
            ia, ib = nodes[a], nodes[b]
            und[(min(ia, ib), max(ia, ib))] = x
        r = [k[0] for k in und]
        c = [k[1] for k in und]
        w = list(und.values())
        adj = coo_matrix((w + w, (r + c, c + r)), shape=(n, n)).tocsr()
        self.dist = dijkstra(adj, directed=False)

    def distance(self, a, b):
        d = float(self.dist[self.index[a], self.index[b]])
        if not np.isfinite(d):   # networkx's all-pairs dict has no entry here: the reference raises KeyError
            raise KeyError("no path between %s and %s in the navigation graph" % (a, b))
        return d


def load_nav_graphs(scans, conn_dir="connectivity"):
    """utils.py:26-57: {scan: NavGraph} from <conn_dir>/<scan>_connectivity.json."""
    graphs = {}
    for scan in scans:
        with open(os.path.join(conn_dir, "%s_connectivity.json" % scan)) as f:
            graphs[scan] = NavGraph(json.load(f))
    return graphs


def load_datasets(splits, data_dir="tasks/R2R/data"):
    """utils.load_datasets: the R2R json of each split."""
    data = []
    for split in splits:
        with open(os.path.join(data_dir, "R2R_%s.json" % split)) as f:
            data += json.load(f)
    return data


class Evaluation(object):
    """eval.py:17-108. Results format: [{'instr_id': str, 'trajectory': [(viewpoint, heading, elevation)]}].
    `items` (the dataset entries) and `conn_dir` default to the reference's on-disk locations."""

    def __init__(self, splits, scans, tok, items=None, conn_dir="connectivity"):
        self.error_margin = 3.0
        self.splits = splits
        self.tok = tok
        self.gt = {}
        self.instr_ids = []
        self.scans = []
        for item in (items if items is not None else load_datasets(splits)):
            if scans is not None and item["scan"] not in scans:
                continue
            self.gt[str(item["path_id"])] = item
            self.scans.append(item["scan"])
            self.instr_ids += ["%s_%d" % (item["path_id"], i) for i in range(len(item["instructions"]))]
        self.scans = set(self.scans)
        self.instr_ids = set(self.instr_ids)
        self.graphs = load_nav_graphs(self.scans, conn_dir)

    def _dist(self, scan, a, b):
        return self.graphs[scan].distance(a, b)

    def _get_nearest(self, scan, goal_id, path):
        near_id = path[0][0]
        near_d = self._dist(scan, near_id, goal_id)
        for item in path:
            d = self._dist(scan, item[0], goal_id)
            if d < near_d:
                near_id, near_d = item[0], d
        return near_id

    def _score_item(self, instr_id, path):
        gt = self.gt[instr_id.split("_")[-2]]
        scan = gt["scan"]
        start, goal = gt["path"][0], gt["path"][-1]
        assert start == path[0][0], "Result trajectories should include the start position"
        final_position = path[-1][0]
        nearest_position = self._get_nearest(scan, goal, path)
        self.scores["nav_errors"].append(self._dist(scan, final_position, goal))
        self.scores["oracle_errors"].append(self._dist(scan, nearest_position, goal))
        self.scores["trajectory_steps"].append(len(path) - 1)
        distance = 0.0
        prev = path[0]
        for curr in path[1:]:
            distance += self._dist(scan, prev[0], curr[0])
            prev = curr
        self.scores["trajectory_lengths"].append(distance)
        self.scores["shortest_lengths"].append(self._dist(scan, start, goal))

    def score(self, output_file):
        self.scores = defaultdict(list)
        instr_ids = set(self.instr_ids)
        if isinstance(output_file, str):
            with open(output_file) as f:
                results = json.load(f)
        else:
            results = output_file
        for item in results:
            if item["instr_id"] in instr_ids:
                instr_ids.remove(item["instr_id"])
                self._score_item(item["instr_id"], item["trajectory"])
        if "train" not in self.splits:
            assert len(instr_ids) == 0, "Missing %d of %d instruction ids from %s - not in %s" % (
                len(instr_ids), len(self.instr_ids), ",".join(self.splits), output_file)
            assert len(self.scores["nav_errors"]) == len(self.instr_ids)
        s = self.scores
        summary = {"nav_error": np.average(s["nav_errors"]), "oracle_error": np.average(s["oracle_errors"]),
                   "steps": np.average(s["trajectory_steps"]), "lengths": np.average(s["trajectory_lengths"])}
        summary["success_rate"] = float(sum(e < self.error_margin for e in s["nav_errors"])) / len(s["nav_errors"])
        summary["oracle_rate"] = float(sum(e < self.error_margin for e in s["oracle_errors"])) / len(s["oracle_errors"])
        spl = [float(e < self.error_margin) * l / max(l, p, 0.01)
               for e, p, l in zip(s["nav_errors"], s["trajectory_lengths"], s["shortest_lengths"])]
        summary["spl"] = np.average(spl)
        return summary, self.scores
