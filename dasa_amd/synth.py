"""Deterministic synthetic data for the DASA policy path: weights, panoramas, instructions and an
R2R-compatible batch environment.

There is no network (no R2R json, no ResNet-152 TSVs, no depth .npy, no BERT checkpoint), so every
benchmark and parity test runs on these synthetic inputs:
  * features: a pool of P viewpoints, RGB and depth [36, 2048] float32 ~ U[0,1) (feature seed 0);
  * angles: the reference's 36-view angle table (utils.py:361-408), 128-d;
  * candidates: per viewpoint 1..15 neighbours, each seen from one of the 36 views;
  * tokens: [101, U{1000..29999} x (len-2), 102] padded with 0 (BERT ids);
  * weights: `init_params(module, seed)` — numpy default_rng(seed) normals in sorted state_dict order,
    so the reference modules (imported in the survey container) and ours receive identical weights.

`SynthR2RBatch` reproduces the observation contract of R2RBatch._get_obs (env.py:317-360) and the
discretized 36-view state machine of MatterSim (MatterSim.cpp:339-367, 470-490) that
Seq2SeqAgent.make_equiv_action drives (agent_dg.py:358-391).
"""
import math

import numpy as np

FEATURE_SIZE = 2048
ANGLE_FEAT_SIZE = 128
NUM_VIEWS = 36
HEADING_INC = math.pi / 6.0
ELEVATION_INC = math.pi / 6.0


# --------------------------------------------------------------------------------------- weights
def param_init_array(name, shape, rng):
    """The value a named parameter receives (consumes rng)."""
    base = rng.standard_normal(shape, dtype=np.float32)
    lname = name.lower()
    if lname.endswith("layernorm.weight") or lname.endswith("layer_norm.weight"):
        return 1.0 + 0.05 * base
    if lname.endswith("layernorm.bias") or lname.endswith("layer_norm.bias"):
        return 0.05 * base
    if lname.endswith("bias") or "bias_" in lname:
        return 0.02 * base
    return 0.02 * base


def init_param_dict(shapes, seed):
    """{key: shape} -> {key: float32 torch tensor}, identical to init_params on a module with that schema."""
    import torch
    rng = np.random.default_rng(seed)
    return {k: torch.from_numpy(np.ascontiguousarray(param_init_array(k, tuple(shapes[k]), rng)))
            for k in sorted(shapes.keys())}


def init_params(module, seed, skip_prefix=()):
    """Overwrite every parameter/buffer-free state entry of `module` deterministically (entries whose
    key starts with one of `skip_prefix` keep their values and draw nothing from the stream)."""
    import torch
    rng = np.random.default_rng(seed)
    sd = module.state_dict()
    new = {}
    for k in sorted(sd.keys()):
        v = sd[k]
        if not torch.is_floating_point(v) or any(k.startswith(p) for p in skip_prefix):
            new[k] = v
            continue
        arr = param_init_array(k, tuple(v.shape), rng)
        new[k] = torch.from_numpy(np.ascontiguousarray(arr)).to(v.dtype)
    module.load_state_dict(new)
    return module


# ---------------------------------------------------------------------------------------- angles
def angle_feature(heading, elevation, size=ANGLE_FEAT_SIZE):
    """utils.angle_feature (utils.py:361-368)."""
    return np.array([math.sin(heading), math.cos(heading), math.sin(elevation), math.cos(elevation)] * (size // 4),
                    dtype=np.float32)


def view_heading(ix):
    return (ix % 12) * HEADING_INC


def view_elevation(ix):
    return (ix // 12 - 1) * ELEVATION_INC


def point_angle_feature(base_view, size=ANGLE_FEAT_SIZE):
    """utils.get_point_angle_feature (utils.py:386-405) without the simulator: [36, size]."""
    base_heading = (base_view % 12) * HEADING_INC
    return np.stack([angle_feature(view_heading(ix) - base_heading, view_elevation(ix), size)
                     for ix in range(NUM_VIEWS)])


_ANGLE_TABLE = None


def angle_table(size=ANGLE_FEAT_SIZE):
    """[36 base views][36 views][size]"""
    global _ANGLE_TABLE
    if _ANGLE_TABLE is None or _ANGLE_TABLE.shape[-1] != size:
        _ANGLE_TABLE = np.stack([point_angle_feature(b, size) for b in range(NUM_VIEWS)]).astype(np.float32)
    return _ANGLE_TABLE


# ---------------------------------------------------------------------------------------- tokens
def make_tokens(batch, max_len=80, seed=2, lengths=None):
    """[batch, max_len] int64 BERT ids: [CLS]=101, words U{1000..29999}, [SEP]=102, pad 0."""
    rng = np.random.default_rng(seed)
    toks = np.zeros((batch, max_len), dtype=np.int64)
    if lengths is None:
        lengths = [max_len] * batch
    for i, n in enumerate(lengths):
        n = int(n)
        toks[i, 0] = 101
        if n > 2:
            toks[i, 1:n - 1] = rng.integers(1000, 30000, size=n - 2)
        toks[i, n - 1] = 102
    return toks


# ----------------------------------------------------------------------------------------- world
class SynthWorld:
    """Feature pool + navigation graph. Viewpoint ids are 'vp%03d'."""

    def __init__(self, n_viewpoints=64, feat_seed=0, graph_seed=3, max_neighbors=15, angle_feat_size=ANGLE_FEAT_SIZE):
        P = n_viewpoints
        self.P = P
        self.angle_feat_size = angle_feat_size
        frng = np.random.default_rng(feat_seed)
        self.rgb = frng.random((P, NUM_VIEWS, FEATURE_SIZE), dtype=np.float32)
        self.depth = frng.random((P, NUM_VIEWS, FEATURE_SIZE), dtype=np.float32)
        g = np.random.default_rng(graph_seed)
        self.pos = g.random((P, 3)) * 20.0
        self.ids = ["vp%03d" % i for i in range(P)]
        self.index = {v: i for i, v in enumerate(self.ids)}
        self._nav_cache, self._loc_cache = {}, {}
        self.neighbors = []   # per vp: list of (nbr index, pointId, dheading, delevation)
        for v in range(P):
            n = int(g.integers(1, max_neighbors + 1))
            others = [u for u in range(P) if u != v and u != (v + 1) % P]
            pick = [(v + 1) % P] + list(g.choice(others, size=n - 1, replace=False))
            points = g.choice(NUM_VIEWS, size=n, replace=False)
            dh = g.uniform(-0.25, 0.25, size=n)
            de = g.uniform(-0.25, 0.25, size=n)
            self.neighbors.append([(int(u), int(p), float(a), float(b)) for u, p, a, b in zip(pick, points, dh, de)])
        # geodesic distances (Dijkstra on euclidean edge lengths) for goal-mode episodes
        self.dist = np.full((P, P), np.inf)
        self.next_hop = np.full((P, P), -1, dtype=np.int64)
        for s in range(P):
            self._dijkstra(s)

    def loc(self, v):
        """Shared MatterSim Location record of viewpoint v (read-only for callers)."""
        lc = self._loc_cache.get(v)
        if lc is None:
            lc = self._loc_cache[v] = _Loc(self.ids[v])
        return lc

    def _edge(self, a, b):
        return float(np.linalg.norm(self.pos[a] - self.pos[b]))

    def _dijkstra(self, goal):
        # distances TO goal along directed edges: run on the reversed graph
        import heapq
        rev = [[] for _ in range(self.P)]
        for v in range(self.P):
            for (u, _, _, _) in self.neighbors[v]:
                rev[u].append(v)
        d = np.full(self.P, np.inf)
        d[goal] = 0.0
        h = [(0.0, goal)]
        while h:
            dv, v = heapq.heappop(h)
            if dv > d[v]:
                continue
            for w in rev[v]:
                nd = dv + self._edge(w, v)
                if nd < d[w]:
                    d[w] = nd
                    heapq.heappush(h, (nd, w))
        self.dist[:, goal] = d
        for v in range(self.P):
            if v == goal:
                self.next_hop[v, goal] = goal
                continue
            best, bu = np.inf, -1
            for (u, _, _, _) in self.neighbors[v]:
                c = self._edge(v, u) + d[u]
                if c < best:
                    best, bu = c, u
            self.next_hop[v, goal] = bu


# ------------------------------------------------------------------------------------- simulator
class _Loc:
    def __init__(self, vid):
        self.viewpointId = vid
        self.rel_heading = 0.0
        self.rel_elevation = 0.0
        self.rel_distance = 0.0


class _State:
    """MatterSim SimState snapshot; navigableLocations is built on first access (the agent polls
    getState().viewIndex while turning, which never needs it)."""
    __slots__ = ("scanId", "location", "viewIndex", "heading", "elevation", "step", "_nav", "_world", "_navlist")

    @property
    def navigableLocations(self):
        if self._navlist is None:
            self._navlist = [_Loc(self._world.ids[u]) for u in self._nav]
        return self._navlist


class SynthSim:
    """Discretized MatterSim: 12 headings x 3 elevations (MatterSim.cpp:339-367, 470-490)."""

    def __init__(self, world):
        self.world = world
        self.vp = 0
        self.heading = 0.0
        self.elevation = 0.0
        self.view_index = 12
        self.step = 0

    def _set_heading_elevation(self, heading, elevation):
        h = math.fmod(heading, 2 * math.pi)
        while h < 0.0:
            h += 2 * math.pi
        step = int(round(h / HEADING_INC))
        # std::lround semantics (half away from zero) for the positive range used here
        step = int(math.floor(h / HEADING_INC + 0.5))
        if step == 12:
            step = 0
        self.heading = step * HEADING_INC
        if elevation < -ELEVATION_INC / 2:
            self.elevation = -ELEVATION_INC
            self.view_index = step
        elif elevation > ELEVATION_INC / 2:
            self.elevation = ELEVATION_INC
            self.view_index = step + 24
        else:
            self.elevation = 0.0
            self.view_index = step + 12

    def newEpisode(self, scan, vp, heading, elevation):
        self.vp = self.world.index[vp] if isinstance(vp, str) else int(vp)
        self.step = 0
        self._set_heading_elevation(heading, elevation)

    def navigable(self):
        nav = self.world._nav_cache.get(self.vp)
        if nav is None:
            nav = self.world._nav_cache[self.vp] = [self.vp] + [u for (u, _, _, _) in self.world.neighbors[self.vp]]
        return nav

    def makeAction(self, index, heading, elevation):
        nav = self.navigable()
        if index < 0 or index >= len(nav):
            raise ValueError("MatterSim: Invalid action index: %d" % index)
        self.vp = nav[index]
        self.step += 1
        if heading > 0:
            heading = HEADING_INC
        elif heading < 0:
            heading = -HEADING_INC
        if elevation > 0:
            elevation = ELEVATION_INC
        elif elevation < 0:
            elevation = -ELEVATION_INC
        self._set_heading_elevation(self.heading + heading, self.elevation + elevation)

    def equiv_action(self, trg_point, nav_idx, path=None):
        """agent_dg.py:372-391 for one agent in a single call: turn up/down to the target's elevation
        level, then right until the view index is trg_point, then move to navigable location nav_idx —
        the state sequence of that many makeAction calls (each turn is one discretized step of
        MatterSim.cpp:339-367: elevation +-30 deg within [-30, 30], heading +30 deg mod 360), with the
        same (viewpoint, heading, elevation) appended to `path` after every action."""
        rec = path.append if path is not None else None
        vid = self.world.ids[self.vp]
        hstep, lvl = self.view_index % 12, self.view_index // 12
        trg_level, trg_step = trg_point // 12, trg_point % 12
        while lvl != trg_level:
            lvl += 1 if lvl < trg_level else -1
            self.elevation = (lvl - 1) * ELEVATION_INC
            self.step += 1
            if rec:
                rec((vid, self.heading, self.elevation))
        while hstep != trg_step:
            hstep = (hstep + 1) % 12
            self.heading = hstep * HEADING_INC
            self.step += 1
            if rec:
                rec((vid, self.heading, self.elevation))
        self.view_index = lvl * 12 + hstep
        nav = self.navigable()
        if nav_idx < 0 or nav_idx >= len(nav):
            raise ValueError("MatterSim: Invalid action index: %d" % nav_idx)
        self.vp = nav[nav_idx]
        self.step += 1
        if rec:
            rec((self.world.ids[self.vp], self.heading, self.elevation))

    def quick_state(self):
        """(viewpointId, heading, elevation, viewIndex) without building a SimState: the agent's turn
        loop polls the view index after every makeAction (agent_dg.py:376-386)."""
        return self.world.ids[self.vp], self.heading, self.elevation, self.view_index

    def navigable_id(self, k):
        return self.world.ids[self.navigable()[k]]

    def getState(self):
        s = _State()
        s.scanId = "synth"
        s.location = self.world.loc(self.vp)
        s.viewIndex = self.view_index
        s.heading = self.heading
        s.elevation = self.elevation
        s.step = self.step
        s._nav = self.navigable()
        s._world = self.world
        s._navlist = None
        return s


class _EnvBatch:
    def __init__(self, sims):
        self.sims = sims


# ---------------------------------------------------------------------------------- batch env
class SynthR2RBatch:
    """R2RBatch stand-in: reset()/_get_obs() return the obs dicts Seq2SeqAgent consumes.

    mode='goal'   : teacher = next hop of the geodesic shortest path; stops at the goal.
    mode='wander' : teacher = a deterministic pseudo-random neighbour (never 'stop'), distance =
                    euclidean to a virtual goal outside the graph: fixed-length rollouts for benchmarks.
    """

    def __init__(self, world, batch_size, seed=7, mode="goal", instr_len=80, variable_len=False,
                 angle_feat_size=ANGLE_FEAT_SIZE, lazy_features=False):
        self.world = world
        self.batch_size = batch_size
        self.rng = np.random.default_rng(seed)
        self.mode = mode
        self.instr_len = instr_len
        self.variable_len = variable_len
        self.feature_size = FEATURE_SIZE
        self.angle_feat_size = angle_feat_size
        self.angle_feature = [point_angle_feature(b, angle_feat_size) for b in range(NUM_VIEWS)]
        self.env = _EnvBatch([SynthSim(world) for _ in range(batch_size)])
        self.batch = []
        self._episode = 0
        self.virtual_goal = np.array([100.0, 100.0, 100.0])
        # lazy_features: obs dicts carry pool indices instead of the [36, 2176] arrays; the agent then
        # assembles the tensors on the device (device_input_feat), as a device-resident feature store would.
        self.lazy_features = lazy_features
        self._store = None
        self._cand_cache = {}
        self._dist_cache = {}
        self._navloc_cache = {}

    # -- episodes
    def _new_batch(self):
        B = self.batch_size
        if self.variable_len:
            lengths = self.rng.integers(8, self.instr_len + 1, size=B)
        else:
            lengths = np.full(B, self.instr_len)
        toks = make_tokens(B, self.instr_len, seed=int(self.rng.integers(1 << 31)), lengths=lengths)
        batch = []
        for i in range(B):
            start = int(self.rng.integers(self.world.P))
            goal = int(self.rng.integers(self.world.P))
            if goal == start:
                goal = (start + 1) % self.world.P
            view = int(self.rng.integers(12, 24))
            batch.append({
                "instr_id": "synth_%d_%d" % (self._episode, i),
                "path_id": self._episode * 1000 + i,
                "scan": "synth",
                "path": [self.world.ids[start], self.world.ids[goal]],
                "heading": view_heading(view),
                "instructions": "synthetic instruction %d" % i,
                "instr_encoding": toks[i],
                "wander_seed": int(self.rng.integers(1 << 31)),
            })
        self._episode += 1
        return batch

    def reset(self, batch=None, **kwargs):
        self.batch = batch if batch is not None else self._new_batch()
        for sim, item in zip(self.env.sims, self.batch):
            sim.newEpisode(item["scan"], item["path"][0], item["heading"], 0.0)
        return self._get_obs()

    def reset_epoch(self, shuffle=False):
        pass

    # -- observations
    def _candidates(self, v, base_view):
        if self.lazy_features:
            # the world is static, so a viewpoint's candidate list depends only on (v, heading step):
            # memoised (the agent never mutates candidates)
            key = (v, base_view % 12)
            c = self._cand_cache.get(key)
            if c is None:
                c = self._cand_cache[key] = self._make_candidates(v, base_view)
            return c
        return self._make_candidates(v, base_view)

    def _make_candidates(self, v, base_view):
        w = self.world
        base_heading = (base_view % 12) * HEADING_INC
        out = []
        for k, (u, point, dh, de) in enumerate(w.neighbors[v]):
            ang = angle_feature(view_heading(point) - base_heading + dh, view_elevation(point) + de,
                                self.angle_feat_size)
            if self.lazy_features:
                out.append({"viewpointId": w.ids[u], "pointId": point, "idx": k + 1, "angle": ang,
                            "heading": view_heading(point) - base_heading + dh,
                            "elevation": view_elevation(point) + de, "scanId": "synth"})
                continue
            out.append({
                "heading": view_heading(point) - base_heading + dh,
                "elevation": view_elevation(point) + de,
                "scanId": "synth",
                "viewpointId": w.ids[u],
                "pointId": point,
                "distance": math.sqrt(dh * dh + de * de),
                "idx": k + 1,
                "feature": np.concatenate((w.rgb[v, point], ang), -1),
                "dfeature": np.concatenate((w.depth[v, point], ang), -1),
            })
        return out

    def _teacher(self, sim, item):
        w = self.world
        if self.mode == "goal":
            goal = w.index[item["path"][-1]]
            return w.ids[int(w.next_hop[sim.vp, goal])]
        nb = w.neighbors[sim.vp]
        h = (item["wander_seed"] * 1000003 + sim.vp * 9176 + sim.step * 7919) % (1 << 31)
        return w.ids[nb[h % len(nb)][0]]

    def _back_teacher(self, sim, item):
        """env.py:348: the next viewpoint on the shortest path back to the episode start (the current one
        once there; also when the start is unreachable on the directed synthetic graph)."""
        w = self.world
        hop = int(w.next_hop[sim.vp, w.index[item["path"][0]]])
        return w.ids[hop if hop >= 0 else sim.vp]

    def _distance(self, sim, item):
        w = self.world
        if self.mode == "goal":
            return float(w.dist[sim.vp, w.index[item["path"][-1]]])
        d = self._dist_cache.get(sim.vp)
        if d is None:
            d = self._dist_cache[sim.vp] = float(np.linalg.norm(w.pos[sim.vp] - self.virtual_goal))
        return d

    def _nav_locs(self, v):
        """The (shared, read-only) navigableLocations list of viewpoint v."""
        locs = self._navloc_cache.get(v)
        if locs is None:
            w = self.world
            nav = [v] + [u for (u, _, _, _) in w.neighbors[v]]
            locs = self._navloc_cache[v] = [w.loc(u) for u in nav]
        return locs

    def _get_obs(self):
        obs = []
        w = self.world
        lazy = self.lazy_features
        for sim, item in zip(self.env.sims, self.batch):
            v = sim.vp
            base = sim.view_index
            ang = self.angle_feature[base]
            obs.append({
                "instr_id": item["instr_id"],
                "scan": "synth",
                "viewpoint": w.ids[v],
                "viewIndex": base,
                "heading": sim.heading,
                "elevation": sim.elevation,
                "feature": None if lazy else np.concatenate((w.rgb[v], ang), -1),
                "dfeature": None if lazy else np.concatenate((w.depth[v], ang), -1),
                "candidate": self._candidates(v, base),
                "navigableLocations": self._nav_locs(v),
                "instructions": item["instructions"],
                "teacher": self._teacher(sim, item),
                "back_teacher": self._back_teacher(sim, item),
                "path_id": item["path_id"],
                "instr_encoding": item["instr_encoding"],
                "distance": self._distance(sim, item),
                "progress": 0.0,
                "path": item["path"],
                # device fast path (agent_dg.get_input_feat): pool index + view index
                "_vp_index": v,
            })
        return obs


def _store(self, device):
    """The env's device-resident feature store (dasa_amd.features.DeviceFeatureStore)."""
    from .features import DeviceFeatureStore
    if self._store is None or self._store.device != device:
        self._store = DeviceFeatureStore.from_world(self.world, device, self.angle_feat_size)
    return self._store


def _device_input_feat(self, obs, device):
    return _store(self, device).input_feat(obs)


def _device_input_feat_steps(self, obs_steps, device):
    return _store(self, device).input_feat_steps(obs_steps)


SynthR2RBatch.device_input_feat = _device_input_feat
SynthR2RBatch.device_input_feat_steps = _device_input_feat_steps


# ---------------------------------------------------------------------------------- the aug half
def speaker_vocab(n=991):
    """A synthetic speaker word list of the R2R train_vocab.txt's size (991 entries; utils.py:22-24's
    base vocabulary <PAD>, <UNK>, <EOS> first), for the bench's auglistener leg."""
    return ["<PAD>", "<UNK>", "<EOS>"] + ["w%04d" % i for i in range(n - 3)]


class HashBTokenizer:
    """Stand-in for the listener's utils.BTokenizer (bert-base-uncased WordPiece, a name-based download
    that is unavailable offline) with its contract: [CLS]=101 + one id per word + [SEP]=102, padded with
    pad_token_id 0 to encoding_length, an over-long encoding cut with [SEP] last. Word ids are a CRC
    of the word (tests/golden_inputs.py's WordHashBTokenizer is the same mapping)."""

    class _T:
        pad_token_id = 0
        sep_token_id = 102

    def __init__(self, encoding_length=80):
        self.tokenizer = self._T()
        self.encoding_length = encoding_length

    def encode_sentence(self, sentence, seps=None):
        import re
        import zlib
        words = [w for w in re.split(r"\s+", sentence.strip().lower()) if w]
        enc = [101] + [1000 + zlib.crc32(w.encode()) % 29000 for w in words] + [102]
        if len(enc) < self.encoding_length:
            enc += [0] * (self.encoding_length - len(enc))
        if len(enc) > self.encoding_length:
            enc[self.encoding_length - 1] = 102
        return np.array(enc[:self.encoding_length])
