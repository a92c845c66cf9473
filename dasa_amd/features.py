"""Real-data panorama features for the policy path: the reference's readers,
restated, and a device-resident store that assembles the agent's input blocks on the GPU.

  * read_img_features   - utils.py:272-312: the ResNet-152 TSV (scanId, viewpointId, image_w, image_h,
                          vfov, features = base64 float32 [views, 2048]) -> {"scan_viewpoint": [views, 2048]};
                          with args.mini, the index / value .npy pair (utils.py:289-296);
  * read_depth_features - env.py:22-29 (Depth_Features): data/viewpointIds.npy [N, 2] (scan, viewpoint)
                          + data/ResNet-152-imagenet-depth.npy [N, 36, 2048] -> {"scan_viewpoint": [36, 2048]};
  * DeviceFeatureStore.from_features - both tables resident in HBM as [P*36, 2048] pools (288 GB holds
                          the full R2R set of ~10.6k viewpoints x 36 x 2048 x 4 B x 2 = 6.2 GB many times);
  * DeviceFeatureEnv    - wraps an R2RBatch-style env (obs dicts as env.py:317-360 builds them) and gives
                          the agent device_input_feat / device_input_feat_steps: the panorama and candidate
                          feature rows are gathered on the device (dasa_gather_rows) instead of numpy-
                          concatenated and copied per step (agent_dg.py:286-323); only the candidates'
                          relative-angle columns (B x C x 128 floats) travel from the host.
"""
import base64
import csv
import sys

import numpy as np

TSV_FIELDNAMES = ["scanId", "viewpointId", "image_w", "image_h", "vfov", "features"]


def read_img_features(feature_store, views=36, mini_index=None, mini_value=None):
    """utils.py:272-312. Returns {scan_viewpoint: float32 [views, F]} (read-only views of the decoded
    bytes, as np.frombuffer gives the reference)."""
    if mini_index is not None:              # args.mini (utils.py:289-296)
        idx, val = np.load(mini_index), np.load(mini_value)
        return {k: v for k, v in zip(idx, val)}
    csv.field_size_limit(sys.maxsize)
    features = {}
    with open(feature_store, "r") as f:
        for item in csv.DictReader(f, delimiter="\t", fieldnames=TSV_FIELDNAMES):
            long_id = item["scanId"] + "_" + item["viewpointId"]
            raw = base64.b64decode(item["features"].encode("ascii"))
            features[long_id] = np.frombuffer(raw, dtype=np.float32).reshape((views, -1))
    return features


def write_img_features(path, features, image_w=640, image_h=480, vfov=60):
    """The inverse of read_img_features: {scan_viewpoint: [views, F]} -> TSV (test data, converters)."""
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, delimiter="\t", fieldnames=TSV_FIELDNAMES)
        for long_id, arr in features.items():
            scan, vp = long_id.split("_", 1)
            w.writerow({"scanId": scan, "viewpointId": vp, "image_w": image_w, "image_h": image_h, "vfov": vfov,
                        "features": base64.b64encode(np.ascontiguousarray(arr, np.float32).tobytes()).decode("ascii")})


def read_depth_features(index_file, value_file):
    """env.py:22-29: {"scan_viewpoint": [36, 2048]} from the (scan, viewpoint) index and value arrays."""
    keys = np.load(index_file)
    values = np.load(value_file, mmap_mode="r")
    return {"{}_{}".format(k[0], k[1]): values[i] for i, k in enumerate(keys)}


class DeviceFeatureStore:
    """RGB and depth pools [P*36, F] + the 36x36 angle table [36*36, 128] resident on the device; the
    agent's input blocks (panorama [B, 36, F+128], candidates [B, C, F+128]) are assembled with one
    dasa_gather_rows launch per block."""

    def __init__(self, rgb, depth, device, keys=None, angle_feat_size=128):
        import torch
        from .synth import angle_table
        P, V, F = rgb.shape
        assert depth.shape == rgb.shape and V == 36
        self.device = device
        self.F = F
        self.A = angle_feat_size
        self.rgb = torch.from_numpy(np.ascontiguousarray(rgb, np.float32).reshape(P * V, F)).to(device)
        self.depth = torch.from_numpy(np.ascontiguousarray(depth, np.float32).reshape(P * V, F)).to(device)
        self.angles = torch.from_numpy(angle_table(angle_feat_size).reshape(V * V, -1)).to(device)
        self.index = {k: i for i, k in enumerate(keys)} if keys is not None else None
        self._angle_cache = {}
        self._cand_cache = {}

    @classmethod
    def from_world(cls, world, device, angle_feat_size=128):
        return cls(world.rgb, world.depth, device, None, angle_feat_size)

    @classmethod
    def from_features(cls, img_features, depth_features, device, angle_feat_size=128):
        """Every viewpoint present in both tables, pooled in sorted key order."""
        keys = sorted(set(img_features) & set(depth_features))
        rgb = np.stack([np.asarray(img_features[k], np.float32) for k in keys])
        depth = np.stack([np.asarray(depth_features[k], np.float32) for k in keys])
        return cls(rgb, depth, device, keys, angle_feat_size)

    def _angle(self, heading, elevation):
        """utils.angle_feature of the agent's own heading / elevation (memoised: a few hundred distinct
        discretized values)."""
        key = (heading, elevation)
        a = self._angle_cache.get(key)
        if a is None:
            from .synth import angle_feature
            if len(self._angle_cache) > 65536:
                self._angle_cache.clear()
            a = self._angle_cache[key] = angle_feature(heading, elevation, self.A)
        return a

    def _cand_arrays(self, cands):
        """(pointIds int32 [n], relative-angle block [n, A]) of a candidate list. Lists of lightweight
        candidates (an "angle" entry instead of feature arrays: envs that memoise their candidate lists,
        like the synthetic one) are memoised per list object; R2RBatch's per-step lists are not kept."""
        e = self._cand_cache.get(id(cands))
        if e is not None and e[0] is cands:
            return e[1], e[2]
        A = self.A
        pts = np.array([c["pointId"] for c in cands], np.int32)
        angs = (np.stack([c["angle"] if "angle" in c else c["feature"][-A:] for c in cands]).astype(np.float32)
                if cands else np.zeros((0, A), np.float32))
        if cands and "angle" in cands[0]:
            if len(self._cand_cache) > 65536:
                self._cand_cache.clear()
            self._cand_cache[id(cands)] = (cands, pts, angs)
        return pts, angs

    def _row(self, ob):
        if "_vp_index" in ob:
            return ob["_vp_index"]
        return self.index[ob["scan"] + "_" + ob["viewpoint"]]

    def input_feat(self, obs):
        a_t, f_t, d_t, cf, cd, cinfo = self.input_feat_steps([obs])
        _, C, leng = cinfo[0]
        B = len(obs)
        return a_t, f_t, d_t, cf.view(B, C, -1), cd.view(B, C, -1), leng

    def _step_arrays(self, obs, base):
        """One step's host-side index blocks, vectorised over the batch (the per-observation loop was
        ≈0.2 ms of host time per decision step, all of it GPU idle in the sampled rollout, which waits on
        it after every action sync): candidate gather rows iac / ibc [B, C] (-1 = padding), candidate
        angles cang [B, C, A], own-angle rows a_t [B, A], viewpoint rows, view indices, C, lengths."""
        A, V = self.A, 36
        B = len(obs)
        vp = np.fromiter((self._row(ob) for ob in obs), np.int64, B)
        view = np.fromiter((ob["viewIndex"] for ob in obs), np.int64, B)
        cand = [self._cand_arrays(ob["candidate"]) for ob in obs]
        ns = np.fromiter((len(p) for p, _ in cand), np.int64, B)
        leng = (ns + 1).tolist()
        C = int(ns.max()) + 1 if B else 1
        a_t = np.stack([self._angle(ob["heading"], ob["elevation"]) for ob in obs]).astype(np.float32, copy=False)
        iac = np.full((B, C), -1, np.int32)
        ibc = np.full((B, C), -1, np.int32)
        cang = np.zeros((B, C, A), np.float32)
        tot = int(ns.sum())
        if tot:
            rows = np.repeat(np.arange(B), ns)
            cols = np.arange(tot) - np.repeat(np.cumsum(ns) - ns, ns)
            iac[rows, cols] = (vp[rows] * V + np.concatenate([p for p, _ in cand])).astype(np.int32)
            ibc[rows, cols] = (base + rows * C + cols).astype(np.int32)
            cang[rows, cols] = np.concatenate([a for _, a in cand if len(a)])
        return iac, ibc, cang, a_t, vp, view, C, leng

    def _step_arrays_loop(self, obs, base):
        """The per-observation form of _step_arrays (test reference)."""
        A = self.A
        B = len(obs)
        leng = [len(ob["candidate"]) + 1 for ob in obs]
        C = max(leng)
        vp = np.array([self._row(ob) for ob in obs], np.int64)
        view = np.array([ob["viewIndex"] for ob in obs], np.int64)
        iac = np.full((B, C), -1, np.int32)
        ibc = np.full((B, C), -1, np.int32)
        cang = np.zeros((B, C, A), np.float32)
        a_t = np.zeros((B, A), np.float32)
        for i, ob in enumerate(obs):
            a_t[i] = self._angle(ob["heading"], ob["elevation"])
            pts, angs = self._cand_arrays(ob["candidate"])
            n = len(pts)
            if n:
                iac[i, :n] = vp[i] * 36 + pts
                ibc[i, :n] = base + i * C + np.arange(n, dtype=np.int32)
                cang[i, :n] = angs
        return iac, ibc, cang, a_t, vp, view, C, leng

    def input_feat_steps(self, obs_steps):
        """The input blocks of several rollout steps stacked along the batch (step-major): a_t [T*B, A],
        panoramas f_t / d_t [T*B, 36, F+A], and the candidates of every step as flat rows cf / cd [R, F+A]
        with cinfo[t] = (first row, C_t, lengths_t) — step t's block is rows [off, off + B*C_t) viewed
        as [B, C_t, F+A]. The END candidate row is zero (agent_dg.py:305-306). One gather per tensor."""
        import torch
        from . import ops
        A, V = self.A, 36
        ia_v, ib_v, ia_c, ib_c, cangs, a_ts, cinfo = [], [], [], [], [], [], []
        rv = np.arange(V)
        row = 0
        base = 0
        for obs in obs_steps:
            B = len(obs)
            iac, ibc, cang, a_t, vp, view, C, leng = self._step_arrays(obs, base)
            ia_v.append((vp[:, None] * V + rv[None]).astype(np.int32).reshape(-1))
            ib_v.append((view[:, None] * V + rv[None]).astype(np.int32).reshape(-1))
            base += B * C
            ia_c.append(iac.reshape(-1))
            ib_c.append(ibc.reshape(-1))
            cangs.append(cang.reshape(B * C, A))
            a_ts.append(a_t)
            cinfo.append((row, C, leng))
            row += B * C
        ia_v, ib_v = np.concatenate(ia_v), np.concatenate(ib_v)
        ia_c, ib_c = np.concatenate(ia_c), np.concatenate(ib_c)
        a_t, cang = np.concatenate(a_ts), np.concatenate(cangs)
        ints = torch.from_numpy(np.concatenate([ia_v, ib_v, ia_c, ib_c])).pin_memory()
        flts = torch.from_numpy(np.concatenate([a_t.reshape(-1), cang.reshape(-1)])).pin_memory()
        ints = ints.to(self.device, non_blocking=True)
        flts = flts.to(self.device, non_blocking=True)
        N, R = a_t.shape[0], ia_c.shape[0]
        n = N * V
        ia_v_d, ib_v_d = ints[:n], ints[n:2 * n]
        ia_c_d, ib_c_d = ints[2 * n:2 * n + R], ints[2 * n + R:]
        a_t_d = flts[:N * A].view(N, A)
        cang_d = flts[N * A:].view(R, A)
        Fa = self.F + A
        f_t = torch.empty(N, V, Fa, dtype=torch.float32, device=self.device)
        d_t = torch.empty_like(f_t)
        cf = torch.empty(R, Fa, dtype=torch.float32, device=self.device)
        cd = torch.empty_like(cf)
        ops.gather_rows(self.rgb, ia_v_d, self.angles, ib_v_d, f_t)
        ops.gather_rows(self.depth, ia_v_d, self.angles, ib_v_d, d_t)
        ops.gather_rows(self.rgb, ia_c_d, cang_d, ib_c_d, cf)
        ops.gather_rows(self.depth, ia_c_d, cang_d, ib_c_d, cd)
        return a_t_d, f_t, d_t, cf, cd, cinfo


class DeviceFeatureEnv:
    """An R2RBatch-style env (env.py:201-504 obs contract) plus device-side input assembly from a
    DeviceFeatureStore; every other attribute is the wrapped env's (reset, _get_obs, env.sims, ...)."""

    def __init__(self, env, store):
        self._env = env
        self._store = store

    def __getattr__(self, k):
        return getattr(self._env, k)

    def device_input_feat(self, obs, device):
        return self._store.input_feat(obs)

    def device_input_feat_steps(self, obs_steps, device):
        return self._store.input_feat_steps(obs_steps)
