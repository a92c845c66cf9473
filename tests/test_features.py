"""Real-data feature readers (dasa_amd/features.py) against the reference's own readers, and the
device-side input assembly against the host path it replaces (agent_dg.py:286-323).

CPU: read_img_features / read_depth_features on tiny real-format files reproduce, key for key and
byte for byte (SHA-256), what the reference's utils.read_img_features (utils.py:272-312) and
env.Depth_Features (env.py:22-29) returned on the same files (tests/golden/io.npz, written by
oracle/golden/make_golden.py io).
GPU: DeviceFeatureStore.from_features + DeviceFeatureEnv build bitwise the tensors the reference's
numpy path builds from R2RBatch-style obs (feature ‖ angle_table[viewIndex], candidates with their
relative-angle tail, zero END row)."""
import hashlib

import numpy as np
import pytest
import torch

from dasa_amd import features as FE
from tests import golden_inputs as GI
from tests.helpers import golden


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_img_tsv_reader_matches_reference(tmp_path):
    G = golden("io")
    img, _, _ = GI.io_tables()
    path = str(tmp_path / "feats.tsv")
    FE.write_img_features(path, img)
    feats = FE.read_img_features(path)
    assert sorted(feats) == list(G["img/keys"])
    for k, v in feats.items():
        assert v.dtype == np.float32 and tuple(v.shape) == tuple(G[f"img/shape/{k}"])
        assert _sha(v) == str(G[f"img/sha256/{k}"]), k


def test_depth_reader_matches_reference(tmp_path):
    G = golden("io")
    _, keys, vals = GI.io_tables()
    np.save(tmp_path / "ids.npy", keys)
    np.save(tmp_path / "vals.npy", vals)
    depth = FE.read_depth_features(str(tmp_path / "ids.npy"), str(tmp_path / "vals.npy"))
    assert sorted(depth) == list(G["depth/keys"])
    for k, v in depth.items():
        assert tuple(v.shape) == tuple(G[f"depth/shape/{k}"])
        assert _sha(v) == str(G[f"depth/sha256/{k}"]), k


def test_mini_reader(tmp_path):
    img, _, _ = GI.io_tables()
    ks = np.array(sorted(img))
    np.save(tmp_path / "i.npy", ks)
    np.save(tmp_path / "v.npy", np.stack([img[k] for k in ks]))
    m = FE.read_img_features(None, mini_index=str(tmp_path / "i.npy"), mini_value=str(tmp_path / "v.npy"))
    assert sorted(m) == list(ks) and all(np.array_equal(m[k], img[k]) for k in ks)


def _obs(img, depth, keys, rng):
    """R2RBatch._get_obs-style observations (env.py:317-360, make_candidate :240-315)."""
    from dasa_amd.synth import angle_feature, angle_table
    table = angle_table(128)
    obs = []
    for i, k in enumerate(keys):
        scan, vp = k.split("_", 1)
        view = int(rng.integers(36))
        cands = []
        for j in range(int(rng.integers(0, 6))):
            point = int(rng.integers(36))
            ang = angle_feature(float(rng.normal()), float(rng.normal()) * 0.3, 128)
            cands.append({"pointId": point, "viewpointId": f"x{j}", "idx": j + 1,
                          "feature": np.concatenate((img[k][point], ang)),
                          "dfeature": np.concatenate((depth[k][point], ang))})
        obs.append({"scan": scan, "viewpoint": vp, "viewIndex": view, "heading": float(rng.normal()),
                    "elevation": float(rng.normal()) * 0.3,
                    "feature": np.concatenate((img[k], table[view]), -1),
                    "dfeature": np.concatenate((depth[k], table[view]), -1), "candidate": cands})
    return obs


def _host_input_feat(obs):
    """The reference's numpy assembly (agent_dg.py:286-323)."""
    from dasa_amd.synth import angle_feature
    B = len(obs)
    a = np.stack([angle_feature(ob["heading"], ob["elevation"], 128) for ob in obs])
    f = np.stack([ob["feature"] for ob in obs]).astype(np.float32)
    d = np.stack([ob["dfeature"] for ob in obs]).astype(np.float32)
    leng = [len(ob["candidate"]) + 1 for ob in obs]
    cf = np.zeros((B, max(leng), 2176), np.float32)
    cd = np.zeros_like(cf)
    for i, ob in enumerate(obs):
        for j, c in enumerate(ob["candidate"]):
            cf[i, j] = c["feature"]
            cd[i, j] = c["dfeature"]
    return a, f, d, cf, cd, leng


@pytest.mark.gpu
def test_device_store_matches_host_assembly(dev):
    img, keys, vals = GI.io_tables()
    depth = {f"{a}_{b}": vals[i] for i, (a, b) in enumerate(keys)}
    both = sorted(set(img) & set(depth))
    img = {k: img[k] for k in both}
    store = FE.DeviceFeatureStore.from_features(img, depth, dev)
    env = FE.DeviceFeatureEnv(object(), store)
    rng = np.random.default_rng(5)
    steps = [_obs(img, depth, [both[i % len(both)] for i in range(5)], rng) for _ in range(3)]
    for obs in steps:
        got = env.device_input_feat(obs, dev)
        want = _host_input_feat(obs)
        for g, w in zip(got[:5], want[:5]):
            assert torch.equal(g.cpu(), torch.from_numpy(np.ascontiguousarray(w)))
        assert got[5] == want[5]
    a_t, f_t, d_t, cf, cd, cinfo = env.device_input_feat_steps(steps, dev)
    for t, obs in enumerate(steps):
        want = _host_input_feat(obs)
        off, C, leng = cinfo[t]
        B = len(obs)
        assert torch.equal(f_t[t * B:(t + 1) * B].cpu(), torch.from_numpy(want[1]))
        assert torch.equal(cd[off:off + B * C].view(B, C, -1).cpu(), torch.from_numpy(want[4]))
        assert leng == want[5]


def test_step_arrays_vectorised_matches_loop():
    """DeviceFeatureStore._step_arrays (the batch-vectorised host index blocks of one decision step) equals
    the per-observation loop it replaced, including observations with no candidates and ragged C."""
    img, keys, vals = GI.io_tables()
    depth = {f"{a}_{b}": vals[i] for i, (a, b) in enumerate(keys)}
    both = sorted(set(img) & set(depth))
    img = {k: img[k] for k in both}
    store = FE.DeviceFeatureStore.from_features(img, depth, torch.device("cpu"))
    rng = np.random.default_rng(7)
    for t in range(4):
        obs = _obs(img, depth, [both[(i * 3 + t) % len(both)] for i in range(6)], rng)
        if t == 2:
            obs[1]["candidate"] = []
        base = 17 * t
        got = store._step_arrays(obs, base)
        want = store._step_arrays_loop(obs, base)
        for g, w in zip(got[:6], want[:6]):
            assert g.dtype == w.dtype and np.array_equal(g, w), t
        assert got[6:] == want[6:]
