"""Shared test helpers: golden fixtures, seeded weights for the oracle and the product modules."""
import json
import os
import zlib

import numpy as np
import torch

from dasa_amd.synth import init_param_dict
from tests import golden_inputs as GI

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_CACHE = {}


def golden(name):
    if name not in _CACHE:
        _CACHE[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    return _CACHE[name]


def sketch_vec(name, n):
    return np.random.default_rng(zlib.crc32(name.encode())).standard_normal(n).astype(np.float64)


N_SKETCH = 8          # independent Gaussian sketches <g, r_i> per recorded gradient
SUBSET_ROWS = 32      # rows of every matrix gradient larger than FULL_MAX kept in full
SUBSET_ELEMS = 512    # elements of every vector gradient larger than FULL_MAX kept in full
FULL_MAX = 4096       # gradients up to this many elements are kept in full


def grad_subset_index(key, shape):
    """The fixed (seeded by the key) row subset of a matrix gradient, or element subset of a vector."""
    rng = np.random.default_rng(zlib.crc32(("rows:" + key).encode()))
    n = shape[0]
    k = min(n, SUBSET_ROWS if len(shape) == 2 else SUBSET_ELEMS)
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.int64)


def grad_record(out, key, g):
    """Fixture entries for one gradient (used by oracle/golden/make_golden.py): its norm, max |g|,
    N_SKETCH sketches, and the full values (small tensors) or a fixed row / element subset."""
    gd = g.detach().double().cpu()
    gf = gd.flatten().numpy()
    out["gnorm/" + key] = np.array(np.linalg.norm(gf))
    out["gmax/" + key] = np.array(np.abs(gf).max() if gf.size else 0.0)
    out["gsketch/" + key] = np.array([gf @ sketch_vec(f"{key}#{i}", gf.size) for i in range(N_SKETCH)])
    if gf.size <= FULL_MAX:
        out["gfull/" + key] = gd.numpy().astype(np.float32)
    elif gd.dim() <= 2:
        idx = grad_subset_index(key, tuple(gd.shape))
        out["grows/" + key] = gd.numpy()[idx].astype(np.float32)


def check_grads(G, prefix, named_grads, rtol=2e-4, atol=1e-6):
    """Compare gradients with a fixture. For each recorded gradient g_ref (error e = g - g_ref):
      * norm:      | ||g|| - ||g_ref|| | <= rtol ||g_ref|| + atol;
      * sketches:  each <e, r_i> ~ N(0, ||e||^2) for the recorded Gaussian r_i, so requiring
                   |<e, r_i>| <= 4 rtol ||g_ref|| over N_SKETCH independent sketches bounds ||e|| by
                   about rtol ||g_ref|| (no sqrt(numel) slack);
      * elements:  the full tensor (<= FULL_MAX elements) or the fixed row / element subset within
                   rtol * max|g_ref| + atol (catches a wrong row block, sign or permutation).
    Returns the number of gradients checked."""
    n = 0
    for name, g in named_grads:
        key = prefix + name
        if "gnorm/" + key not in G:
            continue
        assert g is not None, f"missing grad for {key}"
        gt = g.detach().double().cpu()
        gd = gt.flatten().numpy()
        ref_norm = float(G["gnorm/" + key])
        assert abs(np.linalg.norm(gd) - ref_norm) <= rtol * ref_norm + atol, (key, np.linalg.norm(gd), ref_norm)
        sks = np.atleast_1d(G["gsketch/" + key])
        for i, ref_sk in enumerate(sks):
            sk = float(gd @ sketch_vec(f"{key}#{i}", gd.size))
            assert abs(sk - ref_sk) <= 4.0 * rtol * ref_norm + 10 * atol, (key, i, sk, float(ref_sk), ref_norm)
        gmax = float(G["gmax/" + key]) if "gmax/" + key in G else float(np.abs(gd).max())
        if "gfull/" + key in G:
            ref = torch.from_numpy(G["gfull/" + key]).double()
            err = (gt - ref).abs().max().item()
            assert err <= rtol * max(1.0, ref.abs().max().item()) + atol, (key, err)
        if "grows/" + key in G:
            idx = grad_subset_index(key, tuple(gt.shape))
            ref = torch.from_numpy(G["grows/" + key]).double()
            err = (gt[torch.from_numpy(idx)] - ref).abs().max().item()
            assert err <= rtol * gmax + atol, (key, "row subset", err, gmax)
        n += 1
    return n


def schema_from_golden(module_name):
    G = golden("cfg1_rollout")
    return {k: tuple(v) for k, v in json.loads(str(G["schema/" + module_name])).items()}


def oracle_weights(vl_layers=1, la_layers=9, requires_grad=False):
    from oracle import policy, schema
    enc = init_param_dict(schema.encoder_schema(vl_layers, la_layers), GI.SEED_ENC)
    dec = init_param_dict(schema.decoder_schema(), GI.SEED_DEC)
    cri = init_param_dict(schema.critic_schema(), GI.SEED_CRITIC)
    ada = init_param_dict(schema.ada_schema(), GI.SEED_ADA)
    if requires_grad:
        for d in (enc, dec, cri, ada):
            for v in d.values():
                v.requires_grad_(True)
    return policy.Weights(enc, dec, cri, ada)


def close(a, b, tol, what=""):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item() if a.numel() else 0.0
    if err > tol:
        d = (a - b).abs()
        idx = tuple(int(i) for i in torch.nonzero(d == d.max())[0])
        bad = int((d > tol).sum())
        raise AssertionError(f"{what}: max|diff| {err:.3e} > {tol:.1e} at {idx} (got {a[idx].item():.6g}, want "
                             f"{b[idx].item():.6g}; {bad} of {a.numel()} elements off)")
    return err
