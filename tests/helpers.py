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


def check_grads(G, prefix, named_grads, rtol=2e-4, atol=1e-6):
    """Compare grads against fixture norms / sketches / full small tensors. Returns #checked."""
    n = 0
    for name, g in named_grads:
        key = prefix + name
        if "gnorm/" + key not in G:
            continue
        assert g is not None, f"missing grad for {key}"
        gd = g.detach().double().flatten().cpu().numpy()
        ref_norm = float(G["gnorm/" + key])
        assert abs(np.linalg.norm(gd) - ref_norm) <= rtol * ref_norm + atol, (key, np.linalg.norm(gd), ref_norm)
        sk = float(gd @ sketch_vec(key, gd.size))
        ref_sk = float(G["gsketch/" + key])
        assert abs(sk - ref_sk) <= rtol * ref_norm * np.sqrt(gd.size) * 0.05 + atol * 10, (key, sk, ref_sk)
        if "gfull/" + key in G:
            ref = torch.from_numpy(G["gfull/" + key]).double()
            assert (g.detach().double().cpu() - ref).abs().max().item() <= rtol * max(1.0, ref.abs().max().item()) + atol, key
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
    assert err <= tol, f"{what}: max|diff| {err:.3e} > {tol:.1e}"
    return err
