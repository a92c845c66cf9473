"""CPU-only checks of the host side: the C-ABI library loads and exports every declared symbol, the
reference-API modules have the reference's state_dict schema, the synthetic env follows the
MatterSim discretization, and args parse like the reference's param.py."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "dasa_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dasa_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from dasa_amd import _lib
    L = _lib.lib()
    syms = _declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) <= set(_lib.SIGNATURES), set(syms) - set(_lib.SIGNATURES)
    assert L.dasa_version() >= 1 and b"gfx950" in L.dasa_build_info()


def test_no_packed_fp32(tmp_path):
    """No device kernel of the built library uses packed-FP32 VALU (v_pk_fma/mul/add_f32): r05 traced the
    r04 row-split attention corruption to their results beside a starting MFMA-dense GEMM workgroup
    (dasa_amd/build.py FLAGS, -fno-slp-vectorize). Disassembles every gfx950 code object of the .so."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    from dasa_amd import _lib
    lib = os.path.join(tmp_path, "lib.so")
    shutil.copy(_lib.LIB_PATH, lib)
    subprocess.run([objdump, "--offloading", lib], cwd=tmp_path, capture_output=True, check=True)
    objs = sorted(f for f in os.listdir(tmp_path) if f.endswith("gfx950"))
    assert len(objs) >= 7, objs          # one code object per source
    found = {}
    for f in objs:
        r = subprocess.run([objdump, "-d", "--mcpu=gfx950", os.path.join(tmp_path, f)], capture_output=True, text=True,
                           check=True)
        n = len(re.findall(r"\bv_pk_(?:fma|mul|add)_f32\b", r.stdout))
        if n:
            found[f] = n
    assert not found, found


def test_gemm_workspace_query_is_host_only():
    """dasa_gemm_f32_workspace plans split-K without touching the device."""
    import ctypes
    from dasa_amd import _lib
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.batch, d.opA, d.opB = 20, 4096, 2240, 1, 0, 1
    assert _lib.lib().dasa_gemm_f32_workspace(ctypes.byref(d)) > 0      # skinny decoder GEMM: split-K
    d.M, d.N, d.K = 1600, 3072, 768
    cnt = 64 << 10                                                       # stream-K arrival counters
    assert _lib.lib().dasa_gemm_f32_workspace(ctypes.byref(d)) == cnt   # plenty of tiles: no split
    d.M, d.N, d.K = 1040, 2048, 2048
    assert _lib.lib().dasa_gemm_f32_workspace(ctypes.byref(d)) > cnt    # mid-size long K: stream-K slabs


def test_x6_plan_and_lstm_switches_are_host_only():
    """The bf16x6 workspace query (split-K only on few-tile problems) and the r03 bi-LSTM x6 switches
    (set / query semantics, the large-batch BPTT workspace holding W_hh^T and its three bf16 planes)."""
    import ctypes
    from dasa_amd import _lib
    L = _lib.lib()
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.batch, d.opA, d.opB = 720, 768, 3072, 1, 0, 1
    assert L.dasa_gemm_f32x6_workspace(ctypes.byref(d)) > 0          # 36 tiles: K split over workgroups
    d.M, d.N, d.K = 12800, 3072, 768
    assert L.dasa_gemm_f32x6_workspace(ctypes.byref(d)) == 0         # 2400 tiles: one workgroup per tile
    for hook in (L.dasa_bilstm_bptt_x6, L.dasa_bilstm_fwd_x6, L.dasa_bilstm_bptt_one_tile):
        prev = hook(-1)
        assert prev in (0, 1)
        assert hook(0) == prev and hook(-1) == 0
        assert hook(1) == 0 and hook(-1) == 1
        hook(prev)
    B, H = 700, 1024
    assert L.dasa_bilstm_bwd_workspace(B, H) >= (6 * B * H + 20 * H * H) * 4
    prev = L.dasa_mha_bwd_split(-1)                                   # attention backward split (0 = auto)
    assert L.dasa_mha_bwd_split(3) == prev and L.dasa_mha_bwd_split(-1) == 3
    assert L.dasa_mha_bwd_split(99) == 3 and L.dasa_mha_bwd_split(-1) == 16
    L.dasa_mha_bwd_split(prev)


def test_product_schema_matches_reference():
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1"])
    from dasa_amd.r2r import model, r2rmodel
    from dasa_amd.r2r.agent_dg import DGAdaChannel
    from tests.helpers import schema_from_golden
    A = param.args
    enc = r2rmodel.DicEncoder(2176, A.d_enc_hidden_size, A.d_hidden_size, A.d_dropout_ratio, A.d_bidirectional,
                              A.d_transformer_update, A.d_bert_n_layers, A.d_reverse_input, A.d_top_lstm, 1,
                              A.d_la_layers, A.d_bert_type, update_add_layer=A.d_update_add_layer)
    dec = model.BAttnDecoderLSTM(A.aemb, A.d_hidden_size, A.dropout, feature_size=2176)
    for mod, name in ((enc, "encoder"), (dec, "decoder"), (model.Critic(), "critic"), (DGAdaChannel(2048), "adaIn")):
        got = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
        assert got == schema_from_golden(name), name


def test_product_modules_refuse_cpu_tensors():
    """No silent CPU fallback: the HIP path raises on host tensors."""
    from dasa_amd import _lib, ops
    with pytest.raises(_lib.DasaError):
        ops.linear(torch.zeros(4, 8), torch.zeros(8, 8))


def test_args_match_reference_flags():
    from dasa_amd.r2r import param
    a = param.readme_train()
    assert (a.d_vl_layers, a.shift_kernel_size, a.angle_feat_size, a.batchSize, a.maxAction) == (3, 5, 128, 20, 35)
    assert a.use_shift and a.depth_drop and a.include_vision and a.optimizer is torch.optim.RMSprop
    assert a.ml_weight_org == 0.4 and a.featdropout == 0.4 and a.d_enc_hidden_size == 1024
    b = param.parse([])
    assert b.d_vl_layers == 4 and b.angle_feat_size == 4 and not b.use_shift   # reference defaults
    ref = os.path.join("/root/reference/r2r_src/param.py")
    if os.path.exists(ref):   # every flag the reference declares is accepted here
        flags = set(re.findall(r"add_argument\(\s*['\"](--[A-Za-z0-9_]+)", open(ref).read()))
        ours = {f for f, *_ in param._FLAGS}
        assert flags <= ours, flags - ours


def test_synth_env_discretization_and_obs_contract():
    from dasa_amd.synth import SynthR2RBatch, SynthSim, SynthWorld
    w = SynthWorld(16)
    sim = SynthSim(w)
    sim.newEpisode("synth", "vp000", 0.0, np.radians(-30))
    assert sim.getState().viewIndex == 0
    for ix in range(1, 36):          # utils.get_point_angle_feature's sweep (utils.py:390-403)
        sim.makeAction(0, 1.0, 1.0 if ix % 12 == 0 else 0.0)
        assert sim.getState().viewIndex == ix
    env = SynthR2RBatch(w, 3, seed=1)
    obs = env.reset()
    for ob in obs:
        assert ob["feature"].shape == (36, 2176) and ob["dfeature"].shape == (36, 2176)
        for c in ob["candidate"]:
            assert c["feature"].shape == (2176,)
            assert np.array_equal(c["feature"][:2048], w.rgb[w.index[ob["viewpoint"]], c["pointId"]])
        assert ob["teacher"] in [c["viewpointId"] for c in ob["candidate"]] + [ob["viewpoint"]]


def test_oracle_sort_and_masks():
    from oracle import policy as O
    obs = [{"instr_encoding": np.array([101, 5, 102, 0, 0])}, {"instr_encoding": np.array([101, 5, 6, 7, 102])}]
    seq, mask, lens, perm = O.sort_batch(obs)
    assert lens == [5, 3] and perm == [1, 0] and mask.shape == (2, 5) and mask[1, 3:].all()
    assert O.length2mask([3, 1]).tolist() == [[False, False, False], [False, True, True]]


def test_dropin_launcher_binds_reference_module_names(tmp_path, monkeypatch):
    """dasa_amd.launch runs an unchanged train.py with param/agent_dg/model bound to dasa_amd.r2r and
    reference-only names (e.g. an alternative decoder) falling back to the reference file."""
    import subprocess
    import sys
    (tmp_path / "model.py").write_text("RefOnlyDecoder = 'reference-only-decoder'\n")
    (tmp_path / "train.py").write_text(
        "from param import args\n"
        "import model, agent_dg, speaker\n"
        "assert args.d_vl_layers == 3 and args.use_shift, args.d_vl_layers\n"
        "assert agent_dg.Seq2SeqAgent.__module__.startswith('dasa_amd.r2r')\n"
        "assert model.BAttnDecoderLSTM.__module__ == 'dasa_amd.r2r.model'\n"
        "assert model.RefOnlyDecoder == 'reference-only-decoder'\n"
        "assert model.SpeakerEncoder.__module__ == 'dasa_amd.r2r.model'\n"
        "assert speaker.Speaker.__module__ == 'dasa_amd.r2r.speaker'\n"
        "print('DROPIN-OK')\n")
    from dasa_amd.r2r import param
    r = subprocess.run([sys.executable, "-m", "dasa_amd.launch", str(tmp_path / "train.py")] + param.README_TRAIN_FLAGS,
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0 and "DROPIN-OK" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("mode", ["validspeaker", "speaker"])
def test_dropin_launcher_speaker_modes_use_reference_speaker(tmp_path, mode):
    """--train speaker / validspeaker train or validate the speaker (speaker.train / valid,
    train.py:111,593): the launcher leaves the reference's speaker module and model.Speaker* classes
    bound there (ours provides infer_batch only), while the policy modules stay ours."""
    import subprocess
    import sys
    (tmp_path / "model.py").write_text("SpeakerEncoder = 'ref-speaker-encoder'\nSpeakerDecoder = 'ref-speaker-decoder'\n")
    (tmp_path / "speaker.py").write_text(
        "import model\n"
        "class Speaker:\n"
        "    encoder_cls = model.SpeakerEncoder\n"
        "    def train(self, n):\n        return 'ref-train'\n"
        "    def valid(self, wrapper=None):\n        return 'ref-valid'\n")
    (tmp_path / "train.py").write_text(
        "from param import args\n"
        "import model, agent_dg, speaker\n"
        "assert agent_dg.Seq2SeqAgent.__module__.startswith('dasa_amd.r2r')\n"
        "assert model.BAttnDecoderLSTM.__module__ == 'dasa_amd.r2r.model'\n"
        "assert model.SpeakerEncoder == 'ref-speaker-encoder', model.SpeakerEncoder\n"
        "assert model.SpeakerDecoder == 'ref-speaker-decoder'\n"
        "assert speaker.Speaker.encoder_cls == 'ref-speaker-encoder'\n"
        "assert speaker.Speaker().valid() == 'ref-valid' and speaker.Speaker().train(1) == 'ref-train'\n"
        "print('SPEAKER-MODE-OK')\n")
    from dasa_amd.r2r import param
    flags = list(param.README_TRAIN_FLAGS)
    flags[flags.index("--train") + 1] = mode
    r = subprocess.run([sys.executable, "-m", "dasa_amd.launch", str(tmp_path / "train.py")] + flags,
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0 and "SPEAKER-MODE-OK" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("mode,seed", [("goal", 8), ("wander", 1000)])
def test_teacher_plan_matches_stepwise_oracle(mode, seed):
    """Seq2SeqAgent._teacher_plan (env stepped through a whole teacher-forced episode before the
    batched encoder runs) yields, step by step, the targets, ended flags, rewards and masks of the
    oracle's interleaved loop (agent_dg.py:832-936 restated in oracle/policy.py)."""
    from dasa_amd.r2r import param
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    from dasa_amd.synth import SynthR2RBatch, SynthWorld
    from oracle import policy as O
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "6", "--maxAction", "8"])
    world = SynthWorld(24, 0, 3)
    env = SynthR2RBatch(world, 6, seed=seed, mode=mode, instr_len=80, variable_len=True)
    env2 = SynthR2RBatch(world, 6, seed=seed, mode=mode, instr_len=80, variable_len=True)
    ag = object.__new__(Seq2SeqAgent)
    ag.env, ag.episode_len = env, 8
    obs = np.array(env.reset())
    _, _, _, perm_idx = O.sort_batch(obs)
    perm_obs = obs[perm_idx]
    last = np.array([ob["distance"] for ob in perm_obs], np.float32)
    ended = np.zeros(6, bool)
    traj = [{"path": []} for _ in perm_obs]
    plan, final_obs = ag._teacher_plan(perm_obs, list(perm_idx), ended, last, traj, 3)
    more, final_obs = ag._teacher_plan(final_obs, list(perm_idx), ended, last, traj, 5)
    plan = plan + more
    # the oracle's loop, teacher feedback
    obs2 = np.array(env2.reset())
    po = obs2[perm_idx]
    last2 = np.array([ob["distance"] for ob in po], np.float32)
    ended2 = np.zeros(6, bool)
    for t in range(8):
        tgt = O.teacher_action(po, ended2).numpy()
        assert t < len(plan)
        np.testing.assert_array_equal(plan[t]["target_np"], tgt)
        np.testing.assert_array_equal(plan[t]["ended"], ended2)
        cpu_a = tgt.copy()
        for i, nid in enumerate(cpu_a):
            if nid == len(po[i]["candidate"]) or nid == -100:
                cpu_a[i] = -1
        O.make_equiv_action(env2, cpu_a, po, perm_idx, [[ob["viewpoint"]] for ob in po])
        po = np.array(env2._get_obs())[perm_idx]
        d = np.array([ob["distance"] for ob in po], np.float32)
        rew = np.where(ended2, 0.0, np.where(cpu_a == -1, np.where(d < 3, 2.0, -2.0), np.sign(last2 - d)))
        np.testing.assert_array_equal(plan[t]["reward"], rew.astype(np.float32))
        np.testing.assert_array_equal(plan[t]["mask"], (~ended2).astype(np.float32))
        last2 = d
        ended2 = ended2 | (cpu_a == -1)
        if ended2.all():
            break
    assert len(plan) == t + 1
    np.testing.assert_array_equal(ended, ended2)
    assert [ob["viewpoint"] for ob in final_obs] == [ob["viewpoint"] for ob in po]


def test_train_graph_slot_pads():
    """Captured training steps pad their static inputs so one slot serves every batch of a step index:
    candidates to 16, 32, 64, ...; the instruction context to --maxInput tokens rounded up to 16
    (agent_dg.Seq2SeqAgent._slot_pads)."""
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "2", "--maxAction", "5"])
    from dasa_amd.r2r.agent_dg import Seq2SeqAgent
    L0 = -(-param.args.maxInput // 16) * 16
    assert Seq2SeqAgent._slot_pads(3, 7) == (16, L0)
    assert Seq2SeqAgent._slot_pads(16, L0) == (16, L0)
    assert Seq2SeqAgent._slot_pads(17, 1) == (32, L0)
    assert Seq2SeqAgent._slot_pads(33, 1) == (64, L0)
    assert Seq2SeqAgent._slot_pads(5, L0 + 3)[1] == L0 + 16      # longer than --maxInput: its own extent


def test_synth_back_teacher_is_a_candidate_or_here():
    """env.py:348: back_teacher is the next viewpoint on the shortest path back to the episode start,
    so --pred_back's target (agent_dg._back_teacher_action) is always a candidate or the current
    viewpoint, wherever the agent stands."""
    import numpy as np
    from dasa_amd.r2r import param
    param.readme_train(["--d_vl_layers", "1", "--batchSize", "4", "--maxAction", "5"])
    from dasa_amd.synth import SynthR2RBatch, SynthWorld
    env = SynthR2RBatch(SynthWorld(16, 0, 3), 4, seed=33, mode="goal", instr_len=80, variable_len=True)
    env.reset()
    rng = np.random.default_rng(0)
    for _ in range(8):
        for sim in env.env.sims:
            sim.vp = int(rng.integers(16))
        for ob in env._get_obs():
            assert ob["back_teacher"] == ob["viewpoint"] or any(
                c["viewpointId"] == ob["back_teacher"] for c in ob["candidate"]), ob["viewpoint"]


def test_copy_layout_collapse():
    """ops._copy_layout: the joint (n0, n1, inner, strides) of a copy pair — contiguous dims merged only
    where both sides are contiguous, at most three levels (a strided inner dim becomes 1-element rows), else None."""
    import torch
    from dasa_amd.ops import _copy_layout
    s = torch.zeros(20, 96, 2048)
    assert _copy_layout(torch.zeros(20, 80, 2048), s[:, :80]) == (1, 20, 163840, 0, 163840, 0, 196608)
    assert _copy_layout(torch.zeros(20), torch.zeros(20)) == (1, 1, 20, 0, 0, 0, 0)
    assert _copy_layout(torch.zeros(()), torch.zeros(())) == (1, 1, 1, 0, 0, 0, 0)
    assert _copy_layout(torch.zeros(20, 5).t(), torch.zeros(5, 20)) == (5, 20, 1, 1, 5, 20, 1)
    assert _copy_layout(torch.zeros(3, 5, 7, 9)[:, 1:4, :, :8], torch.zeros(3, 3, 7, 8)) == (3, 21, 8, 315, 9, 168, 8)
    assert _copy_layout(torch.zeros(2, 3, 4, 5)[:, :, :, ::2], torch.zeros(2, 3, 4, 3)) == (24, 3, 1, 5, 2, 3, 1)
    assert _copy_layout(torch.zeros(3, 4, 5, 6)[:, ::2, ::2, ::2], torch.zeros(3, 2, 3, 3)) is None


def test_graph_captures_run_with_gc_disabled(monkeypatch):
    """VERDICT r05 hygiene: a Python garbage collection during a global-mode stream capture runs finalizers
    whose HIP calls abort the capture (r05, `_no_gc` in dasa_amd/graph.py). (1) graph._graph — the capture
    helper of every StepGraphs / AutogradGraphs capture — keeps GC off from capture_begin to capture_end
    whatever its caller does (capture_begin / the body / capture_end record gc.isenabled() through a fake
    graph); (2) every other capture site in the package (torch.cuda.graph / capture_begin outside _graph)
    sits in a `with` whose items enter _no_gc() first."""
    import ast
    import contextlib
    import gc
    from dasa_amd import graph
    seen = []

    class FakeGraph:
        def capture_begin(self, *a, **k):
            seen.append(("begin", gc.isenabled()))

        def capture_end(self):
            seen.append(("end", gc.isenabled()))
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(torch.cuda, "stream", lambda s=None: contextlib.nullcontext())
    gc.enable()
    with graph._graph(FakeGraph()):
        seen.append(("body", gc.isenabled()))
    assert seen == [("begin", False), ("body", False), ("end", False)], seen
    assert gc.isenabled()
    with pytest.raises(RuntimeError):                 # restored on an exception inside the capture too
        with graph._graph(FakeGraph()):
            raise RuntimeError("capture failed")
    assert gc.isenabled()

    pkg = os.path.join(ROOT, "dasa_amd")
    bad, sites = [], 0
    for fn in sorted(os.listdir(pkg)) + ["r2r/" + f for f in sorted(os.listdir(os.path.join(pkg, "r2r")))]:
        if not fn.endswith(".py"):
            continue
        tree = ast.parse(open(os.path.join(pkg, fn)).read())
        helper = [n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "_graph"]
        inside_helper = {id(c) for h in helper for c in ast.walk(h)}
        for node in ast.walk(tree):
            if not isinstance(node, ast.With):
                continue
            funcs = [ast.unparse(it.context_expr.func) if isinstance(it.context_expr, ast.Call) else ""
                     for it in node.items]
            for i, f in enumerate(funcs):
                if f in ("_graph", "graph._graph", "torch.cuda.graph"):
                    sites += 1
                    if f != "torch.cuda.graph" or id(node) in inside_helper:
                        continue           # the helper itself disables GC
                    if "_no_gc" not in [g.split(".")[-1] for g in funcs[:i]]:
                        bad.append((fn, node.lineno, f))
        for node in ast.walk(tree):
            if isinstance(node, ast.Call) and ast.unparse(node.func).endswith("capture_begin") \
                    and id(node) not in inside_helper:
                bad.append((fn, node.lineno, "capture_begin outside graph._graph"))
    assert sites >= 4, sites
    assert not bad, bad


def test_graph_param_watch_tracks_parameter_changes():
    """graph._ParamWatch (the finetune VL region's parameter key, flattened once instead of a module walk per
    call) equals the walk's key and changes with a re-assigned Parameter, a storage swap, a replaced
    submodule and a parameter added to a submodule - not with an in-place update (read by the replays)."""
    import torch.nn as nn
    from dasa_amd.graph import _ParamWatch

    class Att(nn.Module):
        def __init__(self):
            super().__init__()
            self.q, self.k, self.ln = nn.Linear(8, 8), nn.Linear(8, 8), nn.LayerNorm(8)

    mods = [nn.ModuleList([Att() for _ in range(3)]), nn.Linear(4, 4)]
    walk = lambda: tuple((id(p), p.data_ptr()) for m in mods for p in m.parameters())   # noqa: E731
    w = _ParamWatch(mods)
    k0 = w.key()
    assert k0 == walk() and w.key() == k0
    with torch.no_grad():
        mods[0][0].q.weight.add_(1.0)
    assert w.key() == k0
    mods[0][1].q.weight = nn.Parameter(torch.randn(8, 8))
    k1 = w.key()
    assert k1 != k0 and k1 == walk()
    mods[0][2] = Att()
    k2 = w.key()
    assert k2 != k1 and k2 == walk()
    mods[0][2].extra = nn.Parameter(torch.randn(3))
    k3 = w.key()
    assert len(k3) == len(k2) + 1 and sorted(k3) == sorted(walk())
    mods[0][0].q.weight.data = torch.randn(8, 8)
    assert w.key() != k3
