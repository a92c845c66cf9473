"""hipGraph capture of forward-only sub-steps of the rollout (BASELINE north star: "agent_dg.py
rollout inner loop, hipGraph-captured step").

A decision step of `Seq2SeqAgent.vl_rollout` (agent_dg.py:725-936) launches ~100 kernels for the
vision encoder and the d_vl_layers LXRT cross-attention layers (vilmodel.py:1067-1095, 1014-1064).
In the README training configuration those layers are not trained (update_add_layer=False,
vilmodel.py:1408-1410), so they run without autograd, and in evaluation nothing on the step needs
autograd. `StepGraphs` captures such a region once per input shape into a HIP graph (torch.cuda.CUDAGraph
over torch's HIP streams, including the LXRT side stream the region forks and joins) and replays it:
one host call per step instead of ~100 Python-level launches.

Dropout inside a captured region stays random per replay: the region is captured with the library's
device seed source set (include/dasa_hip.h dasa_set_seed_source), the graph's first node bumps that
counter (dasa_seed_bump), and every captured dropout kernel keys its mask on (host seed, counter).

Inputs are copied into the graph's static input buffers before a replay; outputs are cloned out of
the static output buffers (the bi-LSTM that consumes them keeps its input for the deferred backward,
and the next replay overwrites the static buffers). A captured region is re-captured when any
parameter of the modules it reads changes (data pointer or in-place version), e.g. after load_state_dict.
"""
import contextlib
import ctypes
import gc
import os

import torch

from . import _lib
from . import prof

from . import debug as _debug
# DASA_CHECK_FINITE (dasa_amd/debug.py) synchronises after every op: no capture / replay then
ENABLED = os.environ.get("DASA_GRAPH", "1") != "0" and not _debug.active()
_NESTED = [0]    # > 0 while an enclosing region is being warmed up / captured: inner regions run inline


@contextlib.contextmanager
def _no_gc():
    """No Python garbage collection while a stream is being captured: a collection there runs finalizers of
    unrelated garbage (an earlier rollout's events or graphs in a reference cycle) whose HIP calls are not
    permitted during a global-mode capture — the process aborted that way once in r05 (an MHA launch of the
    VL-stack capture, `tests_r05d.log`). torch.cuda.graph collects once before the capture begins."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


@contextlib.contextmanager
def _graph(g, pool=None, stream=None):
    """torch.cuda.graph without its torch.cuda.empty_cache(): that call returns every cached block to the
    driver, so the allocations after each capture go back to hipMalloc — with a capture per new slot of a
    small-batch finetune rollout (cfg4: candidate blocks / steps first seen in later iterations) the
    release-and-reallocate cycle cost up to 155 ms in one iteration (r05 trace). The device is synchronised
    and the capture runs in torch's global error mode on `stream`, as torch.cuda.graph does — with Python's
    garbage collection off throughout (_no_gc), whatever the caller does (tests/test_host_cpu.py)."""
    torch.cuda.synchronize()
    with _no_gc(), torch.cuda.stream(stream):
        g.capture_begin(*(() if pool is None else (pool,)), capture_error_mode="global")
        try:
            yield
        finally:
            g.capture_end()


def capturing():
    """True while a StepGraphs region is being captured (or warmed up for capture)."""
    return _NESTED[0] > 0


class _Entry:
    __slots__ = ("graph", "static_in", "static_out", "pkey")


class StepGraphs:
    """Per-owner cache of captured forward regions, keyed by the caller's shape key."""

    def __init__(self, modules):
        self.modules = list(modules)   # the nn.Modules whose parameters the region reads
        self._params = None
        self.entries = {}
        self.counter = None         # device seed counter (uint64), bumped by every replay
        self.stream = None          # warm-up + capture stream (its workspaces are the graphs' own)
        self.captures = 0
        self.replays = 0

    def _param_key(self):
        # the parameter list is walked once (module traversal costs ~0.3 ms per call); in-place
        # updates (optimizer steps, load_state_dict) bump _version, a re-assigned parameter changes
        # the identity / data pointer
        if self._params is None:
            self._params = [p for m in self.modules for p in m.parameters()]
        return tuple((id(p), p.data_ptr(), p._version) for p in self._params)

    def _capture(self, fn, inputs):
        dev = inputs[0].device
        if self.counter is None:
            self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=dev)
        static_in = tuple(torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=dev) for x in inputs)
        for s, x in zip(static_in, inputs):
            s.copy_(x)
        # warm-up on the capture stream itself: builds every lazily cached tensor (fused QKV weights,
        # and the GEMM / attention workspaces, which ops.py keys by stream) outside the capture, as
        # torch.cuda.graphs requires; the capture then reuses them (one workspace per StepGraphs)
        self.stream.wait_stream(torch.cuda.current_stream())
        _NESTED[0] += 1
        try:
            with torch.cuda.stream(self.stream), torch.no_grad():
                fn(*static_in)
            torch.cuda.current_stream().wait_stream(self.stream)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            L = _lib.lib()
            ctr = ctypes.c_void_p(self.counter.data_ptr())
            L.dasa_set_seed_source(ctr)
            try:
                with _no_gc(), _graph(g, stream=self.stream), torch.no_grad():
                    _lib.check(L.dasa_seed_bump(ctr, ctypes.c_void_p(self.stream.cuda_stream)),
                               "dasa_seed_bump")
                    out = fn(*static_in)
            finally:
                L.dasa_set_seed_source(None)
        finally:
            _NESTED[0] -= 1
        e = _Entry()
        e.graph, e.static_in, e.static_out = g, static_in, out
        e.pkey = self._param_key()
        self.captures += 1
        return e

    def run(self, key, fn, inputs):
        """fn(*inputs) -> tuple of tensors (or None), forward-only; returns fresh copies of its outputs."""
        if prof.active() or _NESTED[0]:
            # per-launch HIP-event profiling (bench.py's kernel table) runs eagerly; inside an enclosing
            # region's capture this region becomes part of that graph
            with torch.no_grad():
                return fn(*inputs)
        from . import ops
        # the GEMM numerics mode is part of what a graph captured (bf16 operands for configs[4], the
        # bf16x6 fp32 emulation switch): a replay in another mode would run the captured one
        key = (key, ops._BF16["on"], ops._EMU["on"], ops._EMU["min_rows"])
        e = self.entries.get(key)
        if e is not None and e.pkey != self._param_key():
            del self.entries[key]
            e = None
        if e is None:
            e = self._capture(fn, inputs)
            self.entries[key] = e
        from . import ops
        ops.copy_many(list(zip(inputs, e.static_in)))      # one launch for all inputs (ops.copy_many)
        e.graph.replay()
        self.replays += 1
        return _copies(e.static_out)

    def clear(self):
        self.entries.clear()


# ------------------------------------------------------------------ training-mode (autograd) regions
class _Slot:
    __slots__ = ("graph", "static_in", "static_out", "counter", "pkey", "fills", "shapes", "leaves", "bwd", "owner", "pool")


class _Bwd:
    """A captured backward of one slot for one pattern of incoming gradients: static grad-output buffers,
    the graph, its static leaf gradients, and the deferred weight-gradient products the capture queued
    (functional.defer_weight_grads: re-queued on every replay, their dz buffers rewritten by it). qrefs / qgen:
    where in the deferral queues the last queueing put its dz buffers, and in which flush generation."""
    __slots__ = ("graph", "gin", "grads", "wq", "bq", "qrefs", "qgen")


# DASA_TRAIN_GRAPH_BWD=0: a captured training region's backward runs its recorded autograd graph eagerly
BWD_GRAPH = os.environ.get("DASA_TRAIN_GRAPH_BWD", "1") != "0"


def _copies(ts):
    """Fresh copies of a replayed graph's static outputs (the next replay overwrites them), in one launch."""
    from . import ops
    with torch.no_grad():
        outs = tuple(torch.empty_like(o) if o is not None else None for o in ts)
        ops.copy_many([(o.detach(), c) for o, c in zip(ts, outs) if o is not None])
    return outs


def _lead(t, shape):
    """The leading sub-block of `t` with `shape` (a padded static input holds its input there)."""
    if tuple(t.shape) == tuple(shape):
        return t
    return t[tuple(slice(0, n) for n in shape)]


class _BridgeFn(torch.autograd.Function):
    """One replay of a captured training region, linked into the caller's autograd graph: forward
    copies the inputs into the slot's static inputs (through .data: no version bump, the captured
    autograd graph saved some of them), replays the graph and returns copies of the outputs; backward
    runs the slot's own autograd graph (recorded at capture, retained) eagerly with the slot's seed
    counter as the device seed source — so every dropout backward regenerates the masks this replay drew
    — and hands the static inputs' gradients back. Parameter gradients accumulate (or are deferred,
    functional.defer_weight_grads) inside that nested backward exactly as in an eager step."""

    @staticmethod
    def forward(ctx, slot, *inputs):
        from . import ops
        with torch.no_grad():
            pairs = []
            for i, (s, x) in enumerate(zip(slot.static_in, inputs)):
                if s is None:
                    continue
                if i in slot.fills and slot.shapes[i] != tuple(x.shape):
                    # another extent than the last input of this padded slot: rows a larger one wrote
                    # past the new extent go back to the padding value (e.g. True in a padded mask)
                    s.data.fill_(slot.fills[i])
                    slot.shapes[i] = tuple(x.shape)
                pairs.append((x.detach(), _lead(s.data, x.shape)))
            ops.copy_many(pairs)       # one launch for the step's inputs instead of one blit each
        slot.graph.replay()
        ctx.slot = slot
        ctx.shapes = [x.shape if x is not None else None for x in inputs]
        # a leaf input may keep the returned gradient as its .grad: it gets a copy, not the static buffer
        ctx.leaf = [x is not None and x.is_leaf and x.requires_grad for x in inputs]
        outs = _copies(slot.static_out)
        nd = [o for o in outs if o is not None and not o.is_floating_point()]
        if nd:
            ctx.mark_non_differentiable(*nd)
        ctx.set_materialize_grads(False)    # an output nobody differentiates arrives as None, not zeros
        return outs

    @staticmethod
    def backward(ctx, *gouts):
        slot = ctx.slot
        outs, grads = [], []
        for o, g in zip(slot.static_out, gouts):
            if o is not None and o.requires_grad and g is not None:
                outs.append(o)
                grads.append(g)
        got = {}
        mask = tuple(o is not None and o.requires_grad and g is not None for o, g in zip(slot.static_out, gouts))
        if outs and slot.leaves and BWD_GRAPH and not prof.active():
            from . import functional as DF
            # a backward captured under defer_weight_grads computes only the dz products and queues the
            # weight / bias GEMMs; a plain loss.backward() on the same slot needs the graph that computes
            # them itself — one captured graph per (gradient pattern, deferral mode)
            bkey = (mask, bool(DF._WG.active))
            bw = slot.bwd.get(bkey)
            if bw is None:
                bw = slot.bwd[bkey] = slot.owner._capture_bwd(slot, outs, grads)
            else:
                from . import ops
                if DF._WG.active and bw.qgen == DF._WG.gen and bw.qrefs:
                    # a second backward through this slot before the queued weight gradients were flushed (the
                    # bi-LSTM input-gradient continuation, functional.defer_bilstm_backward(input_grads=True),
                    # reaches a captured encoder region twice): the earlier products still read the dz buffers
                    # the replay below rewrites, so they keep copies
                    for lst, i in bw.qrefs:
                        lst[i] = lst[i].clone()
                ops.copy_many([(g.detach(), s_) for s_, g in zip(bw.gin, grads)])
                bw.graph.replay()
                _requeue(bw)
            got = {id(v): g for v, g in zip(slot.leaves, bw.grads) if g is not None}
            _accumulate_params(slot, got)
        elif outs and slot.leaves:
            L = _lib.lib()
            L.dasa_set_seed_source(ctypes.c_void_p(slot.counter.data_ptr()))
            try:
                # autograd.grad over the recorded graph's leaves (static inputs + the capture's parameter
                # aliases, AutogradGraphs._aliased): their gradients come back synced to the caller's
                # stream and the parameters' are accumulated into the real parameters' .grad there
                gl = torch.autograd.grad(outs, slot.leaves, grads, retain_graph=True, allow_unused=True)
            finally:
                L.dasa_set_seed_source(None)
            got = {id(v): g for v, g in zip(slot.leaves, gl) if g is not None}
            _accumulate_params(slot, got)
        res = []
        for s, shape, leaf in zip(slot.static_in, ctx.shapes, ctx.leaf):
            g = got.get(id(s)) if s is not None and s.requires_grad else None
            if g is not None:
                g = _lead(g, shape)
                res.append(g.clone() if leaf else g)
            else:
                res.append(None)
        return (None,) + tuple(res)


def _accumulate_params(slot, got):
    """Add the leaf gradients that belong to parameters (through their capture aliases) into .grad."""
    from . import functional as DF
    statics = {id(s) for s in slot.static_in if s is not None}
    with torch.no_grad():
        for v in slot.leaves:
            g = got.get(id(v))
            if g is None or id(v) in statics:
                continue
            v = DF.grad_target(v)
            if v.grad is None:
                v.grad = g.clone()
            else:
                v.grad.add_(g)


def _requeue(bw):
    """Queue the captured backward's deferred weight / bias gradient products again (the replay rewrote
    their dz buffers in place)."""
    from . import functional as DF
    if (bw.wq or bw.bq) and not DF._WG.active:
        raise _lib.DasaError("a backward graph captured under defer_weight_grads replayed outside it")
    bw.qrefs, bw.qgen = [], DF._WG.gen
    for W, dz, x in bw.wq:
        e = DF._WG.w.get(id(W))
        if e is None:
            e = DF._WG.w[id(W)] = [W, [], []]
        bw.qrefs.append((e[1], len(e[1])))
        e[1].append(dz)
        e[2].append(x)
    for b, dz in bw.bq:
        e = DF._WG.b.get(id(b))
        if e is None:
            e = DF._WG.b[id(b)] = [b, []]
        bw.qrefs.append((e[1], len(e[1])))
        e[1].append(dz)


def _graph_leaves(outs):
    """Every leaf tensor (AccumulateGrad node) of the autograd graph behind `outs`."""
    seen, leaves = set(), []
    stack = [o.grad_fn for o in outs if o is not None and o.grad_fn is not None]
    while stack:
        n = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        v = getattr(n, "variable", None)
        if v is not None:
            leaves.append(v)
        stack.extend(f for f, _ in n.next_functions)
    return leaves


_PARAM_WALK = os.environ.get("DASA_PARAM_WALK", "0") == "1"   # A/B: the flat-key regions walk every call


class _ParamWatch:
    """The identity / storage key of the parameters a captured region reads without walking the module
    tree per call (`module.parameters()` recurses through every submodule: ~0.3 ms for the ~130 parameters of
    the finetune's VisionEncoder + LXRT region, per decision step). The tree is flattened once into
    (container dict, name) entries - every module's `_parameters` and `_modules` - and re-flattened when one
    of those dicts changed size or a child module was replaced, so a Parameter or submodule assigned anywhere
    in the tree, or a storage swap (p.data = ...), still changes the key."""

    def __init__(self, modules):
        self.modules = list(modules)
        self._flat = None

    def _flatten(self):
        mods = [mod for m in self.modules for mod in m.modules()]
        self._edges = [(mod._modules, name, child) for mod in mods for name, child in mod._modules.items()]
        self._dicts = [(d, len(d)) for mod in mods for d in (mod._modules, mod._parameters)]
        self._flat = [(mod._parameters, name) for mod in mods for name, p in mod._parameters.items() if p is not None]

    def _stale(self):
        for d, n in self._dicts:
            if len(d) != n:
                return True
        for d, name, child in self._edges:
            if d.get(name) is not child:
                return True
        return False

    def key(self):
        if self._flat is None or self._stale():
            self._flatten()
        return tuple((id(p), p.data_ptr()) for p in (d[n] for d, n in self._flat) if p is not None)


class AutogradGraphs:
    """Training-mode decision steps (agent_dg.py:725-936 with autograd on) as hipGraph
    replays. A region — e.g. the decoder step + the one-kernel policy head — is captured once per slot
    key WITH autograd recording: the capture builds the region's autograd graph over static input
    leaves, and that graph is kept. Each replay rewrites the graph-pool tensors the graph saved, so a
    slot serves ONE live step: the caller keys slots by step index, and `run` adds an occurrence
    number for keys used again before new_iteration() (the auglistener loop's GT and aug halves each
    run a teacher and a sampled rollout before one backward). Dropout / Categorical draws stay fresh
    per replay (a per-slot device seed counter, bumped by the graph's first node) and their backward
    regenerates the same masks (_BridgeFn). Parameters are read in place by the replay (optimizer
    updates need no re-capture); a re-assigned parameter (new storage) re-captures. Host cost of a
    step: the input copies and one graph launch instead of ~30 Python-level launches."""

    def __init__(self, modules, flat_key=False):
        self.modules = list(modules)
        # flat_key: the parameter key without a module walk per call (the finetune's VL region; the decision
        # step's decoder region keeps the walk: a faster host there slowed cfg2)
        self._watch = _ParamWatch(self.modules) if flat_key and not _PARAM_WALK else None
        self.slots = {}
        self.uses = {}
        self.stream = None
        self._alias = {}
        self.captures = 0
        self.captures_bwd = 0
        self.replays = 0

    def _param_key(self):
        # a Parameter object replaced on a module (module.weight = nn.Parameter(...)) changes the key as well
        # as a storage swap (p.data = ...); in-place updates are read by the replays
        if self._watch is not None:
            return self._watch.key()
        return tuple((id(p), p.data_ptr()) for m in self.modules for p in m.parameters())

    @contextlib.contextmanager
    def _aliased(self):
        """The modules' trainable parameters replaced, while a region is warmed up and captured, by alias
        leaves sharing their storage (replays read optimizer updates in place). The retained capture graph
        then holds the aliases' gradient accumulators — created on the capture stream, where the recorded
        backward produces their gradients — and not the parameters' own, which stay per-iteration nodes on
        the stream of the parameters' eager uses. One accumulator node serving both streams is what torch
        warns about (AccumulateGrad stream mismatch) and syncs the streams for. Gradients
        of an alias reach its parameter's .grad (functional.grad_target)."""
        from . import functional as DF
        swapped = []
        for m in self.modules:
            for mod in m.modules():
                for name, p in list(mod._parameters.items()):
                    if p is None or not p.requires_grad:
                        continue
                    a = self._alias.get(id(p))
                    if a is None or a.data_ptr() != p.data_ptr() or a.shape != p.shape:
                        if a is not None:
                            DF._GRAD_OF.pop(id(a), None)
                        a = torch.nn.Parameter(p.data)
                        self._alias[id(p)] = a
                        DF.set_grad_target(a, p)
                    mod._parameters[name] = a
                    swapped.append((mod, name, p))
        try:
            yield
        finally:
            for mod, name, p in swapped:
                mod._parameters[name] = p

    def new_iteration(self):
        """Every slot replayed since the last call has had its backward (or will never get one)."""
        self.uses.clear()

    def _capture(self, fn, inputs, pads):
        dev = next(x for x in inputs if x is not None).device
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=dev)
        slot = _Slot()
        # a memory pool of the slot's own, shared only by its forward and backward graphs: those replay in
        # their capture order every iteration (forward, then backward). One pool across slots would let a
        # slot captured later (a new key mid-rollout) place its saved tensors in an earlier-captured slot's
        # freed temporaries, which that slot's next replay overwrites before the backward reads them
        slot.pool = torch.cuda.graph_pool_handle()
        slot.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        slot.fills, slot.shapes = {}, {}
        static_in = []
        for i, x in enumerate(inputs):
            if x is None:
                static_in.append(None)
                continue
            shape, fill = pads.get(i, (x.shape, 0))
            s = torch.full(shape, fill, dtype=x.dtype, device=dev)    # the padding keeps its fill value
            if i in pads:
                slot.fills[i], slot.shapes[i] = fill, tuple(x.shape)
            with torch.no_grad():       # a LEAF: recorded, the copy would link the slot to x's graph
                _lead(s, x.shape).copy_(x)
            static_in.append(s.requires_grad_(x.requires_grad))
        self.stream.wait_stream(torch.cuda.current_stream())
        from . import ops
        _NESTED[0] += 1
        ops._FRESH_PLANES[0] += 1
        try:
            # warm-up on the capture stream (lazily built workspaces / caches outside the capture); its
            # autograd graph is dropped
            with self._aliased(), torch.cuda.stream(self.stream), torch.enable_grad():
                fn(*static_in)
            torch.cuda.current_stream().wait_stream(self.stream)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            L = _lib.lib()
            ctr = ctypes.c_void_p(slot.counter.data_ptr())
            L.dasa_set_seed_source(ctr)
            try:
                with self._aliased(), _no_gc(), _graph(g, pool=slot.pool, stream=self.stream), \
                        torch.enable_grad():
                    _lib.check(L.dasa_seed_bump(ctr, ctypes.c_void_p(self.stream.cuda_stream)), "dasa_seed_bump")
                    out = fn(*static_in)
            finally:
                L.dasa_set_seed_source(None)
        finally:
            _NESTED[0] -= 1
            ops._FRESH_PLANES[0] -= 1
        slot.graph, slot.static_in, slot.static_out = g, static_in, tuple(out)
        slot.leaves = _graph_leaves(slot.static_out)
        slot.bwd, slot.owner = {}, self
        slot.pkey = self._param_key()
        self.captures += 1
        return slot

    def _capture_bwd(self, slot, outs, grads):
        """Capture the slot's recorded backward (autograd.grad over its leaves) for this pattern of incoming
        gradients as a graph on the capture stream, then replay it once for the current step. Its kernels
        are a fixed sequence for a slot: replaying it costs one launch instead of the ~40 host-issued
        launches of the per-step backward (the launch-bound phase of the iteration, r05 trace). The
        dropout kernels of the backward read the slot's seed counter at run time, as the eager backward."""
        from . import functional as DF
        from . import ops
        bw = _Bwd()
        bw.gin = [g.detach().clone() for g in grads]
        wq0 = {k: len(v[1]) for k, v in DF._WG.w.items()}
        bq0 = {k: len(v[1]) for k, v in DF._WG.b.items()}
        self.stream.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        L = _lib.lib()
        _NESTED[0] += 1
        ops._FRESH_PLANES[0] += 1
        L.dasa_set_seed_source(ctypes.c_void_p(slot.counter.data_ptr()))
        try:
            with _no_gc(), _graph(g, pool=slot.pool, stream=self.stream):
                gl = torch.autograd.grad(outs, slot.leaves, bw.gin, retain_graph=True, allow_unused=True)
        finally:
            L.dasa_set_seed_source(None)
            _NESTED[0] -= 1
            ops._FRESH_PLANES[0] -= 1
        bw.graph, bw.grads = g, tuple(gl)
        bw.wq = [(e[0], dz, x) for k, e in DF._WG.w.items() for dz, x in zip(e[1][wq0.get(k, 0):], e[2][wq0.get(k, 0):])]
        bw.bq = [(e[0], dz) for k, e in DF._WG.b.items() for dz in e[1][bq0.get(k, 0):]]
        bw.qgen = DF._WG.gen     # where the capture queued its dz buffers (see _BridgeFn.backward)
        bw.qrefs = ([(e[1], i) for k, e in DF._WG.w.items() for i in range(wq0.get(k, 0), len(e[1]))]
                    + [(e[1], i) for k, e in DF._WG.b.items() for i in range(bq0.get(k, 0), len(e[1]))])
        g.replay()          # the capture launched nothing: compute this step's gradients now
        self.captures_bwd += 1
        return bw

    def run(self, key, fn, inputs, pads=None):
        """fn(*inputs) -> tuple of tensors / None, recorded with autograd; returns the outputs linked to
        `inputs` for backward. pads: {input index: (static shape >= the input's, fill value of the
        padding)}; the input is copied into the leading sub-block on every replay."""
        from . import ops
        key = (key, ops._BF16["on"], ops._EMU["on"], ops._EMU["min_rows"])
        n = self.uses.get(key, 0)
        self.uses[key] = n + 1
        skey = (key, n)
        slot = self.slots.get(skey)
        if slot is not None and slot.pkey != self._param_key():
            del self.slots[skey]
            slot = None
        if slot is None:
            slot = self._capture(fn, inputs, pads or {})
            self.slots[skey] = slot
        self.replays += 1
        return _BridgeFn.apply(slot, *inputs)

    def clear(self):
        from . import functional as DF
        self.slots.clear()
        self.uses.clear()
        for a in self._alias.values():
            DF._GRAD_OF.pop(id(a), None)
        self._alias.clear()
