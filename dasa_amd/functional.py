"""Autograd wrappers: each forward/backward is a short sequence of libdasa_hip.so kernels.

These are the differentiable building blocks of the reference-API modules in dasa_amd.r2r. Only
the tensors a backward actually needs are saved, and nothing is saved when no input requires grad.
Parameters are held as ctx attributes (ctx.params, a _Kept tuple), not saved tensors: a captured
training step (graph.AutogradGraphs) keeps its autograd graph across optimizer steps, whose in-place
parameter updates would otherwise fail the saved-tensor version check; the backward reads the parameters
as they are at backward time, which in every training loop here is before the optimizer step. Outside a
capture the same version check runs on first access in the backward (_Kept).
"""
import contextlib
import weakref

import numpy as np
import torch

from . import ops

class _SeedStream:
    """Host stream of 63-bit seeds for the counter-RNG kernels (dropout, feature dropout, Categorical
    draws). It follows torch's seed: derived lazily from torch.initial_seed() at first use and again
    whenever torch.manual_seed() changed it (train.py:521 seeds after this module is imported), mixed
    with a per-rank salt (dp.attach) so data-parallel ranks draw different masks and actions."""

    def __init__(self):
        self.rng = None
        self.torch_seed = None
        self.salt = 0
        self.explicit = False

    def get(self):
        s = torch.initial_seed()
        if self.rng is None or (not self.explicit and s != self.torch_seed):
            self.torch_seed = s
            self.rng = np.random.default_rng([s & 0xFFFFFFFFFFFFFFFF, self.salt])
            self.explicit = False
        return self.rng


_SEEDS = _SeedStream()


class _Kept(tuple):
    """The parameters a backward reads (ctx.params), with the in-place guard save_for_backward would
    give them: their _version at forward time is recorded (not inside a hipGraph capture — a captured
    training step's backward legitimately runs after optimizer updates of the same storage), and the
    first access in the backward raises if a parameter was modified in place since."""

    def __new__(cls, params):
        t = super().__new__(cls, params)
        t._ver = None if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing() else \
            tuple(None if q is None else q._version for q in params)
        return t

    def _check(self):
        ver = self._ver
        if ver is not None:
            self._ver = None           # once per backward
            for q, v in zip(tuple.__iter__(self), ver):
                if q is not None and q._version != v:
                    raise RuntimeError("one of the parameters needed for gradient computation has been modified "
                                       f"by an inplace operation: {tuple(q.shape)} is at version {q._version}; "
                                       f"expected version {v} (dasa_amd.functional)")

    def __getitem__(self, i):
        self._check()
        return tuple.__getitem__(self, i)

    def __iter__(self):
        self._check()
        return tuple.__iter__(self)


def new_seed():
    """A fresh 63-bit seed for the counter-RNG dropout kernels."""
    return int(_SEEDS.get().integers(1, 2**63 - 1))


def reseed(seed):
    """Pin the seed stream to `seed` (mixed with the rank salt) until torch's seed changes."""
    _SEEDS.rng = np.random.default_rng([int(seed) & 0xFFFFFFFFFFFFFFFF, _SEEDS.salt])
    _SEEDS.torch_seed = torch.initial_seed()
    _SEEDS.explicit = True


def set_rank_salt(rank):
    """Data-parallel ranks: make the seed stream rank-specific (restarts it from torch's seed)."""
    _SEEDS.salt = int(rank) + 1 if rank else 0
    _SEEDS.rng = None
    _SEEDS.explicit = False


def _flat(t):
    return t.reshape(-1, t.shape[-1])


# ------------------------------------------------------------------- deferred weight gradients
class _WGradDeferral:
    """Weight / bias gradients of one backward pass, computed once per parameter at the end.

    The rollout applies the decoder and critic linears once per step (agent_dg.py:725-993), so the
    backward of one optimizer step produces ~70 skinny products dW_t = dY_t^T X_t (B = 20 rows each)
    per weight, each followed by an autograd accumulation into .grad. Under defer_weight_grads() the
    Functions below queue (dY_t, X_t) instead and flush_weight_grads() computes
    dW = [dY_1; ...; dY_T]^T [X_1; ...; X_T] as ONE MFMA GEMM (K = T*B) per weight, added into .grad.
    Same sums, in a different order; input / state gradients still flow step by step."""

    def __init__(self):
        self.active = False
        self.w = {}      # id(param) -> [param, [dY], [X]]
        self.b = {}      # id(param) -> [param, [dY]]
        self.gen = 0     # flush count: a captured backward replayed twice in one generation clones its queued dY


_WG = _WGradDeferral()


@contextlib.contextmanager
def defer_weight_grads():
    prev = _WG.active
    _WG.active = True
    try:
        yield
    finally:
        _WG.active = prev


# capture-time parameter aliases (graph.AutogradGraphs): id(alias) -> (weakref(alias), weakref(parameter)),
# the parameter whose .grad the alias's gradients feed (weak both ways: a dead alias's id may be reused)
_GRAD_OF = {}


def set_grad_target(alias, p):
    _GRAD_OF[id(alias)] = (weakref.ref(alias), weakref.ref(p))


def grad_target(p):
    e = _GRAD_OF.get(id(p))
    if e is None or e[0]() is not p:
        return p
    q = e[1]()
    return p if q is None else q


def _wgrad(W, dz, x):
    """dW = dz^T x (both [rows, .]), or queued while weight gradients are deferred (returns None)."""
    if _WG.active:
        W = grad_target(W)
        e = _WG.w.get(id(W))
        if e is None:
            e = _WG.w[id(W)] = [W, [], []]
        e[1].append(dz)
        e[2].append(x)
        return None
    return ops.matmul_tn(dz, x)


def _bgrad(b, dz):
    """db = column sums of dz, or queued while weight gradients are deferred (returns None)."""
    if _WG.active:
        b = grad_target(b)
        e = _WG.b.get(id(b))
        if e is None:
            e = _WG.b[id(b)] = [b, []]
        e[1].append(dz)
        return None
    return ops.colsum(dz)


class _SumTermsFn(torch.autograd.Function):
    """sum_t x_t of 0-dim tensors as ONE colsum GEMM over their stack (the rollout's per-step loss terms,
    agent_dg.py:871-872 `total_forth_loss += ce`). The per-step `+=` ran torch's float add kernel, which carries
    packed-FP32 VALU, while the language pipe's GEMMs run on another stream."""

    @staticmethod
    def forward(ctx, *ts):
        x = torch.stack([t.detach().reshape(()) for t in ts]).view(-1, 1)
        ctx.n = len(ts)
        return ops.colsum(x).view(())

    @staticmethod
    def backward(ctx, g):
        return (g,) * ctx.n


def sum_terms(ts):
    return _SumTermsFn.apply(*ts)


def row_sums(x):
    """[T, B] -> [T] row sums as one GEMM with a ones vector (no autograd; logging)."""
    ones = torch.ones(x.shape[1], 1, dtype=torch.float32, device=x.device)
    return ops.matmul_nn(x.float().contiguous(), ones).view(-1)


def _cat_rows(ts):
    ts = [_flat(t) for t in ts]
    return ts[0] if len(ts) == 1 else torch.cat(ts, 0)


def flush_weight_grads():
    """Run the queued weight / bias gradient products into .grad (one GEMM / column sum each)."""
    w, b = _WG.w, _WG.b
    _WG.w, _WG.b = {}, {}
    _WG.gen += 1
    for P, dzs, xs in w.values():
        dz, x = _cat_rows(dzs), _cat_rows(xs)
        if P.grad is None:
            P.grad = ops.matmul_tn(dz, x)
        else:
            ops.matmul_tn(dz, x, out=P.grad, beta=1.0)
    for P, dzs in b.values():
        dz = _cat_rows(dzs)
        if P.grad is None:
            P.grad = ops.colsum(dz)
        else:
            ops.colsum(dz, out=P.grad, beta=1.0)


# ------------------------------------------------------------------------------------ Linear
class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b) (nn.Linear + activation), one fused MFMA GEMM."""

    @staticmethod
    def forward(ctx, x, W, b, act):
        ctx.act = act
        ctx.has_b = b is not None
        ctx.params = _Kept((W, b))
        need = any(ctx.needs_input_grad)
        if need and x.dtype == torch.bfloat16:
            # a bf16 activation (the bf16 GELU hand-off of configs[4]'s matmul mode) reaching a layer whose
            # weight still trains: the fp32 weight-gradient GEMM takes the same values widened to fp32
            x = x.float()
        if need and act == "gelu":
            z = ops.linear(x, W, b)
            y = ops.act_fwd(z, "gelu")
            ctx.save_for_backward(x, z)
        else:
            y = ops.linear(x, W, b, act=act)
            if need:
                ctx.save_for_backward(x, y if act is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, s = ctx.saved_tensors
        W = ctx.params[0]
        N = W.shape[0]
        dz = _flat(dy.contiguous())
        if ctx.act is not None:
            dz = ops.act_bwd(s, dz, ctx.act).view(-1, N)
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.matmul_nn(dz, W).view(x.shape)
        if ctx.needs_input_grad[1]:
            dW = _wgrad(ctx.params[0], dz, _flat(x))
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = _bgrad(ctx.params[1], dz)
        return dx, dW, db, None


def linear(x, W, b=None, act=None):
    if torch.is_grad_enabled() and (x.requires_grad or W.requires_grad or (b is not None and b.requires_grad)):
        return LinearFn.apply(x, W, b, act)
    return ops.linear(x, W, b, act=act)


# ----------------------------------------------------------------------------------- Dropout
class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.p, ctx.seed = p, seed
        return ops.dropout(x, p, seed)

    @staticmethod
    def backward(ctx, dy):
        return ops.dropout(dy.contiguous(), ctx.p, ctx.seed), None, None


def dropout(x, p, training):
    if not training or p <= 0:
        return x
    return DropoutFn.apply(x, p, new_seed())


class FeatDropFn(torch.autograd.Function):
    """BAttnDecoderLSTM.drop_env on the RGB columns of a [.., 2176] view block (model.py:506-508, 556-557);
    the 128 angle columns pass through."""

    @staticmethod
    def forward(ctx, feat, p, seed, n_angle):
        ctx.p, ctx.seed, ctx.na = p, seed, n_angle
        out = torch.empty_like(feat)
        F = feat.shape[-1] - n_angle
        ops.dropout(feat[..., :F], p, seed, out=out[..., :F])
        ops.copy2d(feat[..., F:], out[..., F:])
        return out

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        F = dy.shape[-1] - ctx.na
        ops.dropout(dy[..., :F], ctx.p, ctx.seed, out=dx[..., :F])
        ops.copy2d(dy[..., F:], dx[..., F:])
        return dx, None, None, None


def feat_drop(feat, p, training, n_angle=128):
    if not training or p <= 0:
        return feat
    return FeatDropFn.apply(feat, p, new_seed(), n_angle)


# --------------------------------------------------------------------- depth-guided AdaIN
class AdaFeatFn(torch.autograd.Function):
    """df = f with f[..., :F] replaced by sigmoid(a_fc(d[..., :F])) * f[..., :F] (* shared noise)
    (agent_dg.py:728, 764-768, 780-785; DGAdaChannel.forward :1525-1547)."""

    @staticmethod
    def forward(ctx, f, d, W, b, noise, n_angle):
        F = f.shape[-1] - n_angle
        out = torch.empty(f.shape, dtype=torch.float32, device=f.device)
        need = any(ctx.needs_input_grad)
        f_rgb, d_rgb = f[..., :F], d[..., :F]
        if need:
            s = ops.linear(d_rgb, W, b, act="sigmoid")
            ops.ada_gate_fwd(s, f_rgb, noise, out[..., :F])
            ctx.save_for_backward(f, d, s, noise)
        else:
            ops.linear(d_rgb, W, b, act="sigmoid", out=out[..., :F], aux=f_rgb, colscale=noise)
        ops.copy2d(f[..., F:], out[..., F:])
        ctx.F = F
        return out

    @staticmethod
    def backward(ctx, dy):
        f, d, s, noise = ctx.saved_tensors
        F = ctx.F
        dy = dy.contiguous()
        dz = ops.ada_gate_bwd(dy[..., :F], s, f[..., :F], noise)
        dW = ops.matmul_tn(dz, d[..., :F]) if ctx.needs_input_grad[2] else None
        db = ops.colsum(dz) if ctx.needs_input_grad[3] else None
        return None, None, dW, db, None, None


def ada_feature(f, d, W, b, noise=None, n_angle=128):
    return AdaFeatFn.apply(f, d, W, b, noise, n_angle)


class AdaINMuSigmaFn(torch.autograd.Function):
    """adaptive_instance_normalization (model.py:1832-1840): per-row mu/sigma of content and style
    (unbiased variance + eps), forward dasa_adain_musigma_fwd, backward dasa_adain_musigma_bwd."""

    @staticmethod
    def forward(ctx, content, style, eps):
        ctx.eps = eps
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(content, style)
        return ops.adain_musigma(content, style, eps=eps)

    @staticmethod
    def backward(ctx, dout):
        content, style = ctx.saved_tensors
        dc, ds = ops.adain_musigma_bwd(content, style, dout.contiguous(), ctx.needs_input_grad[0],
                                       ctx.needs_input_grad[1], ctx.eps)
        return dc, ds, None


def _overlaps(a, b):
    """Do the storage byte ranges of a and b intersect (a conservative alias test)?"""
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return False
    def span(t):
        lo = t.data_ptr()
        hi = lo + sum((n - 1) * st for n, st in zip(t.shape, t.stride())) * t.element_size() + t.element_size()
        return lo, hi
    (a0, a1), (b0, b1) = span(a), span(b)
    return a0 < b1 and b0 < a1


def adain_musigma(content, style, eps=1e-5, out=None):
    if torch.is_grad_enabled() and (content.requires_grad or style.requires_grad):
        if out is not None:
            # backward reads the saved content / style; an `out` aliasing them (the agent's in-place
            # f_t[..., :F] = adain(f_t[..., :F], d_t[..., :F]), agent_dg.py:774-777) would overwrite
            # the saved values, so the Function gets private copies
            if _overlaps(out, content):
                content = content.clone()
            if _overlaps(out, style):
                style = style.clone()
        y = AdaINMuSigmaFn.apply(content, style, eps)
        if out is not None:
            out.copy_(y)
            return out
        return y
    return ops.adain_musigma(content, style, out=out, eps=eps)


# -------------------------------------------------------------------- attention heads
class ShiftAttnFn(torch.autograd.Function):
    """ShiftSoftDotAttention (model.py:318-353), output_tilde=False: returns weighted context."""

    @staticmethod
    def forward(ctx, h, feat, W_in, W_s, b_s):
        q = ops.linear(h, W_in)
        z = ops.linear(h, W_s, b_s)
        wctx, attn, shifted, wsm = ops.shift_attn_fwd(q, feat, z)
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(h, feat, q, attn, shifted, wsm)
            ctx.params = _Kept((W_in, W_s, b_s))
        ctx.mark_non_differentiable(attn)
        ctx.set_materialize_grads(False)     # no zero-filled gradient for the attention output
        return wctx, attn

    @staticmethod
    def backward(ctx, dwctx, _dattn):
        if dwctx is None:
            return None, None, None, None, None
        h, feat, q, attn, shifted, wsm = ctx.saved_tensors
        W_in, W_s = ctx.params[0], ctx.params[1]
        dq, dfeat, dz = ops.shift_attn_bwd(q, feat.contiguous(), attn, shifted, wsm, dwctx.contiguous(),
                                           want_dctx=ctx.needs_input_grad[1])
        dh = dWin = dWs = dbs = None
        if ctx.needs_input_grad[0]:
            dh = ops.matmul_nn(dq, W_in)
            ops.matmul_nn(dz, W_s, out=dh, beta=1.0)
        if ctx.needs_input_grad[2]:
            dWin = _wgrad(ctx.params[0], dq, h)
        if ctx.needs_input_grad[3]:
            dWs = _wgrad(ctx.params[1], dz, h)
        if ctx.needs_input_grad[4]:
            dbs = _bgrad(ctx.params[2], dz)
        return dh, dfeat, dWin, dWs, dbs


class SoftDotTildeFn(torch.autograd.Function):
    """SoftDotAttention with output_tilde=True (model.py:268-296): tanh(W_out [wctx, h]), alpha."""

    @staticmethod
    def forward(ctx, h, c, mask, W_in, W_out):
        q = ops.linear(h, W_in)
        _, probs, wctx = ops.softdot_fwd(q, c, mask)
        B, D = wctx.shape
        cat = torch.empty(B, D + h.shape[1], dtype=torch.float32, device=h.device)
        ops.copy2d(wctx, cat[:, :D])
        ops.copy2d(h, cat[:, D:])
        y = ops.linear(cat, W_out, act="tanh")
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(h, c, q, probs, cat, y)
            ctx.params = _Kept((W_in, W_out))
        ctx.mark_non_differentiable(probs)
        ctx.set_materialize_grads(False)     # no zero-filled gradient for the attention weights
        return y, probs

    @staticmethod
    def backward(ctx, dy, _dalpha):
        if dy is None:
            return None, None, None, None, None
        h, c, q, probs, cat, y = ctx.saved_tensors
        W_in, W_out = ctx.params
        dz = ops.act_bwd(y, dy.contiguous(), "tanh")
        D = c.shape[2]
        dh = dc = dWin = dWout = None
        if ctx.needs_input_grad[4]:
            dWout = _wgrad(ctx.params[1], dz, cat)
        dcat = ops.matmul_nn(dz, W_out)
        dq, dc = ops.softdot_bwd(q, c.contiguous(), probs, dwctx=dcat[:, :D].contiguous(),
                                 want_dctx=ctx.needs_input_grad[1])
        if ctx.needs_input_grad[0]:
            dh = dcat[:, D:].contiguous()
            ops.matmul_nn(dq, W_in, out=dh, beta=1.0)
        if ctx.needs_input_grad[3]:
            dWin = _wgrad(ctx.params[0], dq, h)
        return dh, dc, None, dWin, dWout


class SoftDotFn(torch.autograd.Function):
    """SoftDotAttention with output_tilde=False in general (model.py:268-296): the weighted context and
    the attention — the masked softmax, or with want_scores the raw scores with -inf where masked (the
    reference's aliased `logit`, masked in place). wctx and the scores are differentiable (dasa_softdot_bwd
    takes dwctx and dscores); the softmax output is returned detached (no caller differentiates it)."""

    @staticmethod
    def forward(ctx, h, c, mask, W_in, want_scores):
        q = ops.linear(h, W_in)
        scores, probs, wctx = ops.softdot_fwd(q, c, mask)
        if mask is not None and want_scores:
            scores = scores.masked_fill(mask.bool(), -float("inf"))
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(h, c, q, probs, mask.bool() if mask is not None else None)
            ctx.params = _Kept((W_in,))
        ctx.want_scores = want_scores
        if not want_scores:
            ctx.mark_non_differentiable(probs)
        ctx.set_materialize_grads(False)     # backward takes None for an output without gradient
        return wctx, (scores if want_scores else probs)

    @staticmethod
    def backward(ctx, dwctx, dattn):
        h, c, q, probs, mask = ctx.saved_tensors
        W_in = ctx.params[0]
        ds = None
        if ctx.want_scores and dattn is not None:
            ds = dattn.masked_fill(mask, 0.0) if mask is not None else dattn
        if dwctx is None:
            dwctx = torch.zeros_like(q)
        dq, dc = ops.softdot_bwd(q, c.contiguous(), probs, dwctx=dwctx.contiguous(),
                                 dscores=ds.contiguous() if ds is not None else None,
                                 want_dctx=ctx.needs_input_grad[1])
        dh = ops.matmul_nn(dq, W_in) if ctx.needs_input_grad[0] else None
        dW = _wgrad(W_in, dq, h) if ctx.needs_input_grad[3] else None
        return dh, dc, None, dW, None


class CandLogitFn(torch.autograd.Function):
    """SoftDotAttention with output_prob=False, output_tilde=False: the raw candidate logits
    (model.py:276-280, 289-290; used as the policy logits at model.py:559)."""

    @staticmethod
    def forward(ctx, h, cand, W_in):
        q = ops.linear(h, W_in)
        scores, _, _ = ops.softdot_fwd(q, cand, None, want_probs=False, want_wctx=False)
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(h, cand, q, scores)
            ctx.params = _Kept((W_in,))
        return scores

    @staticmethod
    def backward(ctx, dlogit):
        h, cand, q, scores = ctx.saved_tensors
        W_in = ctx.params[0]
        # ds = dscores exactly when no dwctx flows (probs operand unused)
        dq, dcand = ops.softdot_bwd(q, cand.contiguous(), scores, dscores=dlogit.contiguous(),
                                    want_dctx=ctx.needs_input_grad[1])
        dh = ops.matmul_nn(dq, W_in) if ctx.needs_input_grad[0] else None
        dW = _wgrad(ctx.params[0], dq, h) if ctx.needs_input_grad[2] else None
        return dh, dcand, dW


# ------------------------------------------------------------------------------ policy head
class PolicyHeadFn(torch.autograd.Function):
    """agent_dg.py:832-880 in one kernel: logit.masked_fill(cand_mask, -inf) -> CrossEntropyLoss(sum,
    ignore_index) against the teacher target, and the action (argmax, or a Categorical draw) with its
    entropy and log-probability (Categorical(probs)'s clamped log-pmf in sample / forced mode, the
    exact log_softmax in argmax mode). Returns (ce_sum, entropy [B], logp_action [B], action [B] int64)."""

    @staticmethod
    def forward(ctx, logit, cand_len_i32, target, mode, seed, ignore_index, forced=None):
        ce, ent, lpa, action, logp = ops.policy_head_fwd(logit, cand_len_i32, target, mode, seed, ignore_index,
                                                         forced)
        ctx.save_for_backward(logp, cand_len_i32, target, action, ent)
        ctx.ignore, ctx.mode = ignore_index, mode
        if action is None:   # teacher mode: no action drawn
            action = torch.empty(0, dtype=torch.int64, device=logit.device)
        ctx.mark_non_differentiable(action)
        # the kernel takes a null pointer for a loss term without gradient (a teacher rollout's entropy and
        # log-probability): no zero-filled [B] tensors per step
        ctx.set_materialize_grads(False)
        return ce, ent, lpa, action

    @staticmethod
    def backward(ctx, d_ce, d_ent, d_lpa, _d_action):
        if d_ce is None and d_ent is None and d_lpa is None:
            return None, None, None, None, None, None, None
        logp, lens, target, action, ent = ctx.saved_tensors
        if action is not None and action.numel() == 0:
            action = None
        dlogit = ops.policy_head_bwd(logp, lens, target, action, ent,
                                     d_ce.reshape(1).contiguous() if d_ce is not None else None,
                                     d_lpa.contiguous() if d_lpa is not None else None,
                                     d_ent.contiguous() if d_ent is not None else None, ctx.mode, ctx.ignore)
        return dlogit, None, None, None, None, None, None


def policy_head(logit, cand_len_i32, target, mode, ignore_index=-100, forced=None):
    """mode teacher / argmax / sample; "forced" = sample with `forced` [B] as the drawn action."""
    seed = new_seed() if mode == "sample" else 0
    return PolicyHeadFn.apply(logit, cand_len_i32, target, mode, seed, ignore_index, forced)


# ----------------------------------------------------------------------------------- LSTM
class LSTMCellFn(torch.autograd.Function):
    """nn.LSTMCell on the concatenated input [a_emb, attn_feat] (model.py:513-514)."""

    @staticmethod
    def forward(ctx, a_emb, x2, h, c, W_ih, W_hh, b_ih, b_hh):
        B, E = a_emb.shape
        xcat = torch.empty(B, E + x2.shape[1], dtype=torch.float32, device=a_emb.device)
        ops.copy2d(a_emb, xcat[:, :E])
        ops.copy2d(x2, xcat[:, E:])
        gates = ops.linear(xcat, W_ih, b_ih)
        ops.linear(h, W_hh, b_hh, out=gates, beta=1.0)
        need = any(ctx.needs_input_grad)
        h1, c1, act = ops.lstm_cell_fwd(gates, c, save=need)
        if need:
            ctx.save_for_backward(xcat, h, c, c1, act)
            ctx.params = _Kept((W_ih, W_hh, b_ih, b_hh))
        ctx.E = E
        ctx.set_materialize_grads(False)     # the cell kernel takes null dh / dc (the last step's c1)
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        if dh1 is None and dc1 is None:
            return (None,) * 8
        xcat, h, c, c1, act = ctx.saved_tensors
        W_ih, W_hh = ctx.params[0], ctx.params[1]
        dgates, dc_prev = ops.lstm_cell_bwd(act, c, c1, dh1, dc1)
        E = ctx.E
        n = ctx.needs_input_grad
        da = dx2 = dh = dW_ih = dW_hh = db = None
        if n[0] or n[1]:
            dxcat = ops.matmul_nn(dgates, W_ih)
            da = dxcat[:, :E].contiguous() if n[0] else None
            dx2 = dxcat[:, E:].contiguous() if n[1] else None
        if n[2]:
            dh = ops.matmul_nn(dgates, W_hh)
        P = ctx.params
        if n[4]:
            dW_ih = _wgrad(P[0], dgates, xcat)
        if n[5]:
            dW_hh = _wgrad(P[1], dgates, h)
        db_ih = db_hh = None
        if _WG.active:
            if n[6]:
                _bgrad(P[2], dgates)
            if n[7]:
                _bgrad(P[3], dgates)
        elif n[6] or n[7]:
            db_ih = db_hh = ops.colsum(dgates)
        return da, dx2, dh, (dc_prev if n[3] else None), dW_ih, dW_hh, db_ih, db_hh


class _BpttDeferral:
    """Batches the bi-LSTM BPTT of every encoder call of one backward pass.

    The rollout runs the DicEncoder once per step (agent_dg.py:725-936), so one optimizer step holds
    ~70 independent bi-LSTM graphs whose backward passes share nothing but the weights. When the
    sequence input needs no gradient (its BERT/LXRT producer is detached, the README train config),
    BiLSTMFn.backward only queues its saved tensors and the incoming gradients; flush() then runs ONE
    recurrence over all queued sequences (B = steps x batch: an MFMA GEMM per timestep instead of 70
    latency-bound recurrences) and adds dW_ih / dW_hh / db into the parameters' .grad. Same sums as
    the per-call backward, in a different order.

    input_grads=True (r05; the finetune config, --d_update_add_layer True, where the LXRT output feeding the
    bi-LSTM trains): the calls whose input needs a gradient are queued too — their backward returns no input
    gradient, which stops the first backward pass at the bi-LSTM input — and flush() computes every call's
    dx from the same batched recurrence (dx = dgates_f W_ih_f + dgates_b W_ih_b over all queued rows) and
    continues the backward from the queued inputs (torch.autograd.backward(inputs, dx)) through the LXRT /
    VisionEncoder stacks. The first pass must retain its graph (the stopped branches run later)."""

    def __init__(self):
        self.active = False
        self.dx = False
        self.items = []


_BPTT = _BpttDeferral()


@contextlib.contextmanager
def defer_bilstm_backward(input_grads=False):
    prev = (_BPTT.active, _BPTT.dx)
    _BPTT.active = True
    _BPTT.dx = bool(input_grads)
    try:
        yield
    finally:
        _BPTT.active, _BPTT.dx = prev


def _acc_grad(p, g):
    p = grad_target(p)
    if p.grad is None:
        p.grad = g
    else:
        p.grad.add_(g)


def flush_bilstm_backward():
    """Run the queued bi-LSTM backward passes (grouped by weights and shapes) into .grad; for calls queued
    with their input gradient (input_grads mode) continue the backward from their inputs."""
    items, _BPTT.items = _BPTT.items, []
    groups = {}
    for it in items:
        key = (tuple(id(p) for p in it["params"]), tuple(it["x"].shape[1:]))
        groups.setdefault(key, []).append(it)
    xs, dxs = [], []
    with torch.no_grad():
        for grp in groups.values():
            for x, dx in _batched_bptt(grp):
                xs.append(x)
                dxs.append(dx)
    if xs:
        torch.autograd.backward(xs, dxs)


def _batched_bptt(grp):
    W_ih_f, W_hh_f, b_ih_f, b_hh_f, W_ih_b, W_hh_b, b_ih_b, b_hh_b = grp[0]["params"]
    n = grp[0]["needs"]
    B, L, E = grp[0]["x"].shape
    H = W_hh_f.shape[1]
    NB = sum(it["x"].shape[0] for it in grp)
    sa = torch.cat([it["sa"] for it in grp], dim=2)          # [L][2][NB][4H]
    sc = torch.cat([it["sc"] for it in grp], dim=2)          # [L][2][NB][H]
    dout = torch.cat([it["dout"] if it["dout"] is not None else torch.zeros_like(it["out"]) for it in grp], 0)

    def carry(k):
        if all(it[k] is None for it in grp):
            return None
        return torch.cat([it[k] if it[k] is not None else torch.zeros(2, it["x"].shape[0], H, device=sa.device)
                          for it in grp], 1)
    lens = torch.cat([it["lens"] for it in grp], 0)
    dgates = ops.bilstm_bwd(W_hh_f, W_hh_b, lens, (sa, sc), dout, carry("dh_n"), carry("dc_n"), H)
    del sa, sc, dout
    out_all = torch.cat([it["out"] for it in grp], 0)                       # [NB][L][2H]
    x2 = torch.cat([it["x"].detach() for it in grp], 0).reshape(NB * L, E)
    want_dx = any(it["needs"][0] for it in grp)
    dx = None
    for d, (iw, ihh, ibi, ibh) in enumerate(((2, 3, 4, 5), (6, 7, 8, 9))):
        dg = dgates[:, :, d, :]                                # [NB, L, 4H] rows of stride 8H
        P = grp[0]["params"]
        if want_dx:                                            # dx = sum_d dgates_d . W_ih_d (all rows at once)
            Wih = P[iw - 2]
            if dx is None:
                dx = ops.matmul_nn(dg, Wih)
            else:
                ops.matmul_nn(dg, Wih, out=dx, beta=1.0)
        if n[iw]:
            _acc_grad(P[iw - 2], ops.matmul_tn(dg, x2))
        if n[ihh]:
            _acc_grad(P[ihh - 2], ops.bilstm_dw_hh(dgates, out_all, d, H))
        if n[ibi] or n[ibh]:
            db = ops.colsum(dg)
            if n[ibi]:
                _acc_grad(P[ibi - 2], db)
            if n[ibh]:
                _acc_grad(P[ibh - 2], db.clone() if n[ibi] else db)
    out = []
    if dx is not None:
        dx = dx.view(NB, L, E)
        r = 0
        for it in grp:
            b = it["x"].shape[0]
            if it["needs"][0]:
                out.append((it["x"], dx[r:r + b]))
            r += b
    return out


class BiLSTMFn(torch.autograd.Function):
    """Packed single-layer bidirectional nn.LSTM (r2rmodel.py:2339-2343, pack/pad_packed semantics)."""

    @staticmethod
    def forward(ctx, x, lengths_i32, W_ih_f, W_hh_f, b_ih_f, b_hh_f, W_ih_b, W_hh_b, b_ih_b, b_hh_b):
        B, L, E = x.shape
        H = W_hh_f.shape[1]
        x2 = x.reshape(B * L, E)
        xproj = torch.empty(B, L, 2, 4 * H, dtype=torch.float32, device=x.device)
        bf = ops.add2d(b_ih_f.view(1, -1), b_hh_f.view(1, -1)).view(-1)
        bb = ops.add2d(b_ih_b.view(1, -1), b_hh_b.view(1, -1)).view(-1)
        ops.linear(x2, W_ih_f, bf, out=xproj[:, :, 0, :])
        ops.linear(x2, W_ih_b, bb, out=xproj[:, :, 1, :])
        need = any(ctx.needs_input_grad)
        out, h_n, c_n, saved = ops.bilstm_fwd(xproj, W_hh_f, W_hh_b, lengths_i32, H, save=need)
        if need:
            ctx.save_for_backward(x, lengths_i32, out, saved[0], saved[1], W_ih_f, W_hh_f, W_ih_b, W_hh_b)
            ctx.params = _Kept((W_ih_f, W_hh_f, b_ih_f, b_hh_f, W_ih_b, W_hh_b, b_ih_b, b_hh_b))
        ctx.H = H
        ctx.set_materialize_grads(False)     # h_n / c_n usually carry no gradient: null carries, no fills
        return out, h_n, c_n

    @staticmethod
    def backward(ctx, dout, dh_n, dc_n):
        x, lens, out, sa, sc, W_ih_f, W_hh_f, W_ih_b, W_hh_b = ctx.saved_tensors
        H = ctx.H
        B, L, E = x.shape
        n = ctx.needs_input_grad
        if dout is None and dh_n is None and dc_n is None:
            return (None,) * 10
        if _BPTT.active and (not n[0] or _BPTT.dx):
            _BPTT.items.append(dict(x=x, lens=lens, out=out, sa=sa, sc=sc, params=ctx.params, needs=n,
                                    dout=dout.contiguous() if dout is not None else None,
                                    dh_n=dh_n.contiguous() if dh_n is not None else None,
                                    dc_n=dc_n.contiguous() if dc_n is not None else None))
            return (None,) * 10
        if dout is None:
            dout = torch.zeros_like(out)
        dgates = ops.bilstm_bwd(W_hh_f, W_hh_b, lens, (sa, sc), dout, dh_n, dc_n, H)
        x2 = x.reshape(B * L, E)
        grads = [None] * 10
        dx = None
        for d, (iw, ihh, ibi, ibh, Wih) in enumerate(((2, 3, 4, 5, W_ih_f), (6, 7, 8, 9, W_ih_b))):
            dg = dgates[:, :, d, :]          # [B, L, 4H] rows of stride 8H
            if n[iw]:
                grads[iw] = ops.matmul_tn(dg, x2)
            if n[ihh]:
                grads[ihh] = ops.bilstm_dw_hh(dgates, out.contiguous(), d, H)
            if n[ibi] or n[ibh]:
                db = ops.colsum(dg)
                grads[ibi] = db if n[ibi] else None
                grads[ibh] = db if n[ibh] else None
            if n[0]:
                if dx is None:
                    dx = ops.matmul_nn(dg, Wih)
                else:
                    ops.matmul_nn(dg, Wih, out=dx, beta=1.0)
        grads[0] = dx.view(B, L, E) if dx is not None else None
        return tuple(grads)


# --------------------------------------------------------------------------- BERT blocks
class LayerNormFn(torch.autograd.Function):
    """LayerNorm(dropout(x) + res) (BertSelfOutput/BertOutput, vilmodel.py:239-250, 296-309)."""

    @staticmethod
    def forward(ctx, x, res, gamma, beta, eps, p, seed):
        need = any(ctx.needs_input_grad)
        x = x.contiguous()
        if need:
            y, saved = ops.layernorm(x, gamma, beta, eps, res=res.contiguous() if res is not None else None,
                                     drop_p=p, seed=seed, save=True)
            ctx.save_for_backward(gamma, *saved)
        else:
            y = ops.layernorm(x, gamma, beta, eps, res=res.contiguous() if res is not None else None, drop_p=p,
                              seed=seed)
        ctx.p, ctx.seed, ctx.has_res = p, seed, res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        gamma, xsum, mean, rstd = ctx.saved_tensors
        n = ctx.needs_input_grad
        dgamma = torch.zeros_like(gamma) if n[2] else None
        dbeta = torch.zeros_like(gamma) if n[3] else None
        dxs = ops.layernorm_bwd(dy, (xsum, mean, rstd), gamma, dgamma, dbeta)
        dx = None
        if n[0]:
            dx = ops.dropout(dxs, ctx.p, ctx.seed) if ctx.p > 0 else dxs
        dres = dxs if (ctx.has_res and n[1]) else None
        return dx, dres, dgamma, dbeta, None, None, None


def layer_norm(x, gamma, beta, eps, res=None, p=0.0, training=False):
    seed = new_seed() if (training and p > 0) else 0
    p = p if training else 0.0
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (x, res, gamma, beta)):
        return LayerNormFn.apply(x, res, gamma, beta, eps, p, seed)
    return ops.layernorm(x.contiguous(), gamma, beta, eps, res=res.contiguous() if res is not None else None,
                         drop_p=p, seed=seed)


class MHAFn(torch.autograd.Function):
    """softmax(Q K^T / sqrt(dh) + mask) V per head (vilmodel.py:214-236, 481-506)."""

    @staticmethod
    def forward(ctx, Q, K, V, addmask, heads, scale, p, seed):
        need = any(ctx.needs_input_grad)
        if need:
            out, probs = ops.mha(Q, K, V, addmask, heads, scale, p, seed, save_probs=True)
            ctx.save_for_backward(Q, K, V, probs)
        else:
            out = ops.mha(Q, K, V, addmask, heads, scale, p, seed)
        ctx.heads, ctx.scale, ctx.p, ctx.seed = heads, scale, p, seed
        return out

    @staticmethod
    def backward(ctx, dout):
        Q, K, V, probs = ctx.saved_tensors
        dQ, dK, dV = ops.mha_bwd(Q, K, V, probs, dout, ctx.heads, ctx.scale, ctx.p, ctx.seed)
        return dQ, dK, dV, None, None, None, None, None


def mha(Q, K, V, addmask, heads, scale, p=0.0, training=False):
    seed = new_seed() if (training and p > 0) else 0
    p = p if training else 0.0
    if torch.is_grad_enabled() and (Q.requires_grad or K.requires_grad or V.requires_grad):
        return MHAFn.apply(Q, K, V, addmask, heads, scale, p, seed)
    return ops.mha(Q, K, V, addmask, heads, scale, p, seed)
