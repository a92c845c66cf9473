"""Kernel-level parity of libdasa_hip.so against plain fp32 math on the host."""
import ctypes
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, g, scale=1.0):
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


@pytest.mark.parametrize("M,N,K", [(1600, 768, 768), (720, 3072, 768), (20, 4096, 2240), (1040, 2048, 2048),
                                   (37, 45, 100), (1, 1024, 1024), (33, 1, 1024), (130, 130, 36)])
def test_linear(dev, M, N, K):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N)
    x = _rand(M, K, g=g)
    W = _rand(N, K, g=g, scale=0.05)
    b = _rand(N, g=g)
    ref = torch.nn.functional.linear(x.double(), W.double(), b.double()).float()
    y = ops.linear(x.to(dev), W.to(dev), b.to(dev)).cpu()
    assert (y - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


def test_inplace_weight_update_between_forward_and_backward_raises(dev):
    """Parameters ride in ctx.params (not save_for_backward); their version is still checked:
    an in-place update between forward and backward raises like torch's saved-tensor check, while an
    untouched weight gives the plain gradient."""
    from dasa_amd import functional as DF
    g = torch.Generator().manual_seed(5)
    x = _rand(64, 96, g=g).to(dev).requires_grad_()
    W = torch.nn.Parameter(_rand(32, 96, g=g, scale=0.1).to(dev))
    b = torch.nn.Parameter(_rand(32, g=g).to(dev))
    y = DF.linear(x, W, b, "tanh")
    y.sum().backward()
    ref = ((1 - torch.tanh(x.detach().double() @ W.detach().double().t() + b.detach().double()) ** 2).t()
           @ x.detach().double())
    assert (W.grad.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    y = DF.linear(x, W, b, "tanh")
    with torch.no_grad():
        W.mul_(0.5)                                   # in place, after the forward
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        y.sum().backward()


@pytest.mark.parametrize("M,N,K,opB", [(160, 768, 768, 1), (72, 768, 3072, 0), (100, 3072, 768, 1), (33, 70, 1000, 0)])
def test_gemm_short_m_split(dev, M, N, K, opB):
    """The short-GEMM plan (33..192 rows, split-K over 32x64 tiles + the fixed-order reduce) with the fused
    bias / GELU epilogue and beta accumulation, forward (NT) and dX (NN) layouts, vs fp64."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(M + N + K)
    x = _rand(M, K, g=g)
    W = _rand(N, K, g=g, scale=0.05) if opB else _rand(K, N, g=g, scale=0.05)
    b, c0 = _rand(N, g=g), _rand(M, N, g=g)
    Wn = W.double() if opB else W.double().t()
    z = x.double() @ Wn.t() + b.double()
    ref = (z * 0.5 * (1 + torch.erf(z / math.sqrt(2))) + c0.double()).float()
    y = c0.clone().to(dev)
    ops.gemm(x.to(dev), W.to(dev), y, M=M, N=N, K=K, opB=opB, lda=K, ldb=K if opB else N, ldc=N, bias=b.to(dev),
             act="gelu", beta=1.0)
    assert (y.cpu() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("act", ["relu", "gelu", "tanh", "sigmoid"])
def test_linear_act_and_gate(dev, act):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(3)
    M, N, K = 300, 260, 200
    x, W, b = _rand(M, K, g=g), _rand(N, K, g=g, scale=0.1), _rand(N, g=g)
    aux, cs = _rand(M, N, g=g), _rand(N, g=g)
    z = torch.nn.functional.linear(x.double(), W.double(), b.double())
    f = {"relu": torch.relu, "gelu": lambda t: t * 0.5 * (1 + torch.erf(t / math.sqrt(2))), "tanh": torch.tanh,
         "sigmoid": torch.sigmoid}[act]
    ref = (f(z) * aux.double() * cs.double()).float()
    y = ops.linear(x.to(dev), W.to(dev), b.to(dev), act=act, aux=aux.to(dev), colscale=cs.to(dev)).cpu()
    assert (y - ref).abs().max().item() < 1e-5


def test_gemm_layouts(dev):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(5)
    A, B = _rand(70, 92, g=g), _rand(92, 52, g=g)
    ref = (A.double() @ B.double()).float()
    assert (ops.matmul_nn(A.to(dev), B.to(dev)).cpu() - ref).abs().max() < 1e-5
    At = A.t().contiguous()
    assert (ops.matmul_tn(At.to(dev), B.to(dev)).cpu() - ref).abs().max() < 1e-5
    s = ops.colsum(B.to(dev)).cpu()
    assert (s - B.sum(0)).abs().max() < 1e-5
    # strided rows + beta accumulate
    big = _rand(70, 128, g=g).to(dev)
    C0 = _rand(70, 52, g=g)
    out = C0.clone().to(dev)
    ops.matmul_nn(big[:, :92], B.to(dev), out=out, beta=1.0)
    ref2 = (big[:, :92].cpu().double() @ B.double() + C0.double()).float()
    assert (out.cpu() - ref2).abs().max() < 1e-5
    # unaligned row strides take the scalar-load variant
    A2, B2 = _rand(37, 45, g=g), _rand(45, 3, g=g)
    ref3 = (A2.double() @ B2.double()).float()
    assert (ops.matmul_nn(A2.to(dev), B2.to(dev)).cpu() - ref3).abs().max() < 1e-5
    assert (ops.matmul_tn(A2.t().contiguous().to(dev), B2.to(dev)).cpu() - ref3).abs().max() < 1e-5
    assert (ops.colsum(B2.to(dev)).cpu() - B2.sum(0)).abs().max() < 1e-5


def test_gemm_every_config(dev):
    """Force each tile configuration (incl. in-block K-split and split-K) over ragged shapes, both
    operand layouts and the fused epilogue, so a config the shape rules pick only at bench sizes is
    still checked."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    ncfg = lib.dasa_gemm_force_config(-1)
    g = torch.Generator().manual_seed(11)
    # K % 64 == 0 shapes reach the 64-deep K kernels and their stream-K forms (split tiles summed
    # by the last arriving workgroup)
    shapes = [(37, 45, 100), (130, 200, 36), (64, 128, 1024), (257, 96, 2100), (300, 136, 1536), (520, 64, 4096)]
    try:
        for cfg in range(ncfg):
            lib.dasa_gemm_force_config(cfg)
            for M, N, K in shapes:
                x, W, b = _rand(M, K, g=g), _rand(N, K, g=g, scale=0.05), _rand(N, g=g)
                aux = _rand(M, N, g=g)
                z = torch.nn.functional.linear(x.double(), W.double(), b.double())
                ref = (torch.tanh(z) * aux.double()).float()
                y = ops.linear(x.to(dev), W.to(dev), b.to(dev), act="tanh", aux=aux.to(dev)).cpu()
                assert (y - ref).abs().max().item() < 1e-5, (cfg, M, N, K)
                B = _rand(K, N, g=g)
                ref_nn = (x.double() @ B.double()).float()
                tol = 1e-4 * max(1.0, ref_nn.abs().max().item())
                assert (ops.matmul_nn(x.to(dev), B.to(dev)).cpu() - ref_nn).abs().max() < tol, (cfg, M, N, K)
                xt = x.t().contiguous()
                assert (ops.matmul_tn(xt.to(dev), B.to(dev)).cpu() - ref_nn).abs().max() < tol, (cfg, M, N, K)
    finally:
        lib.dasa_gemm_force_config(-1)


def test_layernorm_and_embed(dev):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(7)
    x, r = _rand(123, 768, g=g), _rand(123, 768, g=g)
    gm, bt = _rand(768, g=g), _rand(768, g=g)
    ref = torch.nn.functional.layer_norm(x + r, (768,), gm, bt, 1e-12)
    y = ops.layernorm(x.to(dev), gm.to(dev), bt.to(dev), 1e-12, res=r.to(dev)).cpu()
    assert (y - ref).abs().max() < 1e-4
    ids = torch.randint(0, 1000, (3, 17), generator=g)
    word, pos, typ = _rand(1000, 768, g=g), _rand(512, 768, g=g), _rand(2, 768, g=g)
    e = word[ids] + pos[:17][None] + typ[0]
    ref = torch.nn.functional.layer_norm(e, (768,), gm, bt, 1e-12)
    y = ops.bert_embed(ids.to(dev), word.to(dev), pos.to(dev), typ[0].to(dev), gm.to(dev), bt.to(dev), 1e-12).cpu()
    assert (y - ref).abs().max() < 1e-4


@pytest.mark.parametrize("Lq,Lk", [(80, 80), (80, 36), (36, 80), (5, 100)])
def test_mha(dev, Lq, Lk):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(Lq + Lk)
    B, h = 3, 12
    Q, K, V = _rand(B, Lq, 768, g=g), _rand(B, Lk, 768, g=g), _rand(B, Lk, 768, g=g)
    m = torch.zeros(B, Lk)
    m[1, Lk // 2:] = -10000.0
    q4 = Q.view(B, Lq, h, 64).permute(0, 2, 1, 3)
    k4 = K.view(B, Lk, h, 64).permute(0, 2, 1, 3)
    v4 = V.view(B, Lk, h, 64).permute(0, 2, 1, 3)
    s = q4 @ k4.transpose(-1, -2) / 8.0 + m[:, None, None, :]
    p = torch.softmax(s, -1)
    ref = (p @ v4).permute(0, 2, 1, 3).reshape(B, Lq, 768)
    out = ops.mha(Q.to(dev), K.to(dev), V.to(dev), m.to(dev), 12, 1 / 8.0).cpu()
    assert (out - ref).abs().max() < 1e-5


@pytest.mark.parametrize("M,N", [(123, 768), (1, 768), (1700, 768), (37, 2048), (9, 12)])
def test_layernorm_bwd_vs_autograd(dev, M, N):
    """dx / dgamma / dbeta of dasa_layernorm_bwd vs torch autograd (fp32); dgamma / dbeta accumulate into what
    the caller passes and are bit-identical run to run (fixed-order column reduction, no atomics)."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(M + N)
    x, dy = _rand(M, N, g=g), _rand(M, N, g=g)
    gm, bt = _rand(N, g=g), _rand(N, g=g)
    xr, gr, br = x.clone().requires_grad_(), gm.clone().requires_grad_(), bt.clone().requires_grad_()
    torch.nn.functional.layer_norm(xr, (N,), gr, br, 1e-12).backward(dy)
    y, saved = ops.layernorm(x.to(dev), gm.to(dev), bt.to(dev), 1e-12, save=True)
    outs = []
    for _ in range(2):
        dg0, db0 = torch.full((N,), 0.5, device=dev), torch.full((N,), -0.25, device=dev)
        dx = ops.layernorm_bwd(dy.to(dev), saved, gm.to(dev), dg0, db0)
        outs.append((dx.cpu(), dg0.cpu() - 0.5, db0.cpu() + 0.25))
    dx, dg, db = outs[0]
    tol = 2e-4 * max(1.0, M / 64)
    assert (dx - xr.grad).abs().max() < 1e-3
    assert (dg - gr.grad).abs().max() < tol
    assert (db - br.grad).abs().max() < tol
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))


def _mha_ref(Q, K, V, m, h, scale, dscale=None):
    B, Lq, Hd = Q.shape
    Lk = K.shape[1]
    q4 = Q.view(B, Lq, h, 64).permute(0, 2, 1, 3)
    k4 = K.view(B, Lk, h, 64).permute(0, 2, 1, 3)
    v4 = V.view(B, Lk, h, 64).permute(0, 2, 1, 3)
    p = torch.softmax(q4 @ k4.transpose(-1, -2) * scale + m[:, None, None, :], -1)
    if dscale is not None:
        p = p * dscale
    return (p @ v4).permute(0, 2, 1, 3).reshape(B, Lq, Hd)


@pytest.mark.parametrize("Lq,Lk,p", [(80, 80, 0.0), (80, 36, 0.0), (36, 80, 0.0), (7, 13, 0.0), (5, 100, 0.0),
                                     (80, 36, 0.1), (13, 7, 0.1)])
def test_mha_bwd_vs_autograd(dev, Lq, Lk, p):
    """dasa_mha_bwd (LDS-staged form for Lq, Lk <= 80; the row-streaming form above) vs torch autograd in
    fp32. With dropout the forward's per-element scale is read back through an identity V (Lk <= 64):
    out[b, i, h*64 + j] = P_dropped[b, h, i, j]."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(3 * Lq + Lk)
    B, h, scale, seed = 2, 12, 1 / 8.0, 1234
    Q, K, V = _rand(B, Lq, 768, g=g), _rand(B, Lk, 768, g=g), _rand(B, Lk, 768, g=g)
    dO = _rand(B, Lq, 768, g=g)
    m = torch.zeros(B, Lk)
    m[1, Lk // 2:] = -10000.0
    dscale = None
    _, probs = ops.mha(Q.to(dev), K.to(dev), V.to(dev), m.to(dev), h, scale, p, seed, save_probs=True)
    if p > 0:
        eye = torch.zeros(B, Lk, 768)
        for hh in range(h):
            eye[:, torch.arange(Lk), hh * 64 + torch.arange(Lk)] = 1.0
        pd = ops.mha(Q.to(dev), K.to(dev), eye.to(dev), m.to(dev), h, scale, p, seed).cpu()
        pd = pd.view(B, Lq, h, 64)[..., :Lk].permute(0, 2, 1, 3)
        pr = probs.cpu()
        dscale = torch.where(pd != 0, torch.full_like(pd, 1 / (1 - p)), torch.zeros_like(pd))
        assert (pd - pr * dscale).abs().max() < 1e-5          # the read-back mask is the forward's
    qr, kr, vr = (t.clone().requires_grad_() for t in (Q, K, V))
    _mha_ref(qr, kr, vr, m, h, scale, dscale).backward(dO)
    dQ, dK, dV = (t.cpu() for t in ops.mha_bwd(Q.to(dev), K.to(dev), V.to(dev), probs, dO.to(dev), h, scale, p, seed))
    for got, ref in ((dQ, qr.grad), (dK, kr.grad), (dV, vr.grad)):
        assert (got - ref).abs().max() < 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("Lq,Lk,p", [(80, 80, 0.1), (36, 80, 0.0), (7, 13, 0.1)])
def test_mha_bwd_parts_bitwise(dev, Lq, Lk, p):
    """The LDS-staged attention backward split over 1-7 workgroups per (batch, head) (dasa_mha_bwd_split;
    the default at the finetune's B = 2 is 4): every split writes the same dQ / dK / dV bitwise."""
    from dasa_amd import _lib, ops
    g = torch.Generator().manual_seed(Lq * Lk)
    B, h, scale, seed = 2, 12, 1 / 8.0, 99
    Q, K, V, dO = (_rand(B, L_, 768, g=g).to(dev) for L_ in (Lq, Lk, Lk, Lq))
    m = torch.zeros(B, Lk, device=dev)
    m[1, Lk // 2:] = -10000.0
    _, probs = ops.mha(Q, K, V, m, h, scale, p, seed, save_probs=True)
    lib = _lib.lib()
    prev = lib.dasa_mha_bwd_split(1)
    try:
        ref = [t.clone() for t in ops.mha_bwd(Q, K, V, probs, dO, h, scale, p, seed)]
        for parts in (2, 3, 4, 7):
            lib.dasa_mha_bwd_split(parts)
            got = ops.mha_bwd(Q, K, V, probs, dO, h, scale, p, seed)
            for a_, b_ in zip(got, ref):
                assert torch.equal(a_, b_), parts
    finally:
        lib.dasa_mha_bwd_split(prev)


@pytest.fixture(params=["split", "rowsplit", "split2", "rowsplit_fwd"])
def attn_mode(request, dev):
    """The attention implementations (include/dasa_hip.h dasa_attn_set_mode): the D-split forms the
    decision step uses at small B (mode 0), the row-split form (large B, N > 80; mode 1), mode 2: the
    two-launch D-split forward for SoftDot as well (masks, N up to 80, strided rows), mode 4: the shift
    forward on the row-split kernel too."""
    from dasa_amd import ops
    ops.attn_set_mode({"split": 0, "rowsplit": 1, "split2": 2, "rowsplit_fwd": 4}[request.param])
    yield request.param
    ops.attn_set_mode(0)


def test_softdot_and_shift(dev, attn_mode):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(11)
    B, N, D = 5, 36, 2176
    q, ctx = _rand(B, D, g=g, scale=0.05), torch.rand(B, N, D, generator=g)
    mask = torch.zeros(B, N, dtype=torch.bool)
    mask[2, 30:] = True
    s = torch.einsum("bnd,bd->bn", ctx, q)
    p = torch.softmax(s.masked_fill(mask, -float("inf")), 1)
    w = torch.einsum("bn,bnd->bd", p, ctx)
    sc, pr, wc = ops.softdot_fwd(q.to(dev), ctx.to(dev), mask.to(dev))
    assert (sc.cpu() - s).abs().max() < 1e-4
    assert (pr.cpu() - p).abs().max() < 1e-5
    assert (wc.cpu() - w).abs().max() < 1e-4
    # shift attention against the reference's conv1d formulation (model.py:337-345)
    z = _rand(B, 5, g=g)
    a = torch.softmax(s, 1)
    a3 = a.view(B, 3, 12)
    kern = torch.softmax(z, -1).unsqueeze(1)
    a3 = torch.cat([a3[:, :, -2:], a3, a3[:, :, :2]], -1).transpose(0, 1)
    a3 = torch.nn.functional.conv1d(a3, kern, groups=B).transpose(0, 1).reshape(B, 1, -1)
    wref = torch.bmm(a3, ctx).squeeze(1)
    wctx, attn, shifted, wsm = ops.shift_attn_fwd(q.to(dev), ctx.to(dev), z.to(dev))
    assert (attn.cpu() - a).abs().max() < 1e-5
    assert (wctx.cpu() - wref).abs().max() < 1e-4


def test_softdot_shift_backward(dev, attn_mode):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(13)
    B, N, D = 4, 36, 2176
    q = (_rand(B, D, g=g, scale=0.05)).requires_grad_()
    ctx = torch.rand(B, N, D, generator=g).requires_grad_()
    z = _rand(B, 5, g=g).requires_grad_()
    gw = _rand(B, D, g=g)
    s = torch.einsum("bnd,bd->bn", ctx, q)
    a = torch.softmax(s, 1)
    a3 = a.view(B, 3, 12)
    kern = torch.softmax(z, -1).unsqueeze(1)
    a3 = torch.cat([a3[:, :, -2:], a3, a3[:, :, :2]], -1).transpose(0, 1)
    a3 = torch.nn.functional.conv1d(a3, kern, groups=B).transpose(0, 1).reshape(B, 1, -1)
    wref = torch.bmm(a3, ctx).squeeze(1)
    (wref * gw).sum().backward()
    qd, cd, zd = q.detach().to(dev), ctx.detach().to(dev), z.detach().to(dev)
    wctx, attn, shifted, wsm = ops.shift_attn_fwd(qd, cd, zd)
    dq, dctx, dz = ops.shift_attn_bwd(qd, cd, attn, shifted, wsm, gw.to(dev))
    assert (dq.cpu() - q.grad).abs().max() < 1e-4 * max(1, q.grad.abs().max())
    assert (dctx.cpu() - ctx.grad).abs().max() < 1e-5
    assert (dz.cpu() - z.grad).abs().max() < 1e-4 * max(1, z.grad.abs().max())
    # softdot with mask: wctx grad + raw-score grad
    mask = torch.zeros(B, N, dtype=torch.bool)
    mask[1, 20:] = True
    q2 = q.detach().clone().requires_grad_()
    c2 = ctx.detach().clone().requires_grad_()
    gs = _rand(B, N, g=g)
    s = torch.einsum("bnd,bd->bn", c2, q2)
    p = torch.softmax(s.masked_fill(mask, -float("inf")), 1)
    w = torch.einsum("bn,bnd->bd", p, c2)
    ((w * gw).sum() + (s * gs).sum()).backward()
    _, pr, _ = ops.softdot_fwd(q2.detach().to(dev), c2.detach().to(dev), mask.to(dev))
    dq, dctx = ops.softdot_bwd(q2.detach().to(dev), c2.detach().to(dev), pr, dwctx=gw.to(dev), dscores=gs.to(dev))
    assert (dq.cpu() - q2.grad).abs().max() < 1e-4 * max(1, q2.grad.abs().max())
    assert (dctx.cpu() - c2.grad).abs().max() < 1e-5 * max(1, c2.grad.abs().max())


@pytest.mark.parametrize("B,N,D,ldn", [(1, 1, 2176, 2176), (3, 7, 2048, 2176), (37, 16, 2176, 2176),
                                         (2, 80, 2048, 2048), (2, 100, 1024, 1024), (2, 9, 4096, 4096),
                                         (4, 36, 2176, 2176)])
def test_softdot_fused_shapes(dev, B, N, D, ldn, attn_mode):
    """The one-launch SoftDot kernels over row counts around the 12/16-row passes, N > 64, strided
    rows (a 2048-column view of 2176-float rows), D = 4096 (1024 threads), B = 1."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(N * 1000 + D)
    q = _rand(B, D, g=g, scale=0.05).double()
    full = torch.rand(B, N, ldn, generator=g).double()
    ctx = full[:, :, :D]
    mask = torch.rand(B, N, generator=g) < 0.3
    mask[:, 0] = False
    gw, gs = _rand(B, D, g=g).double(), _rand(B, N, g=g).double()
    qr, cr = q.clone().requires_grad_(), ctx.clone().requires_grad_()
    s = torch.einsum("bnd,bd->bn", cr, qr)
    p = torch.softmax(s.masked_fill(mask, -float("inf")), 1)
    w = torch.einsum("bn,bnd->bd", p, cr)
    ((w * gw).sum() + (s * gs).sum()).backward()
    fd = full.float().to(dev)
    cd = fd[:, :, :D]
    sc, pr, wc = ops.softdot_fwd(q.float().to(dev), cd, mask.to(dev))
    assert (sc.cpu().double() - s).abs().max() < 1e-4
    assert (pr.cpu().double() - p).abs().max() < 1e-5
    assert (wc.cpu().double() - w).abs().max() < 1e-4
    cc = cd.contiguous()
    dq, dctx = ops.softdot_bwd(q.float().to(dev), cc, pr, dwctx=gw.float().to(dev), dscores=gs.float().to(dev))
    assert (dq.cpu().double() - qr.grad).abs().max() < 2e-4 * max(1, qr.grad.abs().max())
    assert (dctx.cpu().double() - cr.grad).abs().max() < 1e-5 * max(1, cr.grad.abs().max())
    # scores only (the candidate-logit path) and its dscores-only backward
    sc2, _, _ = ops.softdot_fwd(q.float().to(dev), cd, None, want_probs=False, want_wctx=False)
    assert (sc2.cpu().double() - s.detach()).abs().max() < 1e-4


@pytest.mark.parametrize("N,D,ldn", [(36, 2176, 2176), (20, 2048, 2176), (7, 2176, 2176), (80, 2048, 2048),
                                     (80, 2048, 2176), (49, 2176, 2176), (84, 1024, 1024)])
def test_attention_whole_row_forward(dev, N, D, ldn):
    """The whole-row forward (B >= 128: one workgroup per batch row, rows streamed 12 at a time with an
    online softmax) against fp64 host math: SoftDot with a mask at N = 7 ... 84 (up to seven 12-row
    slices, the last one partial; strided rows: configs[4]'s N = 80 instruction attention), and the K=5
    shift attention over the 36-view panorama."""
    from dasa_amd import ops
    ops.attn_set_mode(0)
    g = torch.Generator().manual_seed(N + D)
    B = 130
    q = _rand(B, D, g=g, scale=0.05).double()
    full = torch.rand(B, N, ldn, generator=g).double()
    ctx = full[:, :, :D]
    mask = torch.rand(B, N, generator=g) < 0.3
    mask[:, 0] = False
    s = torch.einsum("bnd,bd->bn", ctx, q)
    p = torch.softmax(s.masked_fill(mask, -float("inf")), 1)
    w = torch.einsum("bn,bnd->bd", p, ctx)
    cd = full.float().to(dev)[:, :, :D]
    sc, pr, wc = ops.softdot_fwd(q.float().to(dev), cd, mask.to(dev))
    assert (sc.cpu().double() - s).abs().max() < 1e-4
    assert (pr.cpu().double() - p).abs().max() < 1e-5
    assert (wc.cpu().double() - w).abs().max() < 1e-4
    if N != 36:
        return
    z = _rand(B, 5, g=g).double()
    a = torch.softmax(s, 1)
    a3 = a.view(B, 3, 12)
    kern = torch.softmax(z, -1).unsqueeze(1)
    a3 = torch.cat([a3[:, :, -2:], a3, a3[:, :, :2]], -1).transpose(0, 1)
    a3 = torch.nn.functional.conv1d(a3, kern, groups=B).transpose(0, 1).reshape(B, 1, -1)
    wref = torch.bmm(a3, ctx).squeeze(1)
    wctx, attn, shifted, wsm = ops.shift_attn_fwd(q.float().to(dev), cd, z.float().to(dev))
    assert (attn.cpu().double() - a).abs().max() < 1e-5
    assert (shifted.cpu().double() - a3.squeeze(1)).abs().max() < 1e-5
    assert (wctx.cpu().double() - wref).abs().max() < 1e-4


def test_lstm_cell(dev):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(17)
    B, H = 7, 1024
    gates = _rand(B, 4 * H, g=g, scale=2).requires_grad_()
    c0 = _rand(B, H, g=g).requires_grad_()
    i, f, gg, o = gates.chunk(4, 1)
    c1 = torch.sigmoid(f) * c0 + torch.sigmoid(i) * torch.tanh(gg)
    h1 = torch.sigmoid(o) * torch.tanh(c1)
    gh, gc = _rand(B, H, g=g), _rand(B, H, g=g)
    ((h1 * gh).sum() + (c1 * gc).sum()).backward()
    h, c, act = ops.lstm_cell_fwd(gates.detach().to(dev), c0.detach().to(dev), save=True)
    assert (h.cpu() - h1).abs().max() < 1e-6 and (c.cpu() - c1).abs().max() < 1e-6
    dg, dc0 = ops.lstm_cell_bwd(act, c0.detach().to(dev), c, gh.to(dev), gc.to(dev))
    assert (dg.cpu() - gates.grad).abs().max() < 1e-5 and (dc0.cpu() - c0.grad).abs().max() < 1e-5


@pytest.mark.parametrize("x6", [0, 1])
@pytest.mark.parametrize("B,L", [(20, 80), (3, 11), (40, 9), (160, 12)])
def test_bilstm_persist_fwd_x6(dev, B, L, x6):
    """The persistent forward with the recurrent product as bf16x6 (default at H = 1024) and as native
    fp32 MFMA: both against torch's packed nn.LSTM (fp32, CPU) at the tolerance of test_bilstm."""
    from dasa_amd import _lib
    lib = _lib.lib()
    assert lib.dasa_bilstm_set_mode(2) == 0
    prev = lib.dasa_bilstm_fwd_x6(x6)
    try:
        _check_bilstm(dev, B, L)
    finally:
        lib.dasa_bilstm_fwd_x6(prev)
        lib.dasa_bilstm_set_mode(0)


@pytest.mark.parametrize("x6", [1, 0])
def test_bilstm_step_path_b256(dev, x6):
    """B > 192 takes the per-timestep path: both directions' recurrent product as ONE batched GEMM per step on
    W_hh converted once per call (bf16x6, fp32-accurate; x6 = 0: the native fp32 kernels, two launches)."""
    from dasa_amd import _lib
    lib = _lib.lib()
    prev = lib.dasa_bilstm_fwd_x6(x6)
    try:
        _check_bilstm(dev, 256, 12)
    finally:
        lib.dasa_bilstm_fwd_x6(prev)


def test_bilstm_step_path_bf16(dev):
    """configs[4]'s bf16 mode (dasa_bilstm_fwd_bf16, set by ops.bf16_matmul): h and W_hh rounded to bf16 (RNE)
    for the recurrent product, fp32 accumulation and cell. Against a float64 restatement that rounds the same
    two operands per step: equal up to fp32 summation order (and the rare h element whose bf16 rounding flips
    with it); against the fp32 LSTM: within bf16 precision."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    torch.manual_seed(5)
    B, L, H = 256, 10, 1024
    xproj = (torch.randn(B, L, 2, 4 * H) * 0.5).to(dev)
    whh_f = (torch.rand(4 * H, H) * 0.1 - 0.05).to(dev)
    whh_b = (torch.rand(4 * H, H) * 0.1 - 0.05).to(dev)
    lengths = torch.randint(1, L + 1, (B,))
    lengths[0] = L
    li = lengths.to(torch.int32).to(dev)
    with torch.no_grad(), ops.bf16_matmul():
        assert lib.dasa_bilstm_fwd_bf16(-1) == 1
        out, h_n, c_n, _ = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H)
    assert lib.dasa_bilstm_fwd_bf16(-1) == 0
    out32, _, _, _ = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H)

    def ref(round_bf16):
        xp, ln = xproj.cpu().double(), lengths
        res = torch.zeros(B, L, 2 * H, dtype=torch.float64)
        for d, W in enumerate((whh_f, whh_b)):
            Wd = W.cpu()
            Wd = (Wd.bfloat16() if round_bf16 else Wd).double()
            h = torch.zeros(B, H, dtype=torch.float64)
            c = torch.zeros(B, H, dtype=torch.float64)
            for s in range(L):
                t = s if d == 0 else L - 1 - s
                hr = h.float().bfloat16().double() if round_bf16 else h
                g = xp[:, t, d] + hr @ Wd.T
                i, f, gg, o = g.split(H, 1)
                c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
                h2 = torch.sigmoid(o) * torch.tanh(c2)
                act = (t < ln).unsqueeze(1)
                c = torch.where(act, c2, c)
                h = torch.where(act, h2, h)
                res[:, t, d * H:(d + 1) * H] = torch.where(act, h2, torch.zeros_like(h2))
        return res
    rb = ref(True)
    err = (out.cpu().double() - rb).abs()
    assert err.max() < 5e-3 and err.mean() < 1e-5, (err.max(), err.mean())
    assert (out32.cpu().double() - ref(False)).abs().max() < 2e-5
    assert (out.cpu() - out32.cpu()).abs().max() < 3e-2


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("B,L", [(20, 80), (3, 11), (40, 9), (160, 12)])
def test_bilstm(dev, B, L, mode):
    """mode 1: one launch per timestep; mode 2: the persistent recurrence (forward: 32-row batch tiles
    up to B = 192 at H = 1024; the BPTT of B > 32 takes the batched-GEMM path in both modes)."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    assert lib.dasa_bilstm_set_mode(mode) == 0
    try:
        _check_bilstm(dev, B, L)
    finally:
        lib.dasa_bilstm_set_mode(0)


@pytest.mark.parametrize("B,L", [(40, 9), (700, 16)])
def test_bilstm_bptt_x6_vs_native(dev, B, L):
    """The B > 32 BPTT's recurrent product on the bf16x6 GEMM (default) against dasa_gemm_f32: the
    dgates of every step agree to fp32 rounding (both are fp32-accurate; errors compound over steps)."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    torch.manual_seed(7)
    H = 1024
    whh_f, whh_b = [(torch.rand(4 * H, H, device=dev) - 0.5) * 0.1 for _ in range(2)]
    xproj = torch.randn(B, L, 2, 4 * H, device=dev)
    li = torch.randint(1, L + 1, (B,)).sort(descending=True)[0].to(torch.int32).to(dev)
    out, h_n, c_n, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
    gout = torch.randn(B, L, 2 * H, device=dev)
    ghn, gcn = torch.randn(2, B, H, device=dev), torch.randn(2, B, H, device=dev)
    prev = lib.dasa_bilstm_bptt_x6(1)
    try:
        dg6 = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, ghn, gcn, H)
        lib.dasa_bilstm_bptt_x6(0)
        dgn = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, ghn, gcn, H)
    finally:
        lib.dasa_bilstm_bptt_x6(prev)
    torch.cuda.synchronize()
    assert torch.isfinite(dg6).all()
    scale = dgn.abs().max().item()
    assert (dg6 - dgn).abs().max().item() < 2e-5 * scale


@pytest.mark.parametrize("B,L", [(2, 80), (16, 23), (5, 1)])
def test_bilstm_bptt_one_tile_bitwise(dev, B, L):
    """The persistent BPTT's one-row-tile form (B <= 16, the finetune rollout's B = 2) runs the two-tile
    form's products in the same order: its dgates equal the two-tile form's bitwise, ragged lengths and a
    one-step sequence included."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    torch.manual_seed(B * 100 + L)
    H = 1024
    whh_f, whh_b = [(torch.rand(4 * H, H, device=dev) - 0.5) * 0.1 for _ in range(2)]
    xproj = torch.randn(B, L, 2, 4 * H, device=dev)
    li = torch.randint(1, L + 1, (B,)).sort(descending=True)[0].to(torch.int32)
    li[0] = L
    li = li.to(dev)
    assert lib.dasa_bilstm_set_mode(2) == 0
    prev = lib.dasa_bilstm_bptt_one_tile(1)
    try:
        out, h_n, c_n, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
        gout = torch.randn(B, L, 2 * H, device=dev)
        ghn, gcn = torch.randn(2, B, H, device=dev), torch.randn(2, B, H, device=dev)
        dg1 = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, ghn, gcn, H)
        lib.dasa_bilstm_bptt_one_tile(0)
        dg2 = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, ghn, gcn, H)
    finally:
        lib.dasa_bilstm_bptt_one_tile(prev)
        lib.dasa_bilstm_set_mode(0)
    torch.cuda.synchronize()
    assert torch.isfinite(dg1).all()
    assert torch.equal(dg1, dg2)


@pytest.mark.parametrize("B,L", [(40, 9), (7, 23), (1, 5), (3, 1)])
def test_bilstm_dw_hh_in_place(dev, B, L):
    """ops.bilstm_dw_hh: dW_hh read from strided views of the bi-LSTM output, with the
    cross-sequence pairs removed by one alpha = -1 GEMM, equals dgatesᵀ · h_prev built by the materialised
    shifted copy (dasa_bilstm_hprev, zero at each direction's first step) — real dgates of a ragged batch
    (rows past a sequence's length zero), against fp64 on the same operands."""
    from dasa_amd import ops
    torch.manual_seed(B * 31 + L)
    H = 1024
    whh_f, whh_b = [(torch.rand(4 * H, H, device=dev) - 0.5) * 0.1 for _ in range(2)]
    xproj = torch.randn(B, L, 2, 4 * H, device=dev)
    li = torch.randint(1, L + 1, (B,)).sort(descending=True)[0].to(torch.int32)
    li[0] = L
    li = li.to(dev)
    out, h_n, c_n, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
    gout = torch.randn(B, L, 2 * H, device=dev)
    dgates = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout, None, None, H)
    hprev = ops.bilstm_hprev(out, H)
    for d in range(2):
        dg = dgates[:, :, d, :]
        got = ops.bilstm_dw_hh(dgates, out.contiguous(), d, H)
        want64 = dg.reshape(B * L, 4 * H).double().t() @ hprev[d].reshape(B * L, H).double()
        copy = ops.matmul_tn(dg, hprev[d].reshape(B * L, H))
        # the scale of the summed |products|, shifted pairs and cross-sequence pairs alike (those cancel exactly
        # in exact arithmetic, to fp32 rounding here)
        hd = out[:, :, d * H:(d + 1) * H].reshape(B * L, H)
        scale = (dg.reshape(B * L, 4 * H).abs().double().t() @ hd.abs().double()).max().item() + 1e-30
        err_copy = (copy.double() - want64).abs().max().item()
        err = (got.double() - want64).abs().max().item()
        assert err <= max(3 * err_copy, 1e-6 * scale), (d, err, err_copy, scale)


@pytest.mark.parametrize("input_grads", [False, True])
def test_bilstm_deferred_input_grads(dev, input_grads):
    """defer_bilstm_backward(input_grads=True) (optim_step's path when the language stack trains, cfg4): three
    bi-LSTM calls sharing weights, whose inputs come from one trainable tensor through different ops, run
    their BPTT as one batched recurrence and continue the backward from the queued inputs; the input
    tensor's and the weights' gradients equal the per-call backward's to fp32 re-association."""
    from dasa_amd import functional as DF
    torch.manual_seed(11)
    H, E, L = 1024, 768, 12
    lstm = torch.nn.LSTM(E, H, 1, batch_first=True, bidirectional=True).to(dev)
    with torch.no_grad():
        for p_ in lstm.parameters():
            p_.uniform_(-0.05, 0.05)
    params = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0, lstm.weight_ih_l0_reverse,
              lstm.weight_hh_l0_reverse, lstm.bias_ih_l0_reverse, lstm.bias_hh_l0_reverse]
    a = torch.randn(6, L, E, device=dev).requires_grad_()
    gs = [torch.randn(6, L, 2 * H, device=dev) for _ in range(3)]
    lens = torch.tensor([12, 12, 9, 7, 3, 1], dtype=torch.int32, device=dev)

    def run(deferred):
        for p_ in params + [a]:
            p_.grad = None
        xs = [a * 0.5, torch.tanh(a), a[:, :, torch.arange(E - 1, -1, -1, device=dev)] * 2.0]
        loss = sum((DF.BiLSTMFn.apply(x.contiguous(), lens, *params)[0] * g).sum() for x, g in zip(xs, gs))
        if deferred:
            with DF.defer_bilstm_backward(input_grads=input_grads), DF.defer_weight_grads():
                loss.backward(retain_graph=input_grads)
                DF.flush_bilstm_backward()
            DF.flush_weight_grads()
        else:
            loss.backward()
        torch.cuda.synchronize()
        return [p_.grad.clone() for p_ in params + [a]]

    ref = run(False)
    got = run(True)
    for r, g in zip(ref, got):
        assert torch.isfinite(g).all()
        assert (g - r).abs().max().item() <= 2e-5 * max(1.0, r.abs().max().item())


def _check_bilstm(dev, B, L):
    from dasa_amd import ops
    torch.manual_seed(B + L)
    H, E = 1024, 768
    lstm = torch.nn.LSTM(E, H, 1, batch_first=True, bidirectional=True)
    with torch.no_grad():
        for p_ in lstm.parameters():
            p_.uniform_(-0.05, 0.05)
    lengths = torch.randint(1, L + 1, (B,))
    lengths[0] = L
    lengths, _ = lengths.sort(descending=True)
    x = torch.randn(B, L, E) * 0.5
    packed = torch.nn.utils.rnn.pack_padded_sequence(x, lengths.tolist(), batch_first=True)
    out_p, (hn, cn) = lstm(packed)
    out_ref, _ = torch.nn.utils.rnn.pad_packed_sequence(out_p, batch_first=True, total_length=L)
    gout = torch.randn(B, L, 2 * H)
    ghn, gcn = torch.randn(2, B, H), torch.randn(2, B, H)
    ((out_ref * gout).sum() + (hn * ghn).sum() + (cn * gcn).sum()).backward()
    Wih = torch.cat([lstm.weight_ih_l0, lstm.weight_ih_l0_reverse], 0).detach()
    bias = torch.cat([lstm.bias_ih_l0 + lstm.bias_hh_l0, lstm.bias_ih_l0_reverse + lstm.bias_hh_l0_reverse]).detach()
    whh_f, whh_b = lstm.weight_hh_l0.detach().to(dev), lstm.weight_hh_l0_reverse.detach().to(dev)
    xd = x.to(dev)
    xproj = ops.linear(xd.view(B * L, E), Wih.to(dev), bias.to(dev)).view(B, L, 2, 4 * H)
    li = lengths.to(torch.int32).to(dev)
    out, h_n, c_n, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
    assert (out.cpu() - out_ref).abs().max() < 2e-5
    assert (h_n.cpu() - hn).abs().max() < 2e-5 and (c_n.cpu() - cn).abs().max() < 2e-5
    if True:   # B > 32 takes the GEMM-per-timestep BPTT (the batched deferred path)
        dg = ops.bilstm_bwd(whh_f, whh_b, li, saved, gout.to(dev), ghn.to(dev), gcn.to(dev), H)
        # weight grads from dgates: dW_hh[dir] = sum_t dg^T h_prev
        dgc = dg.cpu()
        dWih = torch.einsum("blg,ble->ge", dgc[:, :, 0], x)
        assert (dWih - lstm.weight_ih_l0.grad).abs().max() < 1e-3 * max(1, lstm.weight_ih_l0.grad.abs().max())
        dWih_r = torch.einsum("blg,ble->ge", dgc[:, :, 1], x)
        assert (dWih_r - lstm.weight_ih_l0_reverse.grad).abs().max() < 1e-3 * max(1, lstm.weight_ih_l0_reverse.grad.abs().max())
        db = dgc[:, :, 0].sum((0, 1))
        assert (db - lstm.bias_ih_l0.grad).abs().max() < 1e-3 * max(1, lstm.bias_ih_l0.grad.abs().max())
        hp = ops.bilstm_hprev(out, H).cpu()
        dWhh = torch.einsum("blg,blh->gh", dgc[:, :, 0], hp[0])
        assert (dWhh - lstm.weight_hh_l0.grad).abs().max() < 1e-3 * max(1, lstm.weight_hh_l0.grad.abs().max())
        dWhh_r = torch.einsum("blg,blh->gh", dgc[:, :, 1], hp[1])
        assert (dWhh_r - lstm.weight_hh_l0_reverse.grad).abs().max() < 1e-3 * max(1, lstm.weight_hh_l0_reverse.grad.abs().max())


def test_attention_group_barrier_timeout_raises(dev):
    """The D-split attention backward's group barrier is bounded like the persistent kernels': a
    timed-out wait NaN-poisons dq / dctx and raises DasaError at the host's next check (bit 4 of the
    error word); the next call runs normally."""
    from dasa_amd import _lib, ops
    g = torch.Generator().manual_seed(5)
    B, D = 6, 2176
    q = (torch.randn(B, D, generator=g) * 0.05).to(dev)
    ctx = torch.rand(B, 36, D, generator=g).to(dev)
    z = torch.randn(B, 5, generator=g).to(dev)
    gw = torch.randn(B, D, generator=g).to(dev)
    ops.attn_set_mode(0)
    ops.check_device_errors()
    _, attn, shifted, wsm = ops.shift_attn_fwd(q, ctx, z)
    dq0, dc0, dz0 = ops.shift_attn_bwd(q, ctx, attn, shifted, wsm, gw)
    assert torch.isfinite(dq0).all() and torch.isfinite(dc0).all()
    ops.force_persist_timeout(True)
    try:
        dq1, dc1, _ = ops.shift_attn_bwd(q, ctx, attn, shifted, wsm, gw)
        torch.cuda.synchronize()
    finally:
        ops.force_persist_timeout(False)
    assert torch.isnan(dq1).all() and torch.isnan(dc1).all()
    with pytest.raises(_lib.DasaError, match="attention: group barrier timed out"):
        ops.check_device_errors()
    dq2, dc2, dz2 = ops.shift_attn_bwd(q, ctx, attn, shifted, wsm, gw)
    assert torch.equal(dq2, dq0) and torch.equal(dc2, dc0) and torch.equal(dz2, dz0)
    ops.check_device_errors()


def test_persistent_barrier_timeout_raises(dev):
    """A persistent bi-LSTM launch whose inter-workgroup barrier times out must not pass for a good
    result: its outputs come back NaN and the host raises DasaError at its next check
    (dasa_set_error_word; test hook dasa_persist_force_timeout makes every barrier time out)."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    B, L, H = 4, 6, 1024
    g = torch.Generator().manual_seed(3)
    xproj = (torch.randn(B, L, 2, 4 * H, generator=g) * 0.1).to(dev)
    whh_f = (torch.randn(4 * H, H, generator=g) * 0.02).to(dev)
    whh_b = (torch.randn(4 * H, H, generator=g) * 0.02).to(dev)
    li = torch.tensor([6, 5, 3, 1], dtype=torch.int32, device=dev)
    assert lib.dasa_bilstm_set_mode(2) == 0        # persistent only
    try:
        ops.check_device_errors()                   # nothing pending
        out, h_n, c_n, saved = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
        assert torch.isfinite(out).all()
        ops.check_device_errors()
        ops.force_persist_timeout(True)
        try:
            out2, h2, c2, _ = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H, save=True)
            dg = ops.bilstm_bwd(whh_f, whh_b, li, saved, torch.ones(B, L, 2 * H, device=dev), None, None, H)
            torch.cuda.synchronize()
        finally:
            ops.force_persist_timeout(False)
        assert torch.isnan(h2).all() and torch.isnan(c2).all() and torch.isnan(out2).all()
        assert torch.isnan(dg).all()
        with pytest.raises(_lib.DasaError, match="barrier timed out"):
            ops.check_device_errors()
        ops.check_device_errors()                   # reported once, then cleared
        out3, _, _, _ = ops.bilstm_fwd(xproj, whh_f, whh_b, li, H)
        assert torch.equal(out3, out)               # and the next launch is healthy again
    finally:
        lib.dasa_bilstm_set_mode(0)


def test_adain_musigma_reverse_dropout(dev):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(19)
    c, s = torch.rand(2, 44, 2048, generator=g), torch.rand(2, 44, 2048, generator=g)

    def ms(x):
        return x.mean(-1, keepdim=True), (x.var(-1, keepdim=True) + 1e-5).sqrt()
    mc, sc = ms(c)
    mss, sss = ms(s)
    ref = (c - mc) / sc * sss + mss
    out = ops.adain_musigma(c.to(dev), s.to(dev)).cpu()
    assert (out - ref).abs().max() < 1e-4
    x = torch.rand(3, 7, 16, generator=g)
    lens = torch.tensor([7, 4, 1], dtype=torch.int32)
    r = ops.reverse_valid(x.to(dev), lens.to(dev)).cpu()
    for b in range(3):
        n = int(lens[b])
        assert torch.equal(r[b, :n], x[b, :n].flip(0)) and (r[b, n:] == 0).all()
    y = ops.dropout(torch.ones(100, 1000, device=dev), 0.4, 1234).cpu()
    keep = (y > 0).float().mean().item()
    assert abs(keep - 0.6) < 0.01 and torch.allclose(y[y > 0], torch.full_like(y[y > 0], 1 / 0.6))
    y2 = ops.dropout(torch.ones(100, 1000, device=dev), 0.4, 1234).cpu()
    assert torch.equal(y, y2)
    # the float4 path and the scalar path (misaligned rows) draw the same (seed, r * cols + c) mask
    buf = torch.ones(100, 1008, device=dev)
    y3 = ops.dropout(buf[:, 1:1001], 0.4, 1234).cpu()
    assert torch.equal(y, y3)
    # mu/sigma AdaIN on strided 2176-float rows (the register path) and a non-2048 width (generic path)
    cf, sf = torch.rand(40, 2176, generator=g), torch.rand(40, 2176, generator=g)
    mc, sc = ms(cf[:, :2048])
    mss, sss = ms(sf[:, :2048])
    outf = torch.zeros(40, 2176, device=dev)
    ops.adain_musigma(cf.to(dev)[:, :2048], sf.to(dev)[:, :2048], out=outf[:, :2048])
    assert (outf[:, :2048].cpu() - ((cf[:, :2048] - mc) / sc * sss + mss)).abs().max() < 1e-4
    assert (outf[:, 2048:] == 0).all()
    c3, s3 = torch.rand(5, 1000, generator=g), torch.rand(5, 1000, generator=g)
    mc, sc = ms(c3)
    mss, sss = ms(s3)
    assert (ops.adain_musigma(c3.to(dev), s3.to(dev)).cpu() - ((c3 - mc) / sc * sss + mss)).abs().max() < 1e-4


def test_policy_head(dev):
    """dasa_policy_head_fwd/bwd (agent_dg.py:832-880) against the PyTorch ops the reference runs:
    masked_fill -> CrossEntropyLoss(sum, ignore_index=-100), argmax + log_softmax gather, Categorical
    entropy / log_prob, and their gradients; the Categorical draw is checked by frequency."""
    from dasa_amd import functional as DF
    g = torch.Generator().manual_seed(21)
    B, C = 37, 19
    logit = torch.randn(B, C, generator=g) * 3
    lens = torch.randint(1, C + 1, (B,), generator=g)
    lens[0] = C
    target = torch.stack([torch.randint(0, int(n), (1,), generator=g)[0] for n in lens])
    target[3] = -100
    mask = torch.arange(C)[None, :] >= lens[:, None]
    w_ent, w_lp = torch.randn(B, generator=g), torch.randn(B, generator=g)
    # reference (CPU fp64)
    x = logit.double().requires_grad_(True)
    z = x.masked_fill(mask, -float("inf"))
    ce = torch.nn.CrossEntropyLoss(ignore_index=-100, reduction="sum")(z, target)
    a_ref = z.max(1)[1]
    lp_ref = torch.log_softmax(z, 1).gather(1, a_ref[:, None])[:, 0]
    cat = torch.distributions.Categorical(torch.softmax(z, 1), validate_args=False)
    ent_ref = cat.entropy()
    (ce * 0.7 + (ent_ref * w_ent.double()).sum() + (lp_ref * w_lp.double()).sum()).backward()
    # product
    xd = logit.to(dev).requires_grad_(True)
    lens32 = lens.to(torch.int32).to(dev)
    ce_d, ent_d, lp_d, a_d = DF.policy_head(xd, lens32, target.to(dev), "argmax")
    (ce_d * 0.7 + (ent_d * w_ent.to(dev)).sum() + (lp_d * w_lp.to(dev)).sum()).backward()
    assert torch.equal(a_d.cpu(), a_ref)
    assert abs(ce_d.item() - ce.item()) < 1e-4 * max(1.0, abs(ce.item()))
    assert (ent_d.cpu().double() - ent_ref).abs().max() < 1e-5
    assert (lp_d.cpu().double() - lp_ref).abs().max() < 1e-5
    assert (xd.grad.cpu().double() - x.grad).abs().max() < 1e-5
    # teacher mode: CE only
    ce_t = DF.policy_head(logit.to(dev), lens32, target.to(dev), "teacher")[0]
    assert abs(ce_t.item() - ce.item()) < 1e-4 * max(1.0, abs(ce.item()))
    # sampling: frequencies of 8192 draws of one row vs its softmax
    N = 8192
    row = torch.randn(1, C, generator=g).repeat(N, 1)
    ln = torch.full((N,), 11, dtype=torch.int32)
    _, _, lps, acts = DF.policy_head(row.to(dev), ln.to(dev), None, "sample")
    acts = acts.cpu()
    assert int(acts.max()) < 11 and int(acts.min()) >= 0
    p = torch.softmax(row[0, :11].double(), 0)
    freq = torch.bincount(acts, minlength=11).double() / N
    assert (freq - p).abs().max() < 0.03
    assert (lps.cpu().double() - torch.log(p)[acts]).abs().max() < 1e-5
    # forced mode: the caller's actions, entropy / log-prob / gradients as torch's fp32
    # Categorical(softmax(z)) computes them (agent_dg.py:874-880), including its clamped log-pmf
    # log(clamp(p, eps, 1 - eps)): rows 0-5 are sharpened so that some probabilities fall below eps
    # (and one action of those rows is forced onto such a candidate) and some rise above 1 - eps
    lf = logit.clone()
    lf[:6] *= 12.0
    a_f = torch.stack([torch.randint(0, int(n), (1,), generator=g)[0] for n in lens])
    x2 = lf.clone().requires_grad_(True)
    z2 = x2.masked_fill(mask, -float("inf"))
    cat2 = torch.distributions.Categorical(torch.softmax(z2, 1), validate_args=False)
    p2 = cat2.probs.detach()
    assert (p2[:6][~mask[:6]] < 1.1920929e-07).any() and (p2[:6] > 1 - 1.1920929e-07).any()
    ent2, lp2 = cat2.entropy(), cat2.log_prob(a_f)
    ce2 = torch.nn.CrossEntropyLoss(ignore_index=-100, reduction="sum")(z2, target)
    (ce2 * 0.3 + (ent2 * w_ent).sum() + (lp2 * w_lp).sum()).backward()
    xf = lf.to(dev).requires_grad_(True)
    ce_f, ent_f, lp_f, a_out = DF.policy_head(xf, lens32, target.to(dev), "forced", forced=a_f.to(dev))
    (ce_f * 0.3 + (ent_f * w_ent.to(dev)).sum() + (lp_f * w_lp.to(dev)).sum()).backward()
    assert torch.equal(a_out.cpu(), a_f)
    assert abs(ce_f.item() - ce2.item()) < 1e-4 * max(1.0, abs(ce2.item()))
    assert (ent_f.cpu() - ent2).abs().max() < 2e-5
    assert (lp_f.cpu() - lp2).abs().max() < 2e-5 * max(1.0, lp2.abs().max().item())
    assert (xf.grad.cpu() - x2.grad).abs().max() < 2e-5 * max(1.0, x2.grad.abs().max().item())


def test_x6_weight_planes_first_use_on_two_streams(dev):
    """ops._x6_weight caches the bf16 planes of a weight per version; the LXRT layer uses one weight
    from its side stream and the main stream (vilmodel.py:309-316). A FRESH weight whose planes are
    built on the side stream and first used on the main stream must wait for the split kernel."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(3)
    M, N, K = 2048, 1024, 768          # 128 output tiles: the bf16x6 path
    x = torch.randn(M, K, generator=g).to(dev)
    ref = None
    side = torch.cuda.Stream(device=dev)
    for trial in range(3):
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev)
        assert ops._emu_ok(M, N, K, K, x)
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            if hasattr(torch.cuda, "_sleep"):
                torch.cuda._sleep(2_000_000)         # keep the side stream busy: the split lags
            y_side = ops.linear(x, W)                # builds the planes on the side stream
        y_main = ops.linear(x, W)                    # first use on the main stream
        main.wait_stream(side)
        ref = (x.double() @ W.double().t())
        for y in (y_side, y_main):
            assert (y.double() - ref).abs().max().item() < 1e-4, trial
        assert torch.equal(y_side, y_main)


def test_adain_musigma_grad_with_aliased_out(dev):
    """adain_musigma(c, s, out=c) on the autograd path (the agent's in-place
    f_t[..., :F] = adain(f_t[..., :F], d_t[..., :F])): the saved content is private, so backward works
    and matches the out-of-place gradient."""
    from dasa_amd import functional as DF
    g = torch.Generator().manual_seed(9)
    c0 = torch.rand(6, 2176, generator=g).to(dev)
    s0 = torch.rand(6, 2176, generator=g).to(dev)
    w = torch.randn(6, 2176, generator=g).to(dev)
    a = c0.clone().requires_grad_(True)
    f = a * 1.0
    DF.adain_musigma(f[:, :2048], s0[:, :2048], out=f[:, :2048])
    (f * w).sum().backward()
    b = c0.clone().requires_grad_(True)
    y = DF.adain_musigma(b[:, :2048], s0[:, :2048])
    ((y * w[:, :2048]).sum() + (b[:, 2048:] * w[:, 2048:]).sum()).backward()
    assert torch.allclose(f[:, :2048], y, atol=1e-6)
    assert (a.grad - b.grad).abs().max().item() < 1e-5


def test_f32_to_bf16_matches_torch_rounding(dev):
    from dasa_amd import ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4096 + 6, generator=g) * 3.0
    x[:6] = torch.tensor([0.0, -0.0, 1e-40, 65504.0, 1.0 + 2.0 ** -8, 1.0 + 3 * 2.0 ** -9])   # ties, subnormal
    y = ops.to_bf16(x.to(dev)).cpu()
    assert torch.equal(y.view(torch.int16), x.to(torch.bfloat16).view(torch.int16))   # RNE, bit-exact


@pytest.mark.parametrize("M,N,K", [(20480, 3072, 768), (1040, 2048, 2048), (300, 130, 64), (1, 1024, 2240),
                                   (517, 768, 3072), (9216, 768, 2176)])
def test_gemm_bf16(dev, M, N, K):
    """bf16-operand GEMM (configs[4]) against fp64 host math on the SAME bf16-rounded operands: bf16
    products are exact in fp32, so the only error is fp32 accumulation (~1e-6 of sum|a*b|)."""
    from dasa_amd import ops, _lib
    g = torch.Generator().manual_seed(M + N + K)
    x = _rand(M, K, g=g)
    W = _rand(N, K, g=g, scale=0.05)
    b = _rand(N, g=g)
    xb, Wb = x.to(torch.bfloat16).double(), W.to(torch.bfloat16).double()
    L = _lib.lib()
    for cfg in [(1 << 20) + c for c in range(11)] + [-1]:
        L.dasa_gemm_force_config(cfg)
        try:
            with torch.no_grad(), ops.bf16_matmul():
                y = ops.linear(x.to(dev), W.to(dev), b.to(dev), act="gelu").cpu().double()
        finally:
            L.dasa_gemm_force_config(-1)
        z = xb @ Wb.t() + b.double()
        ref = 0.5 * z * (1.0 + torch.erf(z / math.sqrt(2.0)))
        scale = (xb.abs() @ Wb.abs().t()).max().item()
        assert (y - ref).abs().max().item() < 2e-6 * scale + 1e-6, cfg


def test_gemm_bf16_epilogue_and_strides(dev):
    """aux gate, column scale, beta accumulate and a row-strided A (the AdaIN feature layout, ld 2176)."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(5)
    M, N, K = 333, 2048, 2048
    buf = _rand(M, 2176, g=g)
    W = _rand(N, K, g=g, scale=0.05)
    b = _rand(N, g=g)
    aux = _rand(M, N, g=g)
    cs = _rand(N, g=g)
    c0 = _rand(M, N, g=g)
    xb, Wb = buf[:, :K].to(torch.bfloat16).double(), W.to(torch.bfloat16).double()
    out = c0.to(dev)
    with torch.no_grad(), ops.bf16_matmul():
        ops.linear(buf.to(dev)[:, :K], W.to(dev), b.to(dev), act="sigmoid", aux=aux.to(dev), colscale=cs.to(dev),
                   out=out, beta=0.5)
    ref = torch.sigmoid(xb @ Wb.t() + b.double()) * aux.double() * cs.double() + 0.5 * c0.double()
    assert (out.cpu().double() - ref).abs().max().item() < 2e-5


@pytest.mark.parametrize("M", [300, 5120])
def test_gemm_bf16_activations(dev, M):
    """dasa_gemm_bf16_ex (configs[4]'s FFN with bf16 activations): the bf16-stored GELU output equals the
    fp32 output rounded to bf16 (RNE, torch's rounding) bit for bit, and the FFN-down GEMM reading it as
    bf16 equals the one reading the fp32 tensor (rounded on load) bit for bit — both tile forms (M = 300:
    128 x 128; M = 5120: 256 x 256)."""
    from dasa_amd import ops, _lib
    g = torch.Generator().manual_seed(M)
    N, K = 3072, 768
    x = _rand(M, K, g=g).to(dev)
    W1, b1 = _rand(N, K, g=g, scale=0.05).to(dev), _rand(N, g=g).to(dev)
    W2, b2 = _rand(K, N, g=g, scale=0.05).to(dev), _rand(K, g=g).to(dev)
    with torch.no_grad(), ops.bf16_matmul():
        assert ops.bf16_acts_ok(x, N)
        h32 = ops.linear(x, W1, b1, act="gelu")
        hbf = ops.linear(x, W1, b1, act="gelu", out_dtype=torch.bfloat16)
        assert hbf.dtype == torch.bfloat16
        assert torch.equal(hbf.view(torch.int16), h32.to(torch.bfloat16).view(torch.int16))
        z32 = ops.linear(h32, W2, b2)
        zbf = ops.linear(hbf, W2, b2)
        zbb = ops.linear(hbf, W2, b2, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(z32, zbf)
    assert torch.equal(zbb.view(torch.int16), z32.to(torch.bfloat16).view(torch.int16))
    with torch.no_grad(), pytest.raises(_lib.DasaError):     # bf16 activations only in bf16 matmul mode
        ops.linear(hbf, W2, b2)


@pytest.mark.parametrize("M,N,K,cbf", [(777, 200, 192, False), (300, 3072, 768, True), (9216, 768, 3072, False),
                                       (20480, 2304, 768, True), (65, 64, 64, False)])
def test_gemm_bf16_dma_matches_register_staged(dev, M, N, K, cbf):
    """The LDS-DMA bf16 GEMM probe form (A already bf16: gemm_bf16_dma_kernel, 256 x 128 / 128 x 128 tiles,
    switched on by dasa_gemm_bf16_dma) against the register-staged default (forced through a bf16 tile form): the same MFMAs over
    the same K order, so bitwise equal - row / column tails, bias + activation epilogue, fp32 and bf16 C."""
    from dasa_amd import ops, _lib
    g = torch.Generator().manual_seed(M + N + K)
    x = _rand(M, K, g=g).to(dev)
    W, b = _rand(N, K, g=g, scale=0.05).to(dev), _rand(N, g=g).to(dev)
    od = torch.bfloat16 if cbf else None
    with torch.no_grad(), ops.bf16_matmul():
        xb = ops.to_bf16(x)
        prev = _lib.lib().dasa_gemm_bf16_dma(1)
        try:
            y_dma = ops.linear(xb, W, b, act="gelu", out_dtype=od)
        finally:
            _lib.lib().dasa_gemm_bf16_dma(prev)
        lib = _lib.lib()
        lib.dasa_gemm_force_config((1 << 20) + (9 if M * N >= 200 * 256 * 256 else 2))
        try:
            y_reg = ops.linear(xb, W, b, act="gelu", out_dtype=od)
        finally:
            lib.dasa_gemm_force_config(-1)
    torch.cuda.synchronize()
    assert torch.equal(y_dma.view(torch.int16) if cbf else y_dma, y_reg.view(torch.int16) if cbf else y_reg)


@pytest.mark.parametrize("M", [300, 5120])
def test_layernorm_bf16_twin(dev, M):
    """configs[4]'s bf16 mode: LayerNorm also writes bf16(y) (dasa_layernorm_fwd_bf16) and the next bf16 GEMM takes
    it as its A operand. y is bitwise the plain LayerNorm's, the twin is torch's RNE rounding of y bit for bit,
    and the GEMM reading the twin equals the GEMM rounding the fp32 y on load bit for bit (both tile forms)."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(M + 1)
    K, N = 768, 2304
    x, r = _rand(M, K, g=g).to(dev), _rand(M, K, g=g).to(dev)
    gam, bet = (1 + _rand(K, g=g, scale=0.1)).to(dev), _rand(K, g=g, scale=0.1).to(dev)
    W, b = _rand(N, K, g=g, scale=0.05).to(dev), _rand(N, g=g).to(dev)
    y_plain = ops.layernorm(x, gam, bet, 1e-12, res=r)
    assert getattr(y_plain, "_dasa_bf16", None) is None
    with torch.no_grad(), ops.bf16_matmul():
        y = ops.layernorm(x, gam, bet, 1e-12, res=r)
        twin = y._dasa_bf16[0]
        z_twin = ops.linear(y, W, b)
        z_load = ops.linear(y.clone(), W, b)       # no twin: A rounded on load
    torch.cuda.synchronize()
    assert torch.equal(y, y_plain)
    assert torch.equal(twin.view(torch.int16), y.to(torch.bfloat16).view(torch.int16))
    assert torch.equal(z_twin, z_load)


@pytest.mark.parametrize("B,Lq,Lk", [(3, 80, 80), (5, 36, 80), (4, 80, 36), (2, 128, 117), (7, 1, 5)])
def test_mha_bf16(dev, B, Lq, Lk):
    """configs[4]'s bf16 attention core (dasa_mha_fwd_bf16) through ops.mha under bf16_matmul: Q/K/V are
    strided views of a fused bf16 QKV buffer, a -10000 key-padding mask. Against a float64 restatement that
    takes the same bf16 Q/K/V and rounds the softmax P to bf16 (RNE) before P V, as the kernel does: within
    2e-3 (P's rounding can flip at a tie boundary; the fp32 QK^T / softmax differ from float64 by ~1e-7);
    the bf16 output is bitwise the fp32 output rounded (RNE)."""
    from dasa_amd import ops, _lib
    heads, dh = 12, 64
    Hd = heads * dh
    g = torch.Generator().manual_seed(B * 1000 + Lq + Lk)
    if Lq == Lk:
        qkv = torch.randn(B, Lq, 3 * Hd, generator=g).to(torch.bfloat16).to(dev)
        Q, K, V = qkv[..., :Hd], qkv[..., Hd:2 * Hd], qkv[..., 2 * Hd:]
    else:
        Q = torch.randn(B, Lq, Hd, generator=g).to(torch.bfloat16).to(dev)
        kv = torch.randn(B, Lk, 2 * Hd, generator=g).to(torch.bfloat16).to(dev)
        K, V = kv[..., :Hd], kv[..., Hd:]
    mask = torch.zeros(B, Lk)
    for b in range(B):
        mask[b, max(1, Lk - 3 * b):] = -10000.0
    mask = mask.to(dev)
    scale = 1.0 / 8.0
    with torch.no_grad(), ops.bf16_matmul():
        out_bf = ops.mha(Q, K, V, mask, heads, scale)
        out32 = torch.empty(B, Lq, Hd, device=dev)
        rc = _lib.lib().dasa_mha_fwd_bf16(Q.data_ptr(), Q.stride(1), K.data_ptr(), K.stride(1), V.data_ptr(),
                                          V.stride(1), mask.data_ptr(), out32.data_ptr(), Hd, 0, B, heads, Lq, Lk, dh,
                                          scale, 0.0, 0, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
    torch.cuda.synchronize()
    assert out_bf.dtype == torch.bfloat16
    q = Q.double().view(B, Lq, heads, dh).transpose(1, 2)
    k = K.double().view(B, Lk, heads, dh).transpose(1, 2)
    v = V.double().view(B, Lk, heads, dh).transpose(1, 2)
    s = q @ k.transpose(-1, -2) * scale + mask.double()[:, None, None, :]
    p = torch.softmax(s, -1).float().to(torch.bfloat16).double()
    ref = (p @ v).transpose(1, 2).reshape(B, Lq, Hd)
    err = (out32.double() - ref).abs().max().item()
    assert err < 2e-3, err
    assert torch.equal(out_bf.view(torch.int16), out32.to(torch.bfloat16).view(torch.int16))
    with torch.no_grad(), pytest.raises(_lib.DasaError):   # bf16 operands only in bf16 matmul mode
        ops.mha(Q, K, V, mask, heads, scale)


def test_bf16_mode_is_forward_only(dev):
    from dasa_amd import ops, _lib
    with pytest.raises(_lib.DasaError):
        with ops.bf16_matmul():
            pass


def test_split3_bf16_exact(dev):
    """dasa_f32_split3_bf16: x = hi + mid + lo exactly (fp64 sum) for normal fp32 values, each plane a
    bf16 (RNE of the running residual)."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(11)
    x = torch.cat([torch.randn(64, 96, generator=g) * s for s in (1e-3, 1.0, 1e3)], 0)
    x[0, :8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.4e37, -2.5e-30, 1 / 3, 65504.0])
    pl = ops.split3_bf16(x.to(dev)).cpu()
    hi, mid, lo = (pl[i].double() for i in range(3))
    assert torch.equal(hi + mid + lo, x.double())
    assert torch.equal(pl[0], x.to(torch.bfloat16))                       # hi = RNE(x)
    assert torch.equal(pl[1], (x.double() - hi).float().to(torch.bfloat16))


@pytest.mark.parametrize("M,N,K", [(517, 200, 96), (1030, 384, 768), (256, 128, 32), (3, 24, 64)])
def test_gemm_f32x6(dev, M, N, K):
    """The bf16x6 fp32-emulated GEMM (dasa_gemm_f32x6), every tile form, ragged edges, the fused
    epilogue (bias, act, aux gate, column scale, beta) and a strided A: its error against fp64 is at
    most that of the native fp32 MFMA GEMM (+10%)."""
    from dasa_amd import _lib, ops
    g = torch.Generator().manual_seed(M + N + K)
    Abuf = torch.randn(M, K + 8, generator=g)
    A = Abuf[:, 4:4 + K]                                     # lda = K + 8, 16-B aligned start
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.1
    aux = torch.rand(M, N, generator=g)
    cs = torch.rand(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = (A.double() @ W.double().t() + bias.double())
    Ad, Wd = Abuf.to(dev)[:, 4:4 + K], W.to(dev)
    planes = ops.split3_bf16(Wd)
    lib = _lib.lib()
    out_nat = torch.empty(M, N, device=dev)
    ops.gemm(Ad, Wd, out_nat, M=M, N=N, K=K, lda=K + 8, ldb=K, ldc=N, bias=bias.to(dev))
    err_nat = (out_nat.cpu().double() - ref).abs().max().item()
    try:
        outs = {}
        for cfg in list(range(10)) + [15, 16, 20, 21, 22, 26]:
            lib.dasa_gemm_force_config((1 << 21) + cfg)
            y = torch.empty(M, N, device=dev)
            ops.gemm_f32x6(Ad, planes, y, M=M, N=N, K=K, lda=K + 8, ldc=N, bias=bias.to(dev))
            outs[cfg] = y.cpu()
            err = (y.cpu().double() - ref).abs().max().item()
            # forms 0, 3, 4, 5, 7, 8 keep the five small products in their own accumulator (default 8):
            # at most the native fp32 kernel's error; forms 1, 2, 6, 15 (one accumulator) within 3x
            assert err <= (3.0 if cfg in (1, 2, 6, 15) else 1.1) * err_nat + 1e-7, (cfg, err, err_nat)
            y2 = c0.clone().to(dev)
            ops.gemm_f32x6(Ad, planes, y2, M=M, N=N, K=K, lda=K + 8, ldc=N, bias=bias.to(dev), act="sigmoid",
                           aux=aux.to(dev), ld_aux=N, colscale=cs.to(dev), beta=0.5)
            want = torch.sigmoid(ref) * aux.double() * cs.double() + 0.5 * c0.double()
            assert (y2.cpu().double() - want).abs().max().item() < 1e-5, cfg
        # form 16 runs form 8's products in form 8's order: bitwise equal to form 8 without split-K (the
        # forced form-8 run above may split K on few-tile shapes)
        lib.dasa_gemm_force_config((1 << 21) + 8 + 32 * 1)
        y8 = torch.empty(M, N, device=dev)
        ops.gemm_f32x6(Ad, planes, y8, M=M, N=N, K=K, lda=K + 8, ldc=N, bias=bias.to(dev))
        for cfg in (16, 20, 21, 22, 26):   # all-DMA, one-LDS-stage, register-A, interleaved forms: form 8 order
            assert torch.equal(outs[cfg], y8.cpu()), cfg
    finally:
        lib.dasa_gemm_force_config(-1)


@pytest.mark.parametrize("M,N,K", [(1664, 1280, 768), (12800, 768, 768)])
def test_gemm_f32x6_balanced_split(dev, M, N, K):
    """Many output tiles whose last round would leave most CUs idle (130 tiles: 0.51 of a round; 600:
    2.34 rounds), with the opt-in balanced plan (dasa_gemm_x6_set_balance(1)): K split 3- / 2-way and
    reduced in-kernel. Error against fp64 at most the native kernel's (+10%) and the unsplit form's,
    bitwise-deterministic repeats."""
    from dasa_amd import _lib, ops
    _lib.lib().dasa_gemm_x6_set_balance(1)
    ops._X6_WS_NEED.clear()
    try:
        _balanced_split_case(dev, M, N, K)
    finally:
        _lib.lib().dasa_gemm_x6_set_balance(0)
        ops._X6_WS_NEED.clear()


def _balanced_split_case(dev, M, N, K):
    from dasa_amd import _lib, ops
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.1
    ref = (A.double() @ W.double().t() + bias.double())
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    planes = ops.split3_bf16(Wd)
    lib = _lib.lib()
    d = ops.GemmDesc()
    d.M, d.N, d.K, d.batch, d.opA, d.opB, d.lda, d.ldb, d.ldc = M, N, K, 1, 0, 1, K, K, N
    assert lib.dasa_gemm_f32x6_workspace(ctypes.byref(d)) > 0          # the plan splits
    out_nat = torch.empty(M, N, device=dev)
    ops.gemm(Ad, Wd, out_nat, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bd)
    err_nat = (out_nat.cpu().double() - ref).abs().max().item()
    outs = []
    for _ in range(2):
        y = torch.full((M, N), float("nan"), device=dev)
        ops.gemm_f32x6(Ad, planes, y, M=M, N=N, K=K, lda=K, ldc=N, bias=bd)
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1])
    err = (outs[0].double() - ref).abs().max().item()
    try:
        lib.dasa_gemm_force_config((1 << 21) + 8 + 32 * 1)                 # form 8, one split
        ops._X6_WS_NEED.clear()
        y1 = torch.empty(M, N, device=dev)
        ops.gemm_f32x6(Ad, planes, y1, M=M, N=N, K=K, lda=K, ldc=N, bias=bd)
        err1 = (y1.cpu().double() - ref).abs().max().item()
    finally:
        lib.dasa_gemm_force_config(-1)
        ops._X6_WS_NEED.clear()
    assert err <= 1.1 * err_nat + 1e-7 and err <= 1.5 * err1 + 1e-7, (err, err_nat, err1)


@pytest.mark.parametrize("M,N,K", [(130, 200, 1000), (512, 768, 70001), (4096, 768, 9000), (6, 2, 33)])
def test_gemm_f32x6_tn(dev, M, N, K):
    """The bf16x6 TN weight-gradient GEMM (dasa_gemm_f32x6_tn: C = alpha AᵀB + beta C, both operands K-major and
    split in-kernel), both forms, planned and forced split counts, ragged M / N tiles, K not a multiple of the
    32-deep step, strided A / B: error against fp64 at most the native fp32 kernel's (+10 %), the alpha / beta
    epilogue, every element of a NaN-filled C written, bitwise-deterministic repeats."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    lda, ldb = M + 6, N + 4
    A = (torch.randn(K, lda, device=dev, generator=g) * 0.1)[:, 2:2 + M]
    B = torch.randn(K, ldb, device=dev, generator=g)[:, :N]
    c0 = torch.randn(M, N, device=dev, generator=g)
    ref = A.double().t() @ B.double()
    y_nat = torch.empty(M, N, device=dev)
    ops.gemm(A, B, y_nat, M=M, N=N, K=K, opA=1, opB=0, lda=lda, ldb=ldb, ldc=N)
    err_nat = (y_nat.double() - ref).abs().max().item()
    try:
        for form in (0, 1):
            for spl in (-1, 1, 3):
                assert lib.dasa_gemm_x6_tn_config(form, spl) == 0
                outs = []
                for _ in range(2):
                    y = torch.full((M, N), float("nan"), device=dev)
                    ops.gemm_f32x6_tn(A, B, y, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N)
                    outs.append(y)
                assert torch.equal(outs[0], outs[1]), (form, spl)
                err = (outs[0].double() - ref).abs().max().item()
                assert err <= 1.1 * err_nat + 1e-6, (form, spl, err, err_nat)
                y2 = c0.clone()
                ops.gemm_f32x6_tn(A, B, y2, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N, alpha=-0.5, beta=0.25)
                want = -0.5 * ref + 0.25 * c0.double()
                assert (y2.double() - want).abs().max().item() <= 0.55 * err_nat + 1e-5, (form, spl)
    finally:
        lib.dasa_gemm_x6_tn_config(-1, -1)
    # ops.matmul_tn takes the TN kernel for long K
    if ops._tn_x6_ok(A, B, M, N, K, lda, ldb):
        y3 = ops.matmul_tn(A, B)
        assert (y3.double() - ref).abs().max().item() <= 1.1 * err_nat + 1e-6


@pytest.mark.parametrize("M,N,K", [(12800, 768, 3072), (11200, 768, 768)])
def test_gemm_f32x6_tail_plan(dev, M, N, K):
    """the default plan's whole-rounds + split-K tail (two launches over row bands, offset A / C /
    aux pointers for the second band) on the language-pipe shapes that take it, with every epilogue term (bias,
    sigmoid, aux gate, column scale, beta 0.5). Against fp64 (at most the native fp32 kernel's error, +10 %)
    and against the one-launch plan (dasa_gemm_x6_set_tail(0)) on the same inputs; bitwise-deterministic."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    aux = torch.rand(M, N, device=dev, generator=g)
    cs = torch.rand(N, device=dev, generator=g)
    c0 = torch.randn(M, N, device=dev, generator=g)
    planes = ops.split3_bf16(W)
    lin = A.double() @ W.double().t() + bias.double()
    want = torch.sigmoid(lin) * aux.double() * cs.double() + 0.5 * c0.double()
    out_nat = torch.empty(M, N, device=dev)
    ops.gemm(A, W, out_nat, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias)
    err_nat = (out_nat.double() - lin).abs().max().item()
    d = ops.GemmDesc()
    d.M, d.N, d.K, d.batch, d.opA, d.opB, d.lda, d.ldb, d.ldc = M, N, K, 1, 0, 1, K, K, N
    res = {}
    try:
        for tail in (1, 0):
            assert lib.dasa_gemm_x6_set_tail(tail) == 0
            ops._X6_WS_NEED.clear()
            ws = lib.dasa_gemm_f32x6_workspace(ctypes.byref(d))
            assert lib.dasa_gemm_f32x6_kernels(ctypes.byref(d), ws) == (2 if tail else 1), tail
            runs = []
            for _ in range(2):
                y = torch.full((M, N), float("nan"), device=dev)
                ops.gemm_f32x6(A, planes, y, M=M, N=N, K=K, lda=K, ldc=N, bias=bias)
                y2 = c0.clone()
                ops.gemm_f32x6(A, planes, y2, M=M, N=N, K=K, lda=K, ldc=N, bias=bias, act="sigmoid", aux=aux,
                               ld_aux=N, colscale=cs, beta=0.5)
                runs.append((y, y2))
            assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1]), tail
            y, y2 = runs[0]
            err = (y.double() - lin).abs().max().item()
            assert err <= 1.1 * err_nat + 1e-7, (tail, err, err_nat)
            assert (y2.double() - want).abs().max().item() < 1e-5, tail
            res[tail] = (y, y2)
    finally:
        lib.dasa_gemm_x6_set_tail(1)
        ops._X6_WS_NEED.clear()
    # the two plans sum K in other orders: equal to fp32 rounding of the same products
    for a, b in zip(res[0], res[1]):
        assert (a - b).abs().max().item() <= 4 * err_nat + 1e-6


@pytest.mark.parametrize("M,N,K", [(517, 200, 768), (720, 768, 768), (1600, 768, 3072), (100, 2048, 2048),
                                   (3, 24, 256)])
def test_gemm_f32x6_splitk(dev, M, N, K):
    """The split-K bf16x6 forms (few output tiles: K split over several workgroups per tile, reduced
    in-kernel by the last split to arrive): error against fp64 at most the native kernel's (+10%), the
    fused epilogue applied once, bitwise-deterministic repeats, and the arrival counters re-armed
    (every call writes every element of a NaN-filled output)."""
    from dasa_amd import _lib, ops
    g = torch.Generator().manual_seed(M * 7 + N + K)
    Abuf = torch.randn(M, K + 8, generator=g)
    A = Abuf[:, 4:4 + K]
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.1
    aux = torch.rand(M, N, generator=g)
    cs = torch.rand(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = (A.double() @ W.double().t() + bias.double())
    Ad, Wd, bd = Abuf.to(dev)[:, 4:4 + K], W.to(dev), bias.to(dev)
    planes = ops.split3_bf16(Wd)
    lib = _lib.lib()
    out_nat = torch.empty(M, N, device=dev)
    ops.gemm(Ad, Wd, out_nat, M=M, N=N, K=K, lda=K + 8, ldb=K, ldc=N, bias=bd)
    err_nat = (out_nat.cpu().double() - ref).abs().max().item()
    try:
        for cfg, spl in ((8, 0), (8, 2), (8, 3), (4, 2), (4, 5), (5, 3)):
            lib.dasa_gemm_force_config((1 << 21) + cfg + 32 * spl if spl else -1)
            outs = []
            for _ in range(3):
                y = torch.full((M, N), float("nan"), device=dev)
                ops.gemm_f32x6(Ad, planes, y, M=M, N=N, K=K, lda=K + 8, ldc=N, bias=bd)
                outs.append(y.cpu())
            err = (outs[0].double() - ref).abs().max().item()
            assert err <= 1.1 * err_nat + 1e-7, (cfg, spl, err, err_nat)
            assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]), (cfg, spl)
            y2 = c0.clone().to(dev)
            ops.gemm_f32x6(Ad, planes, y2, M=M, N=N, K=K, lda=K + 8, ldc=N, bias=bd, act="sigmoid",
                           aux=aux.to(dev), ld_aux=N, colscale=cs.to(dev), beta=0.5)
            want = torch.sigmoid(ref) * aux.double() * cs.double() + 0.5 * c0.double()
            assert (y2.cpu().double() - want).abs().max().item() < 1e-5, (cfg, spl)
    finally:
        lib.dasa_gemm_force_config(-1)


@pytest.mark.parametrize("M,N,K", [(20, 2176, 1024), (20, 4096, 2240), (64, 1000, 512), (1, 1, 32), (7, 130, 96),
                                   (32, 3072, 3072)])
def test_gemm_skinny(dev, M, N, K):
    """Skinny NT GEMMs (the per-step decoder / critic linears at B <= 64: split-K + reduce), the fused
    epilogue and a strided A, against fp64."""
    from dasa_amd import ops
    g = torch.Generator().manual_seed(M * 31 + N + K)
    Abuf = _rand(M, K + 4, g=g)
    W, b = _rand(N, K, g=g, scale=0.05), _rand(N, g=g)
    aux, cs, c0 = _rand(M, N, g=g), _rand(N, g=g), _rand(M, N, g=g)
    z = Abuf[:, :K].double() @ W.double().t() + b.double()
    y = ops.linear(Abuf.to(dev)[:, :K], W.to(dev), b.to(dev)).cpu()
    assert (y.double() - z).abs().max().item() < 2e-6 * max(1.0, z.abs().max().item()) * math.sqrt(K / 256)
    out = c0.clone().to(dev)
    ops.linear(Abuf.to(dev)[:, :K], W.to(dev), b.to(dev), act="tanh", aux=aux.to(dev), colscale=cs.to(dev), out=out,
               beta=0.25)
    want = torch.tanh(z) * aux.double() * cs.double() + 0.25 * c0.double()
    assert (out.cpu().double() - want).abs().max().item() < 1e-5


# (M, N, K): the decoder / critic / attention shapes at B = 20 (model.py:263-264, 437, 970-982) and
# their input gradients, M at the 16 / 32 column-tile edges, N not a multiple of the 16 / 64 column
# block, K not a multiple of the 32-deep step, K shorter than one step, many K splits.
SKINNY_NT = [(20, 2176, 1024), (20, 4096, 2240), (20, 1024, 2048), (20, 4096, 1024), (20, 1024, 3072),
             (1, 5, 1024), (16, 64, 128), (17, 2000, 700), (32, 130, 36), (2, 4096, 8), (31, 48, 12288),
             (19, 37, 12), (20, 520, 5000)]
SKINNY_NN = [(20, 1024, 2176), (20, 2240, 4096), (20, 2048, 1024), (20, 3072, 1024), (1, 8, 1024),
             (16, 68, 100), (17, 1000, 4), (32, 4096, 300), (5, 2176, 12288)]


def _skinny_modes():
    """(target waves, ks) plans to force: the default, the widest-K and the narrowest-K form, and the
    17..20-row shapes without the hybrid MFMA + VALU form (ks + 16)."""
    return [(-1, -1), (-1, 8), (100000, 1), (-1, 16), (100000, 17)]


@pytest.mark.parametrize("M,N,K", SKINNY_NT)
def test_gemm_skinny_nt_kernel(dev, M, N, K):
    """The weight-streaming skinny NT kernel (gemm_skinny_nt_kernel: W on the MFMA row side, K split in
    and across workgroups, last-arriver partial sum) in its default and forced K-split forms, plain and
    with the full fused epilogue, against fp64; bitwise deterministic across repeats."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    g = torch.Generator().manual_seed(M * 131 + N + K)
    Abuf = _rand(M, K + 8, g=g)
    W, b = _rand(N, K, g=g, scale=0.05), _rand(N, g=g)
    aux, cs, c0 = _rand(M, N, g=g), _rand(N, g=g), _rand(M, N, g=g)
    z = Abuf[:, :K].double() @ W.double().t() + b.double()
    tol = 2e-6 * max(1.0, z.abs().max().item()) * math.sqrt(max(1, K) / 256)
    Ad, Wd, bd = Abuf.to(dev)[:, :K], W.to(dev), b.to(dev)
    try:
        for waves, ks in _skinny_modes():
            lib.dasa_gemm_skinny_tune(waves, ks)
            y = ops.linear(Ad, Wd, bd)
            y2 = ops.linear(Ad, Wd, bd)
            assert torch.equal(y, y2), (waves, ks)
            assert (y.cpu().double() - z).abs().max().item() < tol, (waves, ks)
            out = c0.clone().to(dev)
            ops.linear(Ad, Wd, bd, act="sigmoid", aux=aux.to(dev), colscale=cs.to(dev), out=out, beta=0.5)
            want = torch.sigmoid(z) * aux.double() * cs.double() + 0.5 * c0.double()
            assert (out.cpu().double() - want).abs().max().item() < 1e-5, (waves, ks)
    finally:
        lib.dasa_gemm_skinny_tune(-1, -1)


@pytest.mark.parametrize("M,N,K", SKINNY_NN)
def test_gemm_skinny_nn_kernel(dev, M, N, K):
    """The skinny NN kernel (gemm_skinny_nn_kernel: dX = dY . W of an nn.Linear, W read along its rows)
    in its default and forced forms, with beta accumulation and a strided dY, against fp64."""
    from dasa_amd import _lib, ops
    lib = _lib.lib()
    g = torch.Generator().manual_seed(M * 17 + N * 3 + K)
    Abuf = _rand(M, K + 4, g=g)
    B = _rand(K, N, g=g, scale=0.05)
    c0 = _rand(M, N, g=g)
    z = Abuf[:, :K].double() @ B.double()
    tol = 2e-6 * max(1.0, z.abs().max().item()) * math.sqrt(max(1, K) / 256)
    Ad, Bd = Abuf.to(dev)[:, :K], B.to(dev)
    try:
        for waves, ks in _skinny_modes():
            lib.dasa_gemm_skinny_tune(waves, ks)
            y = ops.matmul_nn(Ad, Bd)
            assert torch.equal(y, ops.matmul_nn(Ad, Bd)), (waves, ks)
            assert (y.cpu().double() - z).abs().max().item() < tol, (waves, ks)
            out = c0.clone().to(dev)
            ops.matmul_nn(Ad, Bd, out=out, beta=1.0)
            assert (out.cpu().double() - (z + c0.double())).abs().max().item() < tol + 1e-6, (waves, ks)
    finally:
        lib.dasa_gemm_skinny_tune(-1, -1)


def test_copy_many(dev):
    """ops.copy_many (dasa_copy_segments, the batched static-buffer copies around graph replays): padded
    3-D destinations, strided and expanded sources, bool / int64 / bf16 / 0-dim tensors and more pairs than
    one launch takes (16), each equal to torch's copy_ bit for bit."""
    from dasa_amd import ops
    g = torch.Generator(device=dev).manual_seed(3)
    pairs, refs = [], []

    def add(src, dst):
        ref = dst.clone()
        ref.copy_(src)
        pairs.append((src, dst))
        refs.append(ref)
    big = torch.zeros(20, 96, 2048, device=dev)
    add(torch.rand(20, 80, 2048, device=dev, generator=g), big[:, :80])
    add(torch.rand(20, 16, 2176, device=dev, generator=g)[:, :5], torch.zeros(20, 32, 2176, device=dev)[:, :5])
    add(torch.rand(20, 1024, device=dev, generator=g).t(), torch.zeros(1024, 20, device=dev))
    add(torch.ones(1, device=dev).expand(20, 1024), torch.zeros(20, 1024, device=dev))
    add(torch.rand(20, 80, device=dev, generator=g) < 0.5, torch.ones(20, 96, dtype=torch.bool, device=dev)[:, :80])
    add(torch.randint(0, 9, (20,), device=dev, generator=g), torch.zeros(20, dtype=torch.int64, device=dev))
    add(torch.rand(7, 33, device=dev, generator=g).to(torch.bfloat16), torch.zeros(7, 33, dtype=torch.bfloat16, device=dev))
    add(torch.tensor(3.5, device=dev), torch.zeros((), device=dev))
    add(torch.rand(3, 5, 7, 9, device=dev, generator=g)[:, 1:4, :, :8], torch.zeros(3, 3, 7, 8, device=dev))
    for i in range(14):
        add(torch.rand(i + 1, 13, device=dev, generator=g), torch.zeros(i + 1, 13, device=dev))
    ops.copy_many(pairs)
    torch.cuda.synchronize()
    for (src, dst), ref in zip(pairs, refs):
        assert torch.equal(dst, ref), (src.shape, src.stride(), dst.stride())
    assert torch.equal(big[:, 80:], torch.zeros_like(big[:, 80:]))     # the padding stayed untouched
