"""Bitwise run-to-run determinism of the kernels with in-launch hand-offs (split-K / last-arriver
merges, the persistent bi-LSTM's state exchange) at the sampled rollout's shapes (B = 20).

Every case is deterministic by design (fixed merge order), so two calls on the same input must give the
same bits. Two inputs alternate call by call, so a consumer that read a partial / state word left by the
PREVIOUS call at the same workspace address (a stale line) shows up as a mismatch against the first
result for its input. A side stream keeps a 12800-row bf16x6 GEMM running meanwhile (the language pipe's
load). Prints mismatching calls per case.
    python tools/determinism_stress.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402


def _native(x, W):
    y = torch.empty(x.shape[0], W.shape[0], device=x.device)
    ops.gemm(x, W, y, M=x.shape[0], N=W.shape[0], K=x.shape[1], lda=x.shape[1], ldb=W.shape[1], ldc=W.shape[0])
    return y


def cases(dev, g):
    def rnd(*s, scale=1.0):
        return torch.randn(*s, device=dev, generator=g) * scale
    out = []
    # bf16x6 split-K plans (few output tiles, long K): LXRT / BPTT shapes
    for M, N, K in ((720, 768, 3072), (1600, 768, 3072), (1400, 1024, 4096)):
        W = rnd(N, K, scale=0.02)
        xs = (rnd(M, K), rnd(M, K))
        out.append((f"x6 {M}x{N}x{K}", xs, lambda x, W=W: ops.linear(x, W)))
    # weight-streaming skinny GEMMs at M = 20 (split over workgroups, last arriver sums)
    for N, K in ((2176, 1024), (2048, 1024), (4096, 2240), (4096, 1024), (1024, 3072)):
        W = rnd(N, K, scale=0.02)
        xs = (rnd(20, K), rnd(20, K))
        out.append((f"skinny {N}x{K}", xs, lambda x, W=W: ops.linear(x, W)))
    Wn = rnd(4096, 2240, scale=0.02)
    out.append(("skinny_nn 20x4096.4096x2240", (rnd(20, 4096), rnd(20, 4096)), lambda x: ops.matmul_nn(x, Wn)))
    # attention at B = 20
    ctx, mask = rnd(20, 80, 2048, scale=0.2), torch.zeros(20, 80, dtype=torch.bool, device=dev)
    mask[3, 50:] = True
    out.append(("softdot B20", (rnd(20, 2048, scale=0.05), rnd(20, 2048, scale=0.05)),
                lambda q: torch.cat([t for t in ops.softdot_fwd(q, ctx, mask)], 1)))
    def sd_mode(q, mode):
        ops.attn_set_mode(mode)
        try:
            return torch.cat([t for t in ops.softdot_fwd(q, ctx, mask)], 1)
        finally:
            ops.attn_set_mode(0)
    out.append(("softdot B20 split2", (rnd(20, 2048, scale=0.05), rnd(20, 2048, scale=0.05)),
                lambda q: sd_mode(q, 2)))
    _, pr, _ = ops.softdot_fwd(rnd(20, 2048, scale=0.05), ctx, mask)
    qb = rnd(20, 2048, scale=0.05)
    out.append(("softdot_bwd B20", (rnd(20, 2048), rnd(20, 2048)),
                lambda dw: torch.cat([ops.softdot_bwd(qb, ctx, pr, dwctx=dw)[0],
                                      ops.softdot_bwd(qb, ctx, pr, dwctx=dw)[1].flatten(1)], 1)))
    # B = 256 (configs[4]'s eval rollout): the instruction SoftDot (N = 80) is still on the row-split kernel
    ctx2 = rnd(256, 80, 2048, scale=0.2)
    out.append(("softdot B256 N80", (rnd(256, 2048, scale=0.05), rnd(256, 2048, scale=0.05)),
                lambda q: torch.cat([t for t in ops.softdot_fwd(q, ctx2, None)], 1)))
    feat2 = rnd(256, 36, 2176, scale=0.2)
    out.append(("shift B256", (rnd(256, 2176, scale=0.05), rnd(256, 2176, scale=0.05)),
                lambda q: ops.shift_attn_fwd(q, feat2, rnd(256, 5) * 0 + 0.1)[0]))
    # LXRT / language attention core (mha_fwd: LDS-staged K / V, MFMA), B = 20 x 12 heads, L = 80
    qkv = rnd(20, 80, 3 * 768)
    out.append(("mha B20 L80", (rnd(20, 80, 768), rnd(20, 80, 768)),
                lambda q: ops.mha(q, qkv[..., 768:1536], qkv[..., 1536:], None, 12, 0.125)))
    # the native fp32 MFMA GEMM as a victim (LXRT short-K projection shape)
    Wn2 = rnd(768, 768, scale=0.02)
    out.append(("gemm_f32 1600x768x768", (rnd(1600, 768), rnd(1600, 768)),
                lambda x: _native(x, Wn2)))
    # per-row kernels of the step (wave reductions only)
    gam, bet = rnd(768, scale=0.1) + 1, rnd(768, scale=0.1)
    out.append(("layernorm 1600x768", (rnd(1600, 768), rnd(1600, 768)),
                lambda x: ops.layernorm(x, gam, bet, 1e-12)))
    cprev = rnd(20, 1024)
    out.append(("lstm_cell B20", (rnd(20, 4096), rnd(20, 4096)), lambda gt: ops.lstm_cell_fwd(gt, cprev)[0]))
    sty = rnd(1040, 2048)
    out.append(("adain_musigma 1040x2048", (rnd(1040, 2048), rnd(1040, 2048)), lambda c: ops.adain_musigma(c, sty)))
    feat, z = rnd(20, 36, 2176, scale=0.2), rnd(20, 5)
    out.append(("shift B20", (rnd(20, 2176, scale=0.05), rnd(20, 2176, scale=0.05)),
                lambda q: ops.shift_attn_fwd(q, feat, z)[0]))
    cand = rnd(20, 16, 2176, scale=0.2)
    out.append(("cand B20", (rnd(20, 2176, scale=0.05), rnd(20, 2176, scale=0.05)),
                lambda q: ops.softdot_fwd(q, cand, None, want_probs=False, want_wctx=False)[0]))
    # persistent bi-LSTM at B = 20, L = 80, H = 1024
    H = 1024
    whf, whb = rnd(4 * H, H, scale=0.02), rnd(4 * H, H, scale=0.02)
    lens = torch.full((20,), 80, dtype=torch.int32, device=dev)
    lens[5] = 37
    out.append(("bilstm B20", (rnd(20, 80, 2, 4 * H, scale=0.5), rnd(20, 80, 2, 4 * H, scale=0.5)),
                lambda x: ops.bilstm_fwd(x, whf, whb, lens, H)[0]))
    # teacher rollout's B = 160 forward (five 32-row tiles per workgroup)
    lens160 = torch.full((160,), 12, dtype=torch.int32, device=dev)
    lens160[100:] = 7
    out.append(("bilstm B160", (rnd(160, 12, 2, 4 * H, scale=0.5), rnd(160, 12, 2, 4 * H, scale=0.5)),
                lambda x: ops.bilstm_fwd(x, whf, whb, lens160, H)[0]))
    # persistent BPTT: B = 2 (finetune, one-row tile) and B = 20 (two tiles), gradients of saved forwards
    for Bb in (2, 20):
        lb = torch.full((Bb,), 80, dtype=torch.int32, device=dev)
        lb[-1] = 41
        _, _, _, sv = ops.bilstm_fwd(rnd(Bb, 80, 2, 4 * H, scale=0.5), whf, whb, lb, H, save=True)
        out.append((f"bilstm_bptt B{Bb}", (rnd(Bb, 80, 2 * H), rnd(Bb, 80, 2 * H)),
                    lambda g_, sv=sv, lb=lb: ops.bilstm_bwd(whf, whb, lb, sv, g_, None, None, H)))
    return out


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    only = sys.argv[2] if len(sys.argv) > 2 else None          # substring of the case names to run
    bgk = sys.argv[3] if len(sys.argv) > 3 else "x6"   # side-stream load: x6 | f32 | ew | nobg
    phase = int(sys.argv[4]) if len(sys.argv) > 4 else 0   # the side GEMM is launched before calls i % period == phase
    period = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    use_bg = bgk != "nobg"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bg = torch.cuda.Stream()
    Abg, Wbg = torch.randn(12800, 768, device=dev), torch.randn(3072, 768, device=dev) * 0.02
    ybg = torch.empty(12800, 3072, device=dev)
    ybg0 = ops.linear(Abg, Wbg).clone() if bgk == "x6" else None      # the side GEMM's own reference
    bgbad = torch.zeros(1, dtype=torch.int32, device=dev)
    for name, xs, fn in cases(dev, g):
        if only and only not in name:
            continue
        refs = [fn(x).clone() for x in xs]
        torch.cuda.synchronize()
        bad = torch.zeros(2, dtype=torch.int32, device=dev)
        shown = 0
        for i in range(iters):
            if use_bg and i % period == phase and not name.startswith("bilstm"):   # (the persistent kernel needs the whole chip)
                bg.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(bg):
                    if bgk == "x6":
                        ops.linear(Abg, Wbg, out=ybg)
                        bgbad += (~torch.eq(ybg, ybg0)).any().int()
                    elif bgk == "f32":      # native fp32 MFMA GEMM
                        ops.gemm(Abg, Wbg, ybg, M=12800, N=3072, K=768, lda=768, ldb=768, ldc=3072)
                    else:                   # pure HBM streaming
                        ybg.mul_(1.0)
            j = i & 1
            y = fn(xs[j])
            diff = ~torch.eq(y, refs[j]) & ~(torch.isnan(y) & torch.isnan(refs[j]))
            bad[j] += diff.any().int()
            if only and diff.any().item() and shown < 3:    # where a mismatch sits (diagnosis runs only)
                shown += 1
                pos = torch.nonzero(diff)[:8].tolist()
                print(f"  call {i} input {j}: {int(diff.sum())} elements differ, first at {pos}; "
                      f"got {[y[tuple(q)].item() for q in pos[:3]]} want {[refs[j][tuple(q)].item() for q in pos[:3]]}",
                      flush=True)
        torch.cuda.current_stream().wait_stream(bg)
        torch.cuda.synchronize()
        again = [fn(x) for x in xs]
        torch.cuda.synchronize()
        if not all(torch.equal(a, r) for a, r in zip(again, refs)):
            print(f"  {name}: a quiet re-run after the loop differs from the first results (inputs changed?)")
        b = bad.tolist()
        print(f"{name:32s} mismatching calls: input0 {b[0]}/{iters // 2 + iters % 2}  input1 {b[1]}/{iters // 2}",
              flush=True)
    if ybg0 is not None:
        print(f"side-stream x6 GEMM calls that differ from its quiet result: {int(bgbad.item())}")
    ops.check_device_errors()


if __name__ == "__main__":
    main()
