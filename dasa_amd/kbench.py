"""Isolated timing of the HBM-bound policy kernels (the depth-guided AdaIN gate, the 36-view shift
attention, the instruction / candidate SoftDot attention, the mu/sigma AdaIN) at the shapes one
decision step uses: cfg2 (B=20, the benchmark workload) and cfg5 (B=256, BASELINE.json's HBM/MFMA
roofline stress config).

Each kernel is launched REPS times back to back inside one captured HIP graph and the replay is
bracketed by HIP events, so the per-launch time excludes host launch latency (inside the rollout the
same kernels sit between dependent kernels, where the host is ahead of the GPU). `bytes` is the
algorithmic (compulsory) traffic per launch: every input read once, every output written once. At B=20
a launch's working set (3-34 MB) stays resident in the 256 MB Infinity Cache across replays, so those
rates are cache-assisted; B=256 (80-330 MB per launch) streams from HBM. `step_chain` replays one decision
step's AdaIN gate + shift / instruction / candidate attention back to back; `launch_floor` is a kernel
with no work to speak of, the per-launch time no kernel gets under."""
import torch

from . import ops

HBM_PEAK_GBS = 8000.0
REPS = 50


def _time_graph(fn, reps=REPS):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    from .graph import _no_gc
    with _no_gc(), torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    del g
    return best * 1e3   # us per launch


def _cases(B, dev):
    g = torch.Generator(device=dev).manual_seed(B)
    D, F, V, C, L, H, K = 2176, 2048, 36, 16, 80, 1024, 5

    def rnd(*shape):
        return torch.rand(*shape, device=dev, generator=g)
    cases = []
    # shift attention over the AdaIN'd panorama [B, 36, 2176] (model.py:318-353)
    feat, q, z = rnd(B, V, D), rnd(B, D) * 0.05, rnd(B, K)
    wctx, attn, shifted, wsm = ops.shift_attn_fwd(q, feat, z)
    dw = rnd(B, D)
    cases.append(("shift_attn", 4.0 * B * (V * D + 2 * D + 3 * V), lambda: ops.shift_attn_fwd(q, feat, z)))
    cases.append(("shift_attn_bwd", 4.0 * B * (2 * V * D + 3 * D + 3 * V),
                  lambda: ops.shift_attn_bwd(q, feat, attn, shifted, wsm, dw)))
    # instruction attention over ctx [B, 80, 2048] with the padding mask (model.py:268-296)
    ctx, qi = rnd(B, L, 2 * H), rnd(B, 2 * H) * 0.05
    mask = torch.zeros(B, L, dtype=torch.bool, device=dev)
    _, probs, _ = ops.softdot_fwd(qi, ctx, mask)
    di = rnd(B, 2 * H)
    cases.append(("softdot", 4.0 * B * (L * 2 * H + 2 * 2 * H + 3 * L), lambda: ops.softdot_fwd(qi, ctx, mask)))
    cases.append(("softdot_bwd", 4.0 * B * (2 * L * 2 * H + 3 * 2 * H + 3 * L),
                  lambda: ops.softdot_bwd(qi, ctx, probs, dwctx=di)))
    # candidate logits over [B, 16, 2176] (scores only, output_prob=False)
    cand, qc = rnd(B, C, D), rnd(B, D) * 0.05
    cases.append(("cand_logit", 4.0 * B * (C * D + D + C),
                  lambda: ops.softdot_fwd(qc, cand, None, want_probs=False, want_wctx=False)))
    # DGAdaChannel gate epilogue: out = s * f (* noise) on the RGB columns of [B*(36+C), 2176] rows
    R = B * (V + C)
    s, f, out, noise = rnd(R, F), rnd(R, D), torch.empty(R, D, device=dev), rnd(F)
    cases.append(("ada_gate", 12.0 * R * F, lambda: ops.ada_gate_fwd(s, f[:, :F], noise, out[:, :F])))
    cases.append(("colscale", 8.0 * R * F, lambda: ops.colscale(f[:, :F], noise, out[:, :F])))
    dout = rnd(R, D)
    cases.append(("ada_gate_bwd", 16.0 * R * F, lambda: ops.ada_gate_bwd(dout[:, :F], s, f[:, :F], noise)))
    # mu/sigma AdaIN (adaIn_type default, model.py:1822-1840) on the same rows
    cases.append(("adain_musigma", 12.0 * R * F, lambda: ops.adain_musigma(f[:, :F], dout[:, :F], out=out[:, :F])))
    # the decision step's AdaIN + attention chain as it runs per step (gate, shift, instruction SoftDot,
    # candidate logits back to back): its bytes over its time
    chain = [c for c in cases if c[0] in ("ada_gate", "shift_attn", "softdot", "cand_logit")]
    cases.append(("step_chain", sum(c[1] for c in chain), lambda: [c[2]() for c in chain]))
    # the attention modules' weight-streaming projections at this batch (gemm_skinny_* kernels at
    # B <= 32): SoftDot / Shift linear_in (model.py:263, 311), the decoder LSTMCell input + recurrent
    # products (model.py:437), linear_out of the instruction attention (model.py:264), and the input
    # gradient of the LSTMCell input projection (dX = dY . W_ih). "_cold" rotates over enough weight
    # copies (> 512 MB) that every launch streams its weight from HBM, as inside the rollout where the
    # language stack's traffic evicts the Infinity Cache between decision steps.
    lin = {"linear_in_feat": (D, H), "linear_in_instr": (2 * H, H), "lstm_ih": (4 * H, 64 + D),
           "lstm_hh": (4 * H, H), "linear_out": (H, 3 * H)}
    for name, (N, Kd) in lin.items():
        x = rnd(B, Kd)
        y = torch.empty(B, N, device=dev)
        ncopy = max(2, int(512e6 // (4 * N * Kd)) + 1)
        Ws = [rnd(N, Kd) * 0.05 for _ in range(ncopy)]
        nb = 4.0 * (N * Kd + B * Kd + B * N)
        cases.append((f"skinny_{name}", nb, lambda x=x, W=Ws[0], y=y: ops.linear(x, W, out=y)))
        it = iter(range(1 << 30))
        cases.append((f"skinny_{name}_cold", nb,
                      lambda x=x, Ws=Ws, y=y, it=it: ops.linear(x, Ws[next(it) % len(Ws)], out=y)))
    dy, Wih = rnd(B, 4 * H), rnd(4 * H, 64 + D) * 0.05
    cases.append(("skinny_lstm_ih_dx", 4.0 * (4 * H * (64 + D) + B * 4 * H + B * (64 + D)),
                  lambda: ops.matmul_nn(dy, Wih)))
    # the attention modules end to end as one decision step runs them: linear_in + shift attention,
    # linear_in + instruction SoftDot + linear_out, linear_in + candidate logits (weights cache-warm)
    Wf, Wi, Wo, Wc = rnd(D, H) * 0.05, rnd(2 * H, H) * 0.05, rnd(H, 3 * H) * 0.05, rnd(D, H) * 0.05
    h1 = rnd(B, H)
    qf, qi2, qc2 = torch.empty(B, D, device=dev), torch.empty(B, 2 * H, device=dev), torch.empty(B, D, device=dev)
    cat = rnd(B, 3 * H)
    htl = torch.empty(B, H, device=dev)

    def attn_modules():
        ops.linear(h1, Wf, out=qf)
        ops.shift_attn_fwd(qf, feat, z)
        ops.linear(h1, Wi, out=qi2)
        ops.softdot_fwd(qi2, ctx, mask)
        ops.linear(cat, Wo, act="tanh", out=htl)
        ops.linear(h1, Wc, out=qc2)
        ops.softdot_fwd(qc2, cand, None, want_probs=False, want_wctx=False)
    nb_mod = (4.0 * (D * H + 2 * H * H + 3 * H * H + D * H) + 4.0 * B * (8 * H + 2 * D)
              + 4.0 * B * (V * D + 2 * D + 3 * V) + 4.0 * B * (L * 2 * H + 2 * 2 * H + 3 * L) + 4.0 * B * (C * D + D + C))
    cases.append(("attn_modules", nb_mod, attn_modules))
    # launch floor: a one-row column scale (8 KB) — the time any launch takes inside a replayed graph
    f1, o1 = rnd(1, F), torch.empty(1, F, device=dev)
    cases.append(("launch_floor", 8.0 * F, lambda: ops.colscale(f1, noise, o1)))
    return cases


def hbm_stream(rows=131072, cols=2048):
    """Peak check (confirm the datasheet 8 TB/s on the box): a 1 GiB -> 1 GiB column
    scale (ops.colscale, float4 streaming) timed back to back in a graph; returns GB/s of read + write."""
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.rand(rows, cols, device=dev)
    y = torch.empty_like(x)
    s = torch.rand(cols, device=dev)
    us = _time_graph(lambda: ops.colscale(x, s, y), reps=10)
    nbytes = 8.0 * rows * cols
    del x, y
    return {"us": round(us, 1), "bytes": int(nbytes), "GB/s": round(nbytes / (us * 1e-6) / 1e9, 1),
            "frac": round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}


def hbm_kernels(batches=(20, 256)):
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {"hbm_stream": hbm_stream()}
    for B in batches:
        for name, nbytes, fn in _cases(B, dev):
            us = _time_graph(fn)
            gbs = nbytes / (us * 1e-6) / 1e9
            res.setdefault(name, {})[f"B{B}"] = {"us": round(us, 2), "bytes": int(nbytes), "GB/s": round(gbs, 1),
                                                  "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # BASELINE.json north star: ">= 40 % achieved HBM bandwidth on the AdaIN + attention kernels" - their
    # bytes over their time, each kernel timed alone (byte-weighted aggregate of the five forward kernels)
    fam = ("ada_gate", "adain_musigma", "shift_attn", "softdot", "cand_logit")
    agg = {}
    for B in batches:
        k = f"B{B}"
        nb = sum(res[f][k]["bytes"] for f in fam)
        us = sum(res[f][k]["us"] for f in fam)
        gbs = nb / (us * 1e-6) / 1e9
        agg[k] = {"us": round(us, 2), "bytes": int(nb), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    res["adain_attention_aggregate"] = dict(agg, kernels=list(fam))
    return res


if __name__ == "__main__":
    import json
    import sys
    torch.cuda.set_device(0)
    bs = tuple(int(x) for x in sys.argv[1:]) or (20, 256)
    print(json.dumps(hbm_kernels(bs), indent=1))
