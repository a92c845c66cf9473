"""Where does the row-split SoftDot forward (attn_fwd_kernel, attention mode 1) go wrong beside a
starting bf16x6 form-20 GEMM? (profiles/r04/attn_rowsplit_concurrency.txt)

The stress of tools/determinism_stress.py ("softdot B20", side x6 GEMM launched before calls
i % 4 == 0), with every call's workgroups dumping their intermediate values through
dasa_attn_debug_buffer: each thread's 16 row partials v[r] = x_r . q (after its global loads), a
checksum of its q float4, every wave's reduce-scattered partial as written to LDS red[w][r], the row
dot wave 0 summed from LDS, and the workgroup's HW_ID / XCC_ID. A bad call is compared stage by stage
with the quiet call on the same input:
  loads    some thread's v (or q checksum) differs: the data the loads returned;
  shuffle  every v equal, a wave partial differs: the ds_bpermute reduce-scatter;
  lds      every wave partial equal, the row dot differs: the LDS write / barrier / read;
  merge    the row dot equal, an output differs: the cross-workgroup merge.
    python tools/rowsplit_diag.py [iters] [period] [side: x6|nobg] [mode: 1 = row-split (r05 loads) | 3 = the
    r04 per-row-address loads]"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import ops  # noqa: E402

HDR, MAXT, MAXW = 4, 1024, 16


def hw_fields(u):
    """gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] tg[19:16] vm[23:20] queue[26:24]."""
    return {"wave": u & 15, "simd": (u >> 4) & 3, "cu": (u >> 8) & 15, "sh": (u >> 12) & 1, "se": (u >> 13) & 7,
            "tg": (u >> 16) & 15, "queue": (u >> 24) & 7}


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    period = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    side = sys.argv[3] if len(sys.argv) > 3 else "x6"
    mode = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, N, D = 20, 80, 2048
    ctx = torch.randn(B, N, D, device=dev, generator=g) * 0.2
    mask = torch.zeros(B, N, dtype=torch.bool, device=dev)
    mask[3, 50:] = True
    qs = [torch.randn(B, D, device=dev, generator=g) * 0.05 for _ in range(2)]
    Abg, Wbg = torch.randn(12800, 768, device=dev), torch.randn(3072, 768, device=dev) * 0.02
    ybg = torch.empty(12800, 3072, device=dev)
    bg = torch.cuda.Stream()
    ops.attn_set_mode(mode)                    # row-split kernel only (3: with the r04 loads)
    rec = ops.attn_debug_buffer(None)
    nblk = (N + 15) // 16
    T = D // 4
    per_call = B * nblk * rec

    def call(q, buf):
        ops.attn_debug_buffer(buf)
        out = torch.cat([t for t in ops.softdot_fwd(q, ctx, mask)], 1)
        ops.attn_debug_buffer(None)
        return out

    ref_out, ref_dump = [], []
    for q in qs:
        buf = torch.zeros(per_call, device=dev)
        ref_out.append(call(q, buf).clone())
        ref_dump.append(buf)
    torch.cuda.synchronize()
    dumps = [torch.zeros(per_call, device=dev) for _ in range(iters)]
    outs = []
    for i in range(iters):
        if side == "x6" and i % period == 0:
            bg.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(bg):
                ops.linear(Abg, Wbg, out=ybg)
        outs.append(call(qs[i & 1], dumps[i]))
    torch.cuda.current_stream().wait_stream(bg)
    torch.cuda.synchronize()
    ops.attn_set_mode(0)

    stages = collections.Counter()
    lanes, rowsc, match = collections.Counter(), collections.Counter(), collections.Counter()
    bad_calls = 0
    bad_hw, all_hw = collections.Counter(), collections.Counter()
    shown = 0
    for i in range(iters):
        j = i & 1
        d = dumps[i].view(B * nblk, rec).cpu()
        r0 = ref_dump[j].view(B * nblk, rec).cpu()
        for wg in range(B * nblk):
            u = int(d[wg, 0].view(torch.int32).item()) & 0xFFFFFFFF
            f = hw_fields(u)
            all_hw[(int(d[wg, 1].view(torch.int32).item()), f["se"], f["cu"])] += 1
        diff = ~torch.eq(outs[i], ref_out[j]) & ~(torch.isnan(outs[i]) & torch.isnan(ref_out[j]))
        if not diff.any():
            continue
        bad_calls += 1
        # the first N columns are the scores; their (b, n) rows name the workgroups to inspect
        sc = diff[:, :N]
        rows = torch.nonzero(sc).tolist() if sc.any() else []
        wgs = sorted({(b, n // 16) for b, n in rows}) or [(b, jj) for b in torch.nonzero(diff.any(1)).flatten().tolist()
                                                          for jj in range(nblk)]
        for b, jj in wgs:
            wg = b * nblk + jj
            dv, rv = d[wg], r0[wg]
            v = dv[HDR:HDR + MAXT * 16].view(MAXT, 16)[:T]
            vr = rv[HDR:HDR + MAXT * 16].view(MAXT, 16)[:T]
            qsum, qref = dv[HDR + MAXT * 16:HDR + MAXT * 17][:T], rv[HDR + MAXT * 16:HDR + MAXT * 17][:T]
            red = dv[HDR + MAXT * 17:HDR + MAXT * 17 + MAXW * 16].view(MAXW, 16)[:T // 64]
            redr = rv[HDR + MAXT * 17:HDR + MAXT * 17 + MAXW * 16].view(MAXW, 16)[:T // 64]
            tot, totr = dv[-16:], rv[-16:]
            vbad = torch.nonzero(~torch.eq(v, vr)).tolist()
            for t, r in vbad:
                lanes[t % 64] += 1
                rowsc[r] += 1
                # whose data did the load return? the quiet partial of another row of this thread, or of
                # the same row of another thread (+-16 / 32 / 48 lanes), or nothing seen in the quiet call
                got = v[t, r].item()
                who = "none"
                for r2 in range(16):
                    if r2 != r and vr[t, r2].item() == got:
                        who = f"row{r2 - r:+d}"
                        break
                else:
                    for dt in (-48, -32, -16, 16, 32, 48, -64, 64):
                        if 0 <= t + dt < T and vr[t + dt, r].item() == got:
                            who = f"lane{dt:+d}"
                            break
                match[who] += 1
            qbad = torch.nonzero(~torch.eq(qsum, qref)).flatten().tolist()
            rbad = torch.nonzero(~torch.eq(red, redr)).tolist()
            tbad = torch.nonzero(~torch.eq(tot, totr)).flatten().tolist()
            if vbad or qbad:
                st = "loads"
            elif rbad:
                st = "shuffle"
            elif tbad:
                st = "lds"
            else:
                st = "merge"
            stages[st] += 1
            u = int(dv[0].view(torch.int32).item()) & 0xFFFFFFFF
            f = hw_fields(u)
            bad_hw[(int(dv[1].view(torch.int32).item()), f["se"], f["cu"])] += 1
            if shown < 12:
                shown += 1
                # the shuffle tree of the dumped v: does it sum to the dumped red? (float64 reference sum)
                wsum = v.double().view(T // 64, 64, 16).sum(1)
                line = (f"call {i} in{j} wg (b={b}, j={jj}) stage={st} xcc={int(dv[1].view(torch.int32).item())} "
                        f"hw={f} v-diff {len(vbad)} {vbad[:4]} q-diff {qbad[:4]} red-diff {rbad[:6]} tot-diff {tbad}")
                print(line, flush=True)
                for w, r in rbad[:4]:
                    print(f"    red[{w}][{r}] got {red[w, r].item():.7g} quiet {redr[w, r].item():.7g} "
                          f"sum(dumped v) {wsum[w, r].item():.7g}", flush=True)
                for t, r in vbad[:4]:
                    print(f"    v[t={t}][{r}] got {v[t, r].item():.7g} quiet {vr[t, r].item():.7g}", flush=True)
                for r in tbad[:4]:
                    print(f"    tot[{r}] got {tot[r].item():.7g} quiet {totr[r].item():.7g} "
                          f"sum(dumped red) {red[:, r].double().sum().item():.7g}", flush=True)
    print(f"mode={mode} side={side} period={period}: bad calls {bad_calls}/{iters}; bad workgroups by stage {dict(stages)}")
    print(f"bad workgroups by (xcc, se, cu): {dict(bad_hw.most_common(12))}")
    print(f"bad partials by lane within the wave: {dict(sorted(lanes.items()))}")
    print(f"bad partials by row of the block: {dict(sorted(rowsc.items()))}")
    print(f"a bad partial equals the quiet partial of: {dict(match.most_common(10))}")
    print(f"distinct (xcc, se, cu) over all workgroups: {len(all_hw)}")


if __name__ == "__main__":
    main()
