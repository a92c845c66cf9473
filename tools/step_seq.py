"""Kernel sequence of the last timed iteration of a rocprofv3 --kernel-trace CSV (one bench run), cut at the
decision-step boundaries: prints per kernel family its launches and device time per iteration, and the
kernel list (stream, start offset, duration, gap to the previous kernel of the same stream) of a window
of the iteration, so the small launches around the GEMMs can be attributed.
    python tools/step_seq.py <kernel_trace.csv> [iter_ms] [window_start_ms] [window_ms]"""
import sys
from collections import defaultdict

from timeline import load, short


def main(path, iter_ms=340.0, w0=None, wlen=3.0):
    rows = load(path)
    t1 = max(r[1] for r in rows)
    it = [r for r in rows if r[0] >= t1 - iter_ms * 1e6]
    t0 = it[0][0]
    fam = defaultdict(lambda: [0, 0.0])
    for s, e, n, st in it:
        f = fam[short(n)]
        f[0] += 1
        f[1] += (e - s) / 1e3
    print(f"last {iter_ms} ms: {len(it)} kernels")
    print(f"{'kernel':62s} {'launches':>8s} {'us total':>10s} {'us avg':>8s}")
    for k, (c, us) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:60]:
        print(f"{k:62s} {c:8d} {us:10.1f} {us / c:8.2f}")
    if w0 is None:
        w0 = iter_ms * 0.7
    ws, we = t0 + w0 * 1e6, t0 + (w0 + wlen) * 1e6
    print(f"\nwindow {w0:.2f} .. {w0 + wlen:.2f} ms of the iteration")
    last_end = {}
    for s, e, n, st in it:
        if s < ws or s > we:
            last_end[st] = e
            continue
        gap = (s - last_end[st]) / 1e3 if st in last_end else 0.0
        last_end[st] = e
        print(f"  s{st:<3d} {(s - t0) / 1e6:9.4f} ms  {(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us  {short(n)}")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(float(x) for x in a[1:]))
