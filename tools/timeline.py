"""GPU busy/idle analysis of a rocprofv3 --kernel-trace CSV (one bench run): splits the run at the
long host-side gaps, then reports per window the wall span, the union of kernel intervals (busy),
idle gaps by size, and the top kernels by time."""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r.get("Stream_Id") or 0)))
    rows.sort()
    return rows


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("at::native::", "")
    return n.split("(")[0][:60]


def union_busy(rows):
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _, _ in rows:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy, gaps


def main(path, t_last_ms=None):
    rows = load(path)
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    print(f"kernels {len(rows)}  span {(t1 - t0) / 1e6:.1f} ms")
    # the last iteration = the window after the last gap > 20 ms before the end, roughly; report the
    # whole trace's last `t_last_ms` ms if given
    if t_last_ms:
        rows = [r for r in rows if r[0] >= t1 - t_last_ms * 1e6]
    busy, gaps = union_busy(rows)
    span = max(r[1] for r in rows) - rows[0][0]
    print(f"window span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {(span - busy) / 1e6:.1f} ms")
    hist = defaultdict(lambda: [0, 0])
    for g in gaps:
        k = "<2us" if g < 2e3 else "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist[k][0] += 1
        hist[k][1] += g
    for k in ("<2us", "<10us", "<100us", "<1ms", ">=1ms"):
        print(f"  gaps {k:>7}: {hist[k][0]:6d}  total {hist[k][1] / 1e6:8.2f} ms")
    big = sorted(gaps, reverse=True)[:15]
    print("  largest gaps (ms):", " ".join(f"{g / 1e6:.2f}" for g in big))
    # per stream: kernels, union of its kernel intervals; and how much of the window 0 / 1 / 2+ streams
    # were running a kernel at once (the overlap the language pipe gets beside the rollout)
    by_stream = defaultdict(list)
    for r in rows:
        by_stream[r[3]].append(r)
    for sid, rs in sorted(by_stream.items(), key=lambda kv: -len(kv[1])):
        b, _ = union_busy(sorted(rs))
        tops = defaultdict(int)
        for s_, e_, n_, _ in rs:
            tops[short(n_).split("<")[0][-40:]] += e_ - s_
        top = ", ".join(f"{k} {v / 1e6:.1f}" for k, v in sorted(tops.items(), key=lambda kv: -kv[1])[:3])
        print(f"  stream {sid:>4}: {len(rs):6d} kernels  busy {b / 1e6:8.2f} ms  ({top})")
    ev = []
    for s_, e_, _, sid in rows:
        ev.append((s_, 1, sid))
        ev.append((e_, -1, sid))
    ev.sort()
    active = defaultdict(int)
    level = defaultdict(float)
    prev = ev[0][0]
    for t, d, sid in ev:
        n_act = sum(1 for v in active.values() if v > 0)
        level[min(n_act, 2)] += t - prev
        prev = t
        active[sid] += d
    print("  streams running at once: " + "  ".join(f"{k if k < 2 else '2+'}: {v / 1e6:.1f} ms"
                                                     for k, v in sorted(level.items())))
    # where the idle time sits: gaps >= 5 us by the kernel that ENDS the gap (the host was late to launch
    # it), and the window in 20 slices (busy fraction per slice: rollout / backward / optimizer phases)
    after = defaultdict(lambda: [0, 0])
    cur_e = None
    prev_name = None
    for s_, e_, n_, _ in rows:
        if cur_e is not None and s_ - cur_e >= 5e3:
            k = f"{short(prev_name)[:28]} -> {short(n_)[:28]}"
            after[k][0] += 1
            after[k][1] += s_ - cur_e
        if cur_e is None or e_ > cur_e:
            cur_e, prev_name = e_, n_
    print("  idle gaps >= 5 us by (last kernel -> next kernel):")
    for k, (c, t) in sorted(after.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"    {k:<60} {c:6d} {t / 1e6:8.2f} ms")
    w0, w1 = rows[0][0], max(r[1] for r in rows)
    nsl = 20
    sl = (w1 - w0) / nsl
    line = []
    for i in range(nsl):
        a, b = w0 + i * sl, w0 + (i + 1) * sl
        clip = sorted((max(s_, a), min(e_, b), n_, sid) for s_, e_, n_, sid in rows if e_ > a and s_ < b)
        bb, _ = union_busy(clip) if clip else (0, [])
        line.append(f"{100 * bb / sl:3.0f}")
    print(f"  busy % per {sl / 1e6:.1f} ms slice: " + " ".join(line))
    per = defaultdict(lambda: [0, 0])
    for s, e, n, _ in rows:
        k = short(n)
        per[k][0] += 1
        per[k][1] += e - s
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {k:<70} {c:6d} {t / 1e6:9.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
