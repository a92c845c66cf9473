"""Which packed-FP32 torch kernels run CONCURRENTLY with an MFMA GEMM of another stream?

The r06 reproducer (tools/pk_fp32_repro.py, profiles/r06/pk_repro/) shows v_pk_fma_f32 results wrong on lanes
48-63 while bf16x6 GEMM workgroups start on the same CU; kernels of ONE stream never overlap, so a packed-FP32
kernel is exposed only if a GEMM of another stream runs during it. From a rocprofv3 kernel trace this lists, per
kernel name in the list of packed torch kernels (profiles/r06/pk_repro/torch_timed_path_kernels.txt, "PACKED"), its
dispatches and how many of them overlap in time a gemm / bilstm / mha dispatch of another stream.
    python tools/pk_overlap.py <run_kernel_trace.csv[.gz]> [packed list]"""
import csv
import gzip
import os
import sys
from bisect import bisect_left

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    path = sys.argv[1]
    lst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(HERE), "profiles/r06/pk_repro/torch_timed_path_kernels.txt")
    packed = [l.split("ms  ", 1)[1].strip() for l in open(lst) if l.startswith("PACKED")]
    op = gzip.open if path.endswith(".gz") else open
    rows = list(csv.DictReader(op(path, "rt")))
    mf = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows
          if any(k in r["Kernel_Name"] for k in ("gemm", "bilstm", "mha_"))]
    mf.sort()
    starts = [m[0] for m in mf]
    maxlen = max((e - s for s, e, _ in mf), default=0)
    res = {}
    for r in rows:
        n = r["Kernel_Name"]
        key = next((p for p in packed if n.startswith(p[:150])), None)
        if key is None:
            continue
        s, e, st = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]
        i0 = bisect_left(starts, s - maxlen)
        ov = any(ms < e and me > s and mst != st for ms, me, mst in mf[i0:bisect_left(starts, e)])
        c = res.setdefault(key, [0, 0])
        c[0] += 1
        c[1] += ov
    print("dispatches  overlapping another stream's GEMM / bi-LSTM / MHA  kernel")
    for k, (n, o) in sorted(res.items(), key=lambda x: -x[1][0]):
        print(f"{n:8d}  {o:8d}  {k[:160]}")


if __name__ == "__main__":
    main()
