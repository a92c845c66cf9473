"""Run the packed-FP32 reproducer (tools/pk_fp32_repro.hip) beside a bf16x6 form-20 GEMM,
launched exactly as tools/rowsplit_diag.py launched the row-split SoftDot: the side GEMM (12800 x 3072 x 768,
form 20) on another stream before every `period`-th call, `iters` calls alternating nothing else.

Per call it counts (device side) the (thread, row) results whose packed chain differs from the scalar chain,
per lane, and (here) the calls whose packed or scalar results differ from the quiet run's bits.
    python tools/pk_fp32_repro.py build                 # hipcc -> tools/libpk_fp32_repro.so (on the CPU host)
    python tools/pk_fp32_repro.py [iters] [period] [side: x6|nobg] [mode: 0 = asm packed chains | 1 = the
                                  compiler-packed dot4 of the row-split kernel, its load form]"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "pk_fp32_repro.hip")
LIB = os.path.join(HERE, "libpk_fp32_repro.so")


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", SRC, "-o", LIB],
                   check=True)
    print("built", LIB)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return build()
    import torch
    sys.path.insert(0, os.path.dirname(HERE))
    from dasa_amd import ops
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    period = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    side = sys.argv[3] if len(sys.argv) > 3 else "x6"
    mode = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    lib = ctypes.CDLL(LIB)
    lib.pk_rows_launch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, N, D = 20, 80, 2048
    T, nblk = D // 4, (N + 15) // 16
    x = torch.randn(B, N, D, device=dev, generator=g) * 0.2
    q = torch.randn(B, D, device=dev, generator=g) * 0.05
    Abg, Wbg = torch.randn(12800, 768, device=dev), torch.randn(3072, 768, device=dev) * 0.02
    ybg = torch.empty(12800, 3072, device=dev)
    bg = torch.cuda.Stream()

    def call(pk, sc, bad):
        rc = lib.pk_rows_launch(x.data_ptr(), q.data_ptr(), pk.data_ptr(), sc.data_ptr(), bad.data_ptr(), B, N, D, mode,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc

    n = B * nblk * 16 * T
    ref_pk, ref_sc = torch.empty(n, device=dev), torch.empty(n, device=dev)
    bad0 = torch.zeros(65, dtype=torch.int32, device=dev)
    call(ref_pk, ref_sc, bad0)
    torch.cuda.synchronize()
    assert int(bad0[0]) == 0 and torch.equal(ref_pk, ref_sc), "packed != scalar on a quiet chip"
    bad = torch.zeros(65, dtype=torch.int32, device=dev)
    calls_pk = torch.zeros((), dtype=torch.int32, device=dev)
    calls_sc = torch.zeros((), dtype=torch.int32, device=dev)
    elems_pk = torch.zeros((), dtype=torch.int64, device=dev)
    rows_pk = torch.zeros(16, dtype=torch.int64, device=dev)
    pk, sc = torch.empty(n, device=dev), torch.empty(n, device=dev)
    for i in range(iters):
        if side == "x6" and i % period == 0:
            bg.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(bg):
                ops.linear(Abg, Wbg, out=ybg)
        call(pk, sc, bad)
        dpk = pk != ref_pk
        calls_pk += dpk.any().int()
        calls_sc += (sc != ref_sc).any().int()
        elems_pk += dpk.sum()
        rows_pk += dpk.view(B * nblk, 16, T).sum((0, 2))
    torch.cuda.current_stream().wait_stream(bg)
    torch.cuda.synchronize()
    lanes = {i: int(v) for i, v in enumerate(bad[1:].tolist()) if v}
    print(f"side={side} period={period} iters={iters} mode={mode}")
    print(f"calls with a packed result != quiet bits: {int(calls_pk)}/{iters}  (elements {int(elems_pk)})")
    print(f"calls with a scalar result != quiet bits: {int(calls_sc)}/{iters}")
    print(f"(thread, row) packed != scalar in-kernel: {int(bad[0])}; by lane: {lanes}")
    print(f"packed mismatches by row (0..15): {rows_pk.tolist()}")


if __name__ == "__main__":
    main()
