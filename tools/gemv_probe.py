"""Drive tools/gemv_probe.hip (r06): the M <= 32 fp32 GEMV forms against the library's plan
(ops.linear -> gemm_skinny_nt_kernel) at the decision step's nn.Linear shapes, graph-replayed back to back
(dasa_amd.kbench._time_graph), weights hot (one copy) and cold (rotating over > 512 MB of copies).
    python tools/gemv_probe.py build     # hipcc -> tools/libgemv_probe.so (CPU host)
    python tools/gemv_probe.py           # on the GPU"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "gemv_probe.hip")
LIB = os.path.join(HERE, "libgemv_probe.so")
SHAPES = [(20, 2176, 1024), (20, 1024, 2048), (20, 4096, 1024), (20, 4096, 2240), (20, 1024, 3072), (2, 2176, 1024)]


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", "-fno-slp-vectorize",
                    SRC, "-o", LIB], check=True)
    print("built", LIB)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return build()
    import torch
    sys.path.insert(0, os.path.dirname(HERE))
    from dasa_amd import ops
    from dasa_amd.kbench import _time_graph
    lib = ctypes.CDLL(LIB)
    lib.gemv_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 5 + [
        ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    forms = [(m, w, s) for m in (2, 4) for w in (8, 16) for s in (2, 4)] + [
        (m, 4, s) for m in (51, 52, 54) for s in (1, 2, 4, 8)]
    lib.gemv_set_ws.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    slab = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16384, dtype=torch.int32, device=dev)
    lib.gemv_set_ws(slab.data_ptr(), cnt.data_ptr())
    for M, N, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, K, device=dev, generator=g)
        ncopy = max(2, int(512e6 // (4 * N * K)) + 1)
        Ws = [torch.randn(N, K, device=dev, generator=g) * 0.05 for _ in range(ncopy)]
        y = torch.empty(M, N, device=dev)
        yf = torch.empty(N // 16 + 1, 1024, device=dev)
        y3 = torch.empty(N // 16 + 1, 1024, device=dev)
        ref = (x.double() @ Ws[0].double().t())
        mb = 4.0 * (N * K + M * K + M * N) / 1e6
        res = []
        it = iter(range(1 << 30))
        ops.linear(x, Ws[0], out=y)
        err = float((y.double() - ref).abs().max())
        hot = _time_graph(lambda: ops.linear(x, Ws[0], out=y))
        cold = _time_graph(lambda: ops.linear(x, Ws[next(it) % ncopy], out=y))
        res.append(("plan", hot, cold, err))
        for mode, w, s in forms:
            if mode < 50 and (w * s * 32 < K or w * s * 32 >= 2 * K + 32 * w or (mode == 2 and not 16 < M <= 20)):
                continue
            yo = y3 if mode == 3 else y

            def call(W, mode=mode, w=w, s=s, out=None):
                rc = lib.gemv_launch(mode, x.data_ptr(), W.data_ptr(), (out if out is not None else yo).data_ptr(), M, N,
                                     K, w, s, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert rc == 0, (rc, mode, w, s)
            call(Ws[0])
            torch.cuda.synchronize()
            err = float((y.double() - ref).abs().max()) if mode in (1, 2) else 0.0
            hot = _time_graph(lambda: call(Ws[0]))
            it = iter(range(1 << 30))
            cold = _time_graph(lambda: call(Ws[next(it) % ncopy]))
            fl = _time_graph(lambda: lib.gemv_launch(0, 0, Ws[0].data_ptr(), yf.data_ptr(), M, N, K, w, s,
                                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))) \
                if mode < 50 else 0.0
            res.append((f"m{mode}w{w}s{s}", hot, cold, err, fl))
        print(f"== {M}x{N}x{K}  {mb:.1f} MB", flush=True)
        for r in res:
            fl = f" floor {r[4]:6.2f}" if len(r) > 4 else ""
            print(f"  {r[0]:>10}  hot {r[1]:6.2f} us {mb / r[1]:6.2f} TB/s  cold {r[2]:6.2f} us "
                  f"{mb / r[2]:6.2f} TB/s  err {r[3]:.1e}{fl}", flush=True)


if __name__ == "__main__":
    main()
