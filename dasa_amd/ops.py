"""Torch-facing wrappers over libdasa_hip.so.

Every function here takes/returns torch tensors on the ROCm device and enqueues HIP kernels from
libdasa_hip.so on torch's current stream (so torch.cuda.graph capture records them). There is no
CPU path: a CPU tensor is a usage error and raises.
"""
import ctypes
import os
import weakref

import torch

from . import _lib
from . import prof
from ._lib import ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_SIGMOID, GemmDesc  # noqa: F401


def check(rc, what, family=None, flops=0.0, nbytes=0.0, _ev=None):
    _lib.check(rc, what)


def _call(what, family, fn, *a, flops=0.0, nbytes=0.0, detail=None, kernels=1):
    """Launch through the C-ABI; under prof.collect() bracket it with HIP events on the stream."""
    if prof.active():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = fn(*a)
        e1.record()
        prof.record(family, e0, e1, flops, nbytes, detail, kernels)
    else:
        rc = fn(*a)
    _lib.check(rc, what)

_ACT_IDS = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "gelu": ACT_GELU, "tanh": ACT_TANH,
            "sigmoid": ACT_SIGMOID}


_raw_stream = torch._C._cuda_getCurrentRawStream


def _stream():
    """Raw hipStream_t of torch's current stream on the current device (the fast C accessor: the
    torch.cuda.current_stream() object path costs ~8 us per launch on the host)."""
    return _raw_stream(torch.cuda.current_device())


def _p(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.DasaError("dasa_amd kernels need device tensors (the HIP path has no CPU fallback)")
    return t.data_ptr()


def _f32(t, name):
    if t.dtype != torch.float32:
        raise _lib.DasaError(f"{name}: expected float32, got {t.dtype}")
    return t


def _rows(t):
    """(rows, ld) of a tensor viewed as a 2-D row-major matrix over its last dim (unit inner stride)."""
    if t.is_contiguous():
        n = t.shape[-1] if t.dim() else 1
        return (t.numel() // n if n else 0), n
    if t.stride(-1) != 1:
        raise _lib.DasaError("inner dimension must be contiguous")
    if t.dim() == 1:
        return 1, t.shape[0]
    # all leading dims must collapse with a uniform row stride
    ld = t.stride(-2)
    rows = 1
    exp = ld
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] != 1 and t.stride(d) != exp:
            raise _lib.DasaError("leading dims must collapse to a single row stride")
        exp = t.stride(d) * t.shape[d]
        rows *= t.shape[d]
    return rows, ld


# ------------------------------------------------------------------------------------------ GEMM
_WS = {}
_WS_OLD = []
_WS_SK = (64 << 10) + 2 * 512 * 128 * 128 * 4    # counters + stream-K slabs (<= 512 workgroups)
_WS_MIN = max(32 << 20, _WS_SK)


def _gemm_ws(device, d, need=0):
    """GEMM workspace (include/dasa_hip.h dasa_gemm_f32_workspace): one zero-initialised buffer per
    (device, stream), grown on demand and reused by every GEMM on that stream. Its leading stream-K
    arrival counters are left zero by every call (so it is zeroed only on allocation); split-K
    partials / stream-K slabs follow them, and calls on one stream never overlap. The buffer starts
    large enough for every stream-K plan, so most calls skip the workspace query."""
    key = (device.index, _stream())
    buf = _WS.get(key)
    if buf is None:
        buf = torch.zeros(_WS_MIN // 4, dtype=torch.float32, device=device)
        _WS[key] = buf
    nbytes = buf.numel() * 4
    if need or d.M * d.N * max(1, d.batch) * 16 * 4 + _WS_SK > nbytes:   # split-K is at most 16-way
        need = need or _lib.lib().dasa_gemm_f32_workspace(ctypes.byref(d))
        if need > nbytes:
            _WS_OLD.append(buf)      # kernels already queued / captured in a graph still point at it
            buf = torch.zeros(need // 4 + 1, dtype=torch.float32, device=device)
            _WS[key] = buf
            nbytes = buf.numel() * 4
    return buf.data_ptr(), nbytes


def gemm(A, B, C, *, M, N, K, opA=0, opB=1, lda, ldb, ldc, bias=None, act=None, aux=None, ld_aux=0,
         colscale=None, alpha=1.0, beta=0.0, batch=1, strideA=0, strideB=0, strideC=0, strideAux=0):
    """Raw descriptor call (see include/dasa_hip.h). A/B/C are tensors (base pointers used)."""
    d = GemmDesc()
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), int(batch)
    d.opA, d.opB = int(opA), int(opB)
    d.A, d.lda, d.strideA = _p(A), int(lda), int(strideA)
    d.B, d.ldb, d.strideB = _p(B), int(ldb), int(strideB)
    d.C, d.ldc, d.strideC = _p(C), int(ldc), int(strideC)
    d.bias = _p(bias)
    d.act = _ACT_IDS[act] if not isinstance(act, int) else act
    d.aux, d.ld_aux, d.strideAux = _p(aux), int(ld_aux), int(strideAux)
    d.colscale = _p(colscale)
    d.alpha, d.beta = float(alpha), float(beta)
    L = _lib.lib()
    ws, ws_bytes = _gemm_ws(C.device, d)
    b = max(1, int(batch))
    # M <= 64 (the per-step decoder / critic linears at B = 20) is weight streaming: its own family,
    # judged against HBM (bytes = weight + activations), not the MFMA roof
    fam = "gemm_skinny" if M <= 64 else "gemm"
    _call("dasa_gemm_f32", fam, L.dasa_gemm_f32, ctypes.byref(d), ws, ws_bytes, _stream(),
          flops=2.0 * M * N * K * b, nbytes=4.0 * b * (M * K + K * N + M * N),
          detail=(int(M), int(N), int(K), b, int(opA), int(opB)))


# bf16 matmul mode (BASELINE configs[4]: B = 256, bf16 weights/operands with fp32 accumulation).
# Forward-only: nn.Linear forwards whose K % 64 == 0 run dasa_gemm_bf16 on a bf16 copy of the weight
# (converted once per weight version), and the bi-LSTM's per-timestep recurrent product at B > 192 runs on
# bf16 W_hh / h with fp32 accumulation (dasa_bilstm_fwd_bf16); LayerNorm, softmax, attention cores, the
# cell updates and every elementwise op stay fp32.
_BF16 = {"on": False, "acts": os.environ.get("DASA_BF16_ACTS", "1") != "0",
         "attn": os.environ.get("DASA_BF16_ATTN", "1") != "0"}   # DASA_BF16_ATTN=0: fp32 attention core (A/B)


def bf16_attn_on():
    """Under bf16_matmul with bf16 activations: Q/K/V stored bf16 and the bf16 attention core."""
    return _BF16["on"] and _BF16["acts"] and _BF16["attn"]
_bf16_w = {}


class bf16_matmul:
    """Context manager: the policy's linear layers compute with bf16 operands (no autograd)."""

    def __enter__(self):
        if torch.is_grad_enabled():
            raise _lib.DasaError("bf16 matmul mode is forward-only: enter it under torch.no_grad()")
        self._prev = _BF16["on"]
        _BF16["on"] = True
        self._prev_lstm = _lib.lib().dasa_bilstm_fwd_bf16(1)
        return self

    def __exit__(self, *exc):
        _BF16["on"] = self._prev
        _lib.lib().dasa_bilstm_fwd_bf16(self._prev_lstm)
        if not self._prev:
            _bf16_w.clear()
        return False


def to_bf16(x, out=None):
    """Round an fp32 tensor to bf16 (RNE) on the device: dasa_f32_to_bf16."""
    _f32(x, "to_bf16.x")
    x = x.contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    _call("dasa_f32_to_bf16", "elementwise", _lib.lib().dasa_f32_to_bf16, _p(x), _p(out), x.numel(), _stream(),
          nbytes=6.0 * x.numel())
    return out


def _stream_safe(entry_ev, entry_stream, tensors):
    """A derived weight copy built on `entry_stream` and used from the current stream: the user waits
    for the build (event) and the allocator keeps the copy alive for the user's stream, as
    vilmodel._fused_weights does (the LXRT layer runs the shared visual_attention on two streams)."""
    if _stream() == entry_stream or torch.cuda.is_current_stream_capturing():
        return          # same stream, or built by the pre-capture warm-up the capture stream follows
    cur = torch.cuda.current_stream()
    cur.wait_event(entry_ev)
    for t in tensors:
        t.record_stream(cur)


def _built_here():
    """(event recorded after the build, the building stream's raw handle)."""
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    return ev, _stream()


def _bf16_weight(W):
    key = (W.data_ptr(), W._version, tuple(W.shape), W.stride(0))
    e = _bf16_w.get(key)
    if e is None:
        if len(_bf16_w) > 1024:
            _bf16_w.clear()
        t = to_bf16(W)
        _bf16_w[key] = (t,) + _built_here()
        return t
    _stream_safe(e[1], e[2], (e[0],))
    return e[0]


def gemm_bf16(x, Wb, out, *, M, N, K, lda, ldc, bias=None, act=None, aux=None, ld_aux=0, colscale=None,
              alpha=1.0, beta=0.0):
    """dasa_gemm_bf16_ex; x and out each fp32 or bf16 (a bf16 activation / bf16 output)."""
    d = GemmDesc()
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), 1
    d.opA, d.opB = 0, 1
    d.A, d.lda, d.strideA = _p(x), int(lda), 0
    d.B, d.ldb, d.strideB = _p(Wb), int(Wb.stride(0)), 0
    d.C, d.ldc, d.strideC = _p(out), int(ldc), 0
    d.bias = _p(bias)
    d.act = _ACT_IDS[act] if not isinstance(act, int) else act
    d.aux, d.ld_aux, d.strideAux = _p(aux), int(ld_aux), 0
    d.colscale = _p(colscale)
    d.alpha, d.beta = float(alpha), float(beta)
    flags = (1 if x.dtype == torch.bfloat16 else 0) | (2 if out.dtype == torch.bfloat16 else 0)
    _call("dasa_gemm_bf16_ex", "gemm_bf16", _lib.lib().dasa_gemm_bf16_ex, ctypes.byref(d), flags, _stream(),
          flops=2.0 * M * N * K, nbytes=x.element_size() * M * K + 2.0 * K * N + out.element_size() * M * N,
          detail=(int(M), int(N), int(K)))


# fp32 GEMM emulated on bf16 matrix cores (include/dasa_hip.h dasa_gemm_f32x6): the nn.Linear weight
# is split once per weight version into three bf16 planes (hi, mid, lo) and cached here; the input is
# split inside the kernel. fp32-accurate (the six kept bf16 products are exact, dropped terms are below
# fp32 rounding); DASA_GEMM_EMU=0 routes every nn.Linear back to the native fp32 MFMA kernels.
_X6 = {}
_EMU = {"on": os.environ.get("DASA_GEMM_EMU", "1") != "0", "min_rows": int(os.environ.get("DASA_GEMM_EMU_MIN_M", "512")),
        "short_k": int(os.environ.get("DASA_X6_SHORTK_TILES", "0"))}   # A/B: x6 split-K on few-tile short-K GEMMs


def set_gemm_emulation(on=None, min_rows=None):
    """Switch the bf16x6 fp32 path (returns the previous (on, min_rows))."""
    prev = (_EMU["on"], _EMU["min_rows"])
    if on is not None:
        _EMU["on"] = bool(on)
    if min_rows is not None:
        _EMU["min_rows"] = int(min_rows)
    return prev


def split3_bf16(W):
    """Three bf16 planes [3, N, K] with W = hi + mid + lo (dasa_f32_split3_bf16)."""
    _f32(W, "split3.W")
    N, K = W.shape
    planes = torch.empty(3, N, K, dtype=torch.bfloat16, device=W.device)
    _call("dasa_f32_split3_bf16", "elementwise", _lib.lib().dasa_f32_split3_bf16, _p(W), W.stride(0), _p(planes),
          N, K, _stream(), nbytes=10.0 * N * K)
    return planes


_FRESH_PLANES = [0]   # > 0 while a training region is captured (graph.AutogradGraphs): see _x6_weight


def _x6_weight(W):
    """The cached bf16 planes of W for this weight version (recomputed after in-place updates). Inside a
    captured TRAINING region the split is recorded into the graph instead (fresh planes on every replay):
    the region's weights change in place with every optimizer step, which a cached plane buffer baked
    into the graph would not see."""
    if _FRESH_PLANES[0]:
        return split3_bf16(W)
    wid = id(W)
    e = _X6.get(wid)
    if e is not None and e[0]() is W and e[1] == W._version and e[2] == W.data_ptr():
        _stream_safe(e[4], e[5], (e[3],))
        return e[3]
    planes = split3_bf16(W)

    def _drop(ref, wid=wid):
        ent = _X6.get(wid)
        if ent is not None and ent[0] is ref:
            del _X6[wid]
    _X6[wid] = (weakref.ref(W, _drop), W._version, W.data_ptr(), planes) + _built_here()
    return planes


def _x6_splitk(M, N, K):
    """Split count of the bf16x6 plan (gemm.hip x6_plan): 1 at >= 128 output tiles of 128x128, else the
    most splits keeping tiles x splits <= 256 with >= 8 32-deep K steps per split."""
    tiles = -(-M // 128) * -(-N // 128)
    return 1 if tiles >= 128 else max(1, min(256 // tiles, K // 256))


def _emu_ok(M, N, K, lda, x):
    """Plan rule (profiles/r02/gemm_x6_sweep_b.txt, gemm_x6_splitk.txt): the 128x128-tile bf16x6 kernel
    beats the native fp32 MFMA kernels (by 1.1-1.5x) once it fills the chip — >= 128 output tiles (the
    12800-row language stack, the 1600-row LSTM input projections and LXRT language branch, the 720 x 3072
    vision FFN), or, at K >= 2048, >= 192 workgroups with K split over the tiles (the 1600 / 720 x 768 x
    3072 FFN outputs, the 720 x 2048 x 2048 AdaIN gate). The short-K LXRT projections (36-108 tiles,
    K = 768) stay on the native fp32 kernels: split there, they win in isolation but lose in the
    iteration, where they share the chip with the concurrent language stream."""
    if not (_EMU["on"] and M >= _EMU["min_rows"] and K % 32 == 0 and N % 8 == 0 and lda % 4 == 0
            and x.data_ptr() % 16 == 0):
        return False
    tiles = -(-M // 128) * -(-N // 128)
    if _EMU["short_k"] and tiles >= _EMU["short_k"] and K >= 512:
        return True
    return tiles >= 128 or (K >= 2048 and tiles * _x6_splitk(M, N, K) >= 192)


_X6_WS_NEED = {}   # (M, N, K) -> split-K workspace bytes of the many-tile bf16x6 plan (a per-shape constant)


def gemm_f32x6(x, planes, out, *, M, N, K, lda, ldc, bias=None, act=None, aux=None, ld_aux=0, colscale=None,
               alpha=1.0, beta=0.0):
    d = GemmDesc()
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), 1
    d.opA, d.opB = 0, 1
    d.A, d.lda, d.strideA = _p(x), int(lda), 0
    d.B, d.ldb, d.strideB = _p(planes), int(K), 0
    d.C, d.ldc, d.strideC = _p(out), int(ldc), 0
    d.bias = _p(bias)
    d.act = _ACT_IDS[act] if not isinstance(act, int) else act
    d.aux, d.ld_aux, d.strideAux = _p(aux), int(ld_aux), 0
    d.colscale = _p(colscale)
    d.alpha, d.beta = float(alpha), float(beta)
    L = _lib.lib()
    ws, ws_bytes = 0, 0
    if -(-M // 128) * -(-N // 128) < 128:          # few tiles: the split-K form needs the workspace
        need = L.dasa_gemm_f32x6_workspace(ctypes.byref(d))
    else:                                          # many tiles: the plan may split to fill the last round
        need = _X6_WS_NEED.get((M, N, K))
        if need is None:
            need = _X6_WS_NEED[(M, N, K)] = L.dasa_gemm_f32x6_workspace(ctypes.byref(d))
    if need:
        ws, ws_bytes = _gemm_ws(out.device, d, need)
    kernels = 1
    if prof.active():      # the tail plan launches two kernels: per-kernel durations -> per-call rates
        kernels = int(L.dasa_gemm_f32x6_kernels(ctypes.byref(d), int(ws_bytes)))
    _call("dasa_gemm_f32x6", "gemm_x6", L.dasa_gemm_f32x6_ws, ctypes.byref(d), int(N) * int(K), ws, ws_bytes,
          _stream(), flops=2.0 * M * N * K, nbytes=4.0 * M * K + 6.0 * K * N + 4.0 * M * N,
          detail=(int(M), int(N), int(K)), kernels=kernels)


def bf16_acts_ok(x, N):
    """Under bf16_matmul: may this linear's output be handed on as a bf16 activation (the consumer is a
    bf16 GEMM)? DASA_BF16_ACTS=0 keeps every activation fp32 (A/B)."""
    K = x.shape[-1]
    return (_BF16["on"] and _BF16["acts"] and x.dtype in (torch.float32, torch.bfloat16) and K % 64 == 0
            and N % 64 == 0 and _rows(x)[1] % 8 == 0 and x.data_ptr() % 16 == 0)


def linear(x, W, b=None, act=None, out=None, aux=None, colscale=None, beta=0.0, alpha=1.0, out_dtype=None):
    """y = act(x @ W^T + b) [* aux] [* colscale] (+ beta*out). x [..., K] (row-strided ok), W [N, K].
    Under bf16_matmul, x may be a bf16 activation and out_dtype=torch.bfloat16 stores y as bf16."""
    bf_io = x.dtype == torch.bfloat16 or out_dtype == torch.bfloat16 or (out is not None and out.dtype == torch.bfloat16)
    if not bf_io:
        _f32(x, "linear.x")
    K = x.shape[-1]
    N = W.shape[0]
    assert W.shape[1] == K and W.stride(1) == 1, "W must be [N, K] with contiguous rows"
    M, lda = _rows(x)
    if out is None:
        out = torch.empty(*x.shape[:-1], N, dtype=out_dtype or torch.float32, device=x.device)
    Mo, ldc = _rows(out)
    assert Mo == M and out.shape[-1] == N
    ld_aux = 0
    if aux is not None:
        Ma, ld_aux = _rows(aux)
        assert Ma == M
    if bf_io:
        if not (_BF16["on"] and K % 64 == 0 and lda % 8 == 0 and x.data_ptr() % 16 == 0 and beta == 0.0):
            raise _lib.DasaError("bf16 activations: bf16_matmul mode, K % 64 == 0, 16-B rows and beta 0 only")
        gemm_bf16(x, _bf16_weight(W), out, M=M, N=N, K=K, lda=lda, ldc=ldc, bias=b, act=act, aux=aux,
                  ld_aux=ld_aux, colscale=colscale, alpha=alpha, beta=beta)
        return out
    if _BF16["on"] and K % 64 == 0 and lda % 4 == 0 and x.data_ptr() % 16 == 0:
        tw = getattr(x, "_dasa_bf16", None)   # a LayerNorm output's bf16 twin (layernorm), still current
        if tw is not None and tw[1] == x._version and beta == 0.0 and lda == K and tw[0].data_ptr() % 16 == 0:
            x = tw[0]
        gemm_bf16(x, _bf16_weight(W), out, M=M, N=N, K=K, lda=lda, ldc=ldc, bias=b, act=act, aux=aux,
                  ld_aux=ld_aux, colscale=colscale, alpha=alpha, beta=beta)
        return out
    if _emu_ok(M, N, K, lda, x):
        gemm_f32x6(x, _x6_weight(W), out, M=M, N=N, K=K, lda=lda, ldc=ldc, bias=b, act=act, aux=aux,
                   ld_aux=ld_aux, colscale=colscale, alpha=alpha, beta=beta)
        return out
    gemm(x, W, out, M=M, N=N, K=K, opA=0, opB=1, lda=lda, ldb=W.stride(0), ldc=ldc, bias=b, act=act,
         aux=aux, ld_aux=ld_aux, colscale=colscale, alpha=alpha, beta=beta)
    return out


def matmul_nn(A, B, out=None, beta=0.0):
    """out[M,N] = A[M,K] @ B[K,N] (both row-major, row-strided ok)."""
    M, lda = _rows(A)
    K = A.shape[-1]
    Kb, ldb = _rows(B)
    assert Kb == K
    N = B.shape[-1]
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=A.device)
    _, ldc = _rows(out)
    gemm(A, B, out, M=M, N=N, K=K, opA=0, opB=0, lda=lda, ldb=ldb, ldc=ldc, beta=beta)
    return out


# TN weight-gradient GEMMs on the bf16x6 TN kernel (gemm_tn.hip) when K is long and the output has enough tiles
# (profiles/r06/tn/probe.log: the bi-LSTM's 4096 x {768, 1024} x 112000 1.9x / 1.65x the native kernel, 4096 x
# 2240 x 1400 1.4x, 2048 x 2176 x 1400 equal); DASA_X6_TN=0 keeps them on the native fp32 kernels (A/B)
_X6_TN = {"on": os.environ.get("DASA_X6_TN", "1") != "0", "min_k": int(os.environ.get("DASA_X6_TN_MIN_K", "1024"))}


def _tn_x6_ok(A, B, M, N, K, lda, ldb):
    tiles = -(-M // 128) * -(-N // 128)
    return (_X6_TN["on"] and _EMU["on"] and K >= _X6_TN["min_k"] and tiles >= (128 if K >= 8192 else 384)
            and M % 2 == 0 and N % 2 == 0 and lda % 2 == 0 and ldb % 2 == 0 and A.data_ptr() % 8 == 0
            and B.data_ptr() % 8 == 0)


def gemm_f32x6_tn(A, B, out, *, M, N, K, lda, ldb, ldc, alpha=1.0, beta=0.0):
    """out = alpha * A[K,M]^T B[K,N] + beta * out at fp32 accuracy on the bf16 matrix cores (dasa_gemm_f32x6_tn)."""
    d = GemmDesc()
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), 1
    d.opA, d.opB = 1, 0
    d.A, d.lda, d.strideA = _p(A), int(lda), 0
    d.B, d.ldb, d.strideB = _p(B), int(ldb), 0
    d.C, d.ldc, d.strideC = _p(out), int(ldc), 0
    d.bias, d.act, d.aux, d.ld_aux, d.strideAux, d.colscale = None, 0, None, 0, 0, None
    d.alpha, d.beta = float(alpha), float(beta)
    L = _lib.lib()
    need = L.dasa_gemm_f32x6_tn_workspace(ctypes.byref(d))
    ws, ws_bytes = _gemm_ws(out.device, d, need) if need else (0, 0)
    _call("dasa_gemm_f32x6_tn", "gemm_x6_tn", L.dasa_gemm_f32x6_tn, ctypes.byref(d), ws, ws_bytes, _stream(),
          flops=2.0 * M * N * K, nbytes=4.0 * (M * K + K * N + M * N), detail=(int(M), int(N), int(K)))


def matmul_tn(A, B, out=None, beta=0.0, alpha=1.0):
    """out[M,N] = alpha * A[K,M]^T @ B[K,N] (+ beta * out) (weight gradients: dW = dY^T X). Long-K products
    with enough output tiles (the bi-LSTM weight gradients, K = 112000) run on the bf16x6 TN kernel."""
    K, lda = _rows(A)
    M = A.shape[-1]
    Kb, ldb = _rows(B)
    assert Kb == K
    N = B.shape[-1]
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=A.device)
    _, ldc = _rows(out)
    if K > 0 and _tn_x6_ok(A, B, M, N, K, lda, ldb):
        gemm_f32x6_tn(A, B, out, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=ldc, alpha=alpha, beta=beta)
        return out
    gemm(A, B, out, M=M, N=N, K=K, opA=1, opB=0, lda=lda, ldb=ldb, ldc=ldc, alpha=alpha, beta=beta)
    return out


def colsum(X, out=None, beta=0.0):
    """out[N] = sum over rows of X[M,N] (bias gradients), as a 1 x M GEMM."""
    M, ldx = _rows(X)
    N = X.shape[-1]
    ones = torch.ones(1, M, dtype=torch.float32, device=X.device)
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=X.device)
    gemm(ones, X, out, M=1, N=N, K=M, opA=0, opB=0, lda=M, ldb=ldx, ldc=N, beta=beta)
    return out


# ------------------------------------------------------------------------------------ elementwise
def act_fwd(x, act):
    x = x.contiguous()
    y = torch.empty_like(x)
    _call("dasa_act_fwd", "elementwise", _lib.lib().dasa_act_fwd, _p(x), _p(y), x.numel(), _ACT_IDS[act], _stream(),
          nbytes=8.0 * x.numel())
    return y


def add2d(a, b, out=None):
    rows, lda = _rows(a)
    _, ldb = _rows(b)
    if out is None:
        out = torch.empty(a.shape, dtype=torch.float32, device=a.device)
    _, ldo = _rows(out)
    _call("dasa_add2d", "elementwise", _lib.lib().dasa_add2d, _p(a), lda, _p(b), ldb, _p(out), ldo, rows, a.shape[-1], _stream(),
          nbytes=12.0 * rows * a.shape[-1])
    return out


def act_bwd(y_or_x, dy, act):
    dx = torch.empty_like(dy)
    _call("dasa_act_bwd", "elementwise", _lib.lib().dasa_act_bwd, _p(y_or_x.contiguous()), _p(dy.contiguous()), _p(dx), dy.numel(),
          _ACT_IDS[act], _stream(), nbytes=12.0 * dy.numel())
    return dx


def dropout(x, p, seed, out=None):
    """Counter-RNG dropout on a [rows, cols] (row-strided) block; same seed -> same mask."""
    rows, ldx = _rows(x)
    cols = x.shape[-1]
    if out is None:
        out = torch.empty_like(x)
    _, ldy = _rows(out)
    _call("dasa_dropout_fwd", "elementwise", _lib.lib().dasa_dropout_fwd, _p(x), ldx, _p(out), ldy, rows, cols, float(p), int(seed) & (2**64 - 1),
          _stream(), nbytes=8.0 * rows * cols)
    return out


_BATCHED_COPY = os.environ.get("DASA_BATCHED_COPY", "1") != "0"     # 0: torch copies (A/B)


def _copy_layout(src, dst):
    """Joint (n0, n1, inner elements, src s0, src s1, dst s0, dst s1) in elements for a pair whose innermost
    dim is contiguous in both and whose other dims collapse (contiguous in BOTH) to at most two, else None."""
    if src.dim() == 0:
        return 1, 1, 1, 0, 0, 0, 0
    dims = []                       # (extent, src stride, dst stride), innermost first
    for n, a, b in zip(reversed(src.shape), reversed(src.stride()), reversed(dst.stride())):
        if n == 1:
            continue
        if dims and a == dims[-1][0] * dims[-1][1] and b == dims[-1][0] * dims[-1][2]:
            dims[-1] = (dims[-1][0] * n, dims[-1][1], dims[-1][2])
        else:
            dims.append((n, a, b))
    if not dims:
        return 1, 1, 1, 0, 0, 0, 0
    if dims[0][1] != 1 or dims[0][2] != 1:
        dims.insert(0, (1, 1, 1))
    if len(dims) > 3:
        return None
    while len(dims) < 3:
        dims.append((1, 0, 0))
    (inner, _, _), (n1, a1, b1), (n0, a0, b0) = dims
    return n0, n1, inner, a0, a1, b0, b1


def copy_many(pairs):
    """dst.copy_(src) for every (src, dst) pair (same shape and dtype, same device) in batched launches of
    dasa_copy_segments; a pair whose layouts do not fit a segment is copied by torch."""
    segs = []
    nbytes = 0.0
    for src, dst in pairs:
        if src is None or dst is None or src.numel() == 0:
            continue
        if not _BATCHED_COPY:
            dst.copy_(src)
            continue
        assert src.shape == dst.shape and src.dtype == dst.dtype, (src.shape, dst.shape, src.dtype, dst.dtype)
        lay = _copy_layout(src, dst) if src.device == dst.device and src.is_cuda else None
        if lay is None:
            dst.copy_(src)
            continue
        es = src.element_size()
        seg = _lib.CopySeg()
        seg.src, seg.dst = src.data_ptr(), dst.data_ptr()
        seg.n0, seg.n1, seg.row_bytes = lay[0], lay[1], lay[2] * es
        seg.src_s0, seg.src_s1, seg.dst_s0, seg.dst_s1 = lay[3] * es, lay[4] * es, lay[5] * es, lay[6] * es
        segs.append(seg)
        nbytes += 2.0 * src.numel() * es
    L = _lib.lib()
    for i in range(0, len(segs), _lib.COPY_MAX_SEGS):
        chunk = segs[i:i + _lib.COPY_MAX_SEGS]
        arr = (_lib.CopySeg * len(chunk))(*chunk)
        _call("dasa_copy_segments", "elementwise", L.dasa_copy_segments, arr, len(chunk), _stream(), nbytes=nbytes)
        nbytes = 0.0


def copy2d(x, out):
    rows, ldx = _rows(x)
    _, ldo = _rows(out)
    _call("dasa_copy2d", "elementwise", _lib.lib().dasa_copy2d, _p(x), ldx, _p(out), ldo, rows, x.shape[-1], _stream(),
          nbytes=8.0 * rows * x.shape[-1])
    return out


def colscale(x, scale, out):
    rows, ldx = _rows(x)
    _, ldo = _rows(out)
    _call("dasa_colscale", "elementwise", _lib.lib().dasa_colscale, _p(x), ldx, _p(scale.contiguous()), _p(out), ldo, rows, x.shape[-1], _stream(),
          nbytes=8.0 * rows * x.shape[-1])
    return out


def ada_gate_fwd(s, f, noise, out):
    rows, lds = _rows(s)
    _, ldf = _rows(f)
    _, ldo = _rows(out)
    _call("dasa_ada_gate_fwd", "ada_gate", _lib.lib().dasa_ada_gate_fwd, _p(s), lds, _p(f), ldf, _p(noise), _p(out), ldo, rows, s.shape[-1],
          _stream(), nbytes=12.0 * rows * s.shape[-1])
    return out


def ada_gate_bwd(dout, s, f, noise):
    rows, lddo = _rows(dout)
    _, lds = _rows(s)
    _, ldf = _rows(f)
    dz = torch.empty(rows, s.shape[-1], dtype=torch.float32, device=s.device)
    _call("dasa_ada_gate_bwd", "ada_gate", _lib.lib().dasa_ada_gate_bwd, _p(dout), lddo, _p(s), lds, _p(f), ldf, _p(noise), _p(dz), s.shape[-1],
          rows, s.shape[-1], _stream(), nbytes=16.0 * rows * s.shape[-1])
    return dz


# -------------------------------------------------------------------------------------- LayerNorm
def layernorm(x, gamma, beta, eps, res=None, drop_p=0.0, seed=0, save=False):
    M, ld = _rows(x)
    N = x.shape[-1]
    assert ld == N, "layernorm expects contiguous rows"
    y = torch.empty_like(x)
    mean = rstd = xsum = None
    if save:
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        xsum = torch.empty_like(x)
    if not save and _BF16["on"] and _BF16["acts"] and N % 64 == 0:
        # configs[4] bf16 mode: a bf16 twin of y for the next bf16 GEMM's A operand (linear() takes it)
        ybf = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        _call("dasa_layernorm_fwd_bf16", "layernorm", _lib.lib().dasa_layernorm_fwd_bf16, _p(x), _p(res), _p(gamma),
              _p(beta), _p(y), _p(ybf), None, None, None, M, N, float(eps), float(drop_p), int(seed) & (2**64 - 1),
              _stream(), nbytes=M * N * (4.0 * (3 if res is not None else 2) + 2.0))
        y._dasa_bf16 = (ybf, y._version)
        return y
    _call("dasa_layernorm_fwd", "layernorm", _lib.lib().dasa_layernorm_fwd, _p(x), _p(res), _p(gamma), _p(beta),
          _p(y), _p(mean), _p(rstd), _p(xsum), M, N, float(eps), float(drop_p), int(seed) & (2**64 - 1), _stream(),
          nbytes=4.0 * M * N * (3 if res is not None else 2))
    if save:
        return y, (xsum, mean, rstd)
    return y


def layernorm_bwd(dy, saved, gamma, dgamma, dbeta):
    xsum, mean, rstd = saved
    M, _ = _rows(xsum)
    N = xsum.shape[-1]
    dx = torch.empty_like(xsum)
    _call("dasa_layernorm_bwd", "layernorm_bwd", _lib.lib().dasa_layernorm_bwd, _p(dy.contiguous()), _p(xsum), _p(gamma), _p(mean), _p(rstd), _p(dx),
                                        _p(dgamma), _p(dbeta), M, N, _stream(), nbytes=12.0 * M * N)
    return dx


def bert_embed(ids, word, pos, type0, gamma, beta, eps, drop_p=0.0, seed=0):
    B, L = ids.shape
    H = word.shape[1]
    out = torch.empty(B, L, H, dtype=torch.float32, device=word.device)
    ids = ids.contiguous().to(torch.int64)
    _call("dasa_bert_embed_fwd", "embed", _lib.lib().dasa_bert_embed_fwd, _p(ids), _p(word), _p(pos), _p(type0),
          _p(gamma), _p(beta), _p(out), B, L, H, float(eps), float(drop_p), int(seed) & (2**64 - 1), _stream(),
          nbytes=4.0 * 3 * B * L * H)
    return out


def mha(Q, K, V, addmask, heads, scale, drop_p=0.0, seed=0, save_probs=False):
    """Q [B, Lq, heads*64], K/V [B, Lk, heads*64] (row-strided ok), addmask [B, Lk] or None."""
    B, Lq, Hd = Q.shape
    Lk = K.shape[1]
    dh = Hd // heads
    for t in (Q, K, V):   # rows may be strided views of a fused QKV buffer, heads contiguous inside a row
        assert t.stride(2) == 1 and t.stride(0) == t.shape[1] * t.stride(1)
    if Q.dtype == torch.bfloat16 or K.dtype == torch.bfloat16 or V.dtype == torch.bfloat16:
        # configs[4]'s bf16 mode: the bf16 attention core, bf16 output (its consumer, the attention output
        # projection, is a bf16 GEMM that takes a bf16 A operand)
        if not (_BF16["on"] and Q.dtype == K.dtype == V.dtype == torch.bfloat16) or save_probs:
            raise _lib.DasaError("bf16 attention: bf16_matmul mode, bf16 Q/K/V, forward only")
        out = torch.empty(B, Lq, Hd, dtype=torch.bfloat16, device=Q.device)
        _call("dasa_mha_fwd_bf16", "mha", _lib.lib().dasa_mha_fwd_bf16, _p(Q), Q.stride(1), _p(K), K.stride(1), _p(V),
              V.stride(1), _p(addmask.contiguous() if addmask is not None else None), _p(out), Hd, 1, B, heads, Lq,
              Lk, dh, float(scale), float(drop_p), int(seed) & (2**64 - 1), _stream(),
              flops=4.0 * B * Lq * Lk * Hd, nbytes=2.0 * B * (2 * Lq + 2 * Lk) * Hd)
        return out
    out = torch.empty(B, Lq, Hd, dtype=torch.float32, device=Q.device)
    probs = torch.empty(B, heads, Lq, Lk, dtype=torch.float32, device=Q.device) if save_probs else None
    _call("dasa_mha_fwd", "mha", _lib.lib().dasa_mha_fwd, _p(Q), Q.stride(1), _p(K), K.stride(1), _p(V), V.stride(1),
          _p(addmask.contiguous() if addmask is not None else None), _p(out), Hd, _p(probs),
          B, heads, Lq, Lk, dh, float(scale), float(drop_p), int(seed) & (2**64 - 1), _stream(),
          flops=4.0 * B * Lq * Lk * Hd, nbytes=4.0 * B * (2 * Lq + 2 * Lk) * Hd)
    return (out, probs) if save_probs else out


def mha_bwd(Q, K, V, probs, dout, heads, scale, drop_p=0.0, seed=0):
    B, Lq, Hd = Q.shape
    Lk = K.shape[1]
    Q, K, V, dout = Q.contiguous(), K.contiguous(), V.contiguous(), dout.contiguous()
    dQ, dK, dV = torch.empty_like(Q), torch.empty_like(K), torch.empty_like(V)
    _call("dasa_mha_bwd", "mha_bwd", _lib.lib().dasa_mha_bwd, _p(Q), Hd, _p(K), Hd, _p(V), Hd, _p(probs), _p(dout), Hd, _p(dQ), _p(dK), _p(dV),
                                  B, heads, Lq, Lk, Hd // heads, float(scale), float(drop_p), int(seed) & (2**64 - 1),
                                  _stream(), flops=8.0 * B * Lq * Lk * Hd, nbytes=4.0 * B * (4 * Lq + 4 * Lk) * Hd)
    return dQ, dK, dV


# ------------------------------------------------------------------------------ policy head
POLICY_MODES = {"teacher": 0, "argmax": 1, "sample": 2, "forced": 3, "sample_argmax": 4}


def policy_head_fwd(logit, cand_len_i32, target, mode, seed, ignore_index=-100, forced=None):
    """One step's candidate mask + CE + action (include/dasa_hip.h dasa_policy_head_fwd).
    mode "forced": `forced` [B] int64 (device) is the action, entropy / log-prob as in "sample".
    Returns (ce_sum [], ent [B], logp_a [B], action [B] int64 or None, logp [B, C])."""
    _f32(logit, "policy_head.logit")
    B, C = logit.shape
    assert logit.stride(1) == 1
    dev = logit.device
    logp = torch.empty(B, C, dtype=torch.float32, device=dev)
    ce = torch.empty((), dtype=torch.float32, device=dev)
    ent = torch.empty(B, dtype=torch.float32, device=dev)
    logp_a = torch.empty(B, dtype=torch.float32, device=dev)
    m = POLICY_MODES[mode]
    if m == 3:
        if forced is None or forced.dtype != torch.int64 or forced.shape != (B,):
            raise _lib.DasaError("policy_head mode 'forced' needs an int64 [B] action tensor")
        action = forced.contiguous()
    else:
        action = torch.empty(B, dtype=torch.int64, device=dev) if m != 0 else None
    ws = torch.empty(B, dtype=torch.float32, device=dev)
    tgt = target.contiguous() if target is not None else None
    _call("dasa_policy_head_fwd", "policy_head", _lib.lib().dasa_policy_head_fwd, _p(logit), logit.stride(0),
          _p(cand_len_i32), _p(tgt), B, C, m, int(ignore_index), int(seed), _p(logp), _p(ce), _p(ent),
          _p(logp_a), _p(action), _p(ws), _stream(), nbytes=4.0 * B * (3 * C + 6))
    return ce, ent, logp_a, action, logp


def policy_head_bwd(logp, cand_len_i32, target, action, ent, d_ce, d_logp_a, d_ent, mode, ignore_index=-100):
    B, C = logp.shape
    dlogit = torch.empty(B, C, dtype=torch.float32, device=logp.device)
    _call("dasa_policy_head_bwd", "policy_head", _lib.lib().dasa_policy_head_bwd, _p(logp), _p(cand_len_i32),
          _p(target), _p(action), _p(ent), _p(d_ce), _p(d_logp_a), _p(d_ent), _p(dlogit), C, B, C,
          POLICY_MODES[mode], int(ignore_index), _stream(), nbytes=4.0 * B * 3 * C)
    return dlogit


# ------------------------------------------------------------------------------ SoftDot attention
_AWS = {}


def attn_set_mode(mode):
    """Attention implementation (include/dasa_hip.h dasa_attn_set_mode): 0 automatic (B < 128: the
    two-launch D-split forms), 1 row-split only (tests), 2 = 0."""
    _lib.check(_lib.lib().dasa_attn_set_mode(int(mode)), "dasa_attn_set_mode")


def attn_debug_buffer(buf):
    """Diagnosis hook (include/dasa_hip.h dasa_attn_debug_buffer): the next row-split forward launch dumps
    its per-workgroup records into `buf` (float32, device; None disarms). Returns the record size in
    floats."""
    if buf is None:
        _lib.check(_lib.lib().dasa_attn_debug_buffer(None, 0), "dasa_attn_debug_buffer")
    else:
        _lib.check(_lib.lib().dasa_attn_debug_buffer(_p(buf), buf.numel() * 4), "dasa_attn_debug_buffer")
    return int(_lib.lib().dasa_attn_debug_record_floats())


def _attn_ws(device, B, N, D):
    """Attention workspace (include/dasa_hip.h dasa_attn_workspace): one zero-initialised buffer per
    (device, stream), grown on demand. Its leading arrival counters are left zero by every call, so
    the buffer is zeroed only when (re)allocated; calls on one stream never overlap. The D-split form
    polls them with a bounded wait, so every call also joins the error-word registry."""
    _error_word(device)
    need = int(_lib.lib().dasa_attn_workspace(int(B), int(N), int(D)))
    key = (device.index, _stream())
    buf = _AWS.get(key)
    if buf is None or buf.numel() * 4 < need:
        if buf is not None:
            _WS_OLD.append(buf)      # kernels already queued / captured in a graph still point at it
        buf = torch.zeros(max(need, 1 << 20) // 4 + 4, dtype=torch.float32, device=device)
        _AWS[key] = buf
    return buf


def softdot_fwd(q, ctx, mask=None, want_scores=True, want_probs=True, want_wctx=True):
    """q [B, D]; ctx [B, N, D] (rows may be strided, e.g. a 2176 block); mask [B, N] bool."""
    B, N, D = ctx.shape
    ldn = ctx.stride(1)
    assert ctx.stride(2) == 1 and ctx.stride(0) == N * ldn
    q = q.contiguous()
    scores = torch.empty(B, N, dtype=torch.float32, device=q.device)
    probs = torch.empty(B, N, dtype=torch.float32, device=q.device) if want_probs else None
    wctx = torch.empty(B, D, dtype=torch.float32, device=q.device) if want_wctx else None
    m = mask.to(torch.uint8).contiguous() if mask is not None else None
    ws = _attn_ws(q.device, B, N, D)
    fam = "softdot" if (probs is not None or wctx is not None) else "cand_logit"
    _call("dasa_softdot_fwd", fam, _lib.lib().dasa_softdot_fwd, _p(q), _p(ctx), ldn, _p(m), _p(scores), _p(probs),
          _p(wctx), B, N, D, _p(ws), _stream(),
          nbytes=4.0 * B * (N * D + D + (D if wctx is not None else 0) + 2 * N))
    return scores, probs, wctx


def softdot_bwd(q, ctx, probs, dwctx=None, dscores=None, want_dctx=True):
    B, N, D = ctx.shape
    ldn = ctx.stride(1)
    dq = torch.empty(B, D, dtype=torch.float32, device=q.device)
    dctx = torch.empty(B, N, D, dtype=torch.float32, device=q.device) if want_dctx else None
    ws = _attn_ws(q.device, B, N, D)
    if dctx is not None:
        assert ldn == D, "dctx is written dense; pass a contiguous ctx for backward"
    fam = "softdot_bwd" if dwctx is not None else "cand_logit_bwd"
    _call("dasa_softdot_bwd", fam, _lib.lib().dasa_softdot_bwd, _p(q.contiguous()), _p(ctx), ldn, _p(probs),
          _p(dwctx.contiguous() if dwctx is not None else None),
          _p(dscores.contiguous() if dscores is not None else None), _p(dq), _p(dctx), 0,
          B, N, D, _p(ws), _stream(),
          nbytes=4.0 * B * (N * D + (N * D if dctx is not None else 0) + 3 * D + 3 * N))
    return dq, dctx


def shift_attn_fwd(q, ctx, shift_logits):
    B, N, D = ctx.shape
    assert N == 36
    ldn = ctx.stride(1)
    assert ctx.stride(2) == 1 and ctx.stride(0) == N * ldn
    K = shift_logits.shape[1]
    attn = torch.empty(B, N, dtype=torch.float32, device=q.device)
    shifted = torch.empty_like(attn)
    wsm = torch.empty(B, K, dtype=torch.float32, device=q.device)
    wctx = torch.empty(B, D, dtype=torch.float32, device=q.device)
    ws = _attn_ws(q.device, B, N, D)
    _call("dasa_shift_attn_fwd", "shift_attn", _lib.lib().dasa_shift_attn_fwd, _p(q.contiguous()), _p(ctx), ldn,
          _p(shift_logits.contiguous()), _p(attn), _p(shifted), _p(wsm), _p(wctx), B, D, K, _p(ws), _stream(),
          nbytes=4.0 * B * (N * D + 2 * D + 3 * N))
    return wctx, attn, shifted, wsm


def shift_attn_bwd(q, ctx, attn, shifted, wsm, dwctx, want_dctx=True):
    B, N, D = ctx.shape
    ldn = ctx.stride(1)
    K = wsm.shape[1]
    dq = torch.empty(B, D, dtype=torch.float32, device=q.device)
    dctx = torch.empty(B, N, D, dtype=torch.float32, device=q.device) if want_dctx else None
    if dctx is not None:
        assert ldn == D, "dctx is written dense; pass a contiguous ctx for backward"
    dz = torch.empty(B, K, dtype=torch.float32, device=q.device)
    ws = _attn_ws(q.device, B, N, D)
    _call("dasa_shift_attn_bwd", "shift_attn_bwd", _lib.lib().dasa_shift_attn_bwd, _p(q.contiguous()), _p(ctx), ldn,
          _p(attn), _p(shifted), _p(wsm), _p(dwctx.contiguous()), _p(dq), _p(dctx), _p(dz), 0, B, D, K, _p(ws),
          _stream(), nbytes=4.0 * B * (N * D + (N * D if dctx is not None else 0) + 3 * D + 3 * N))
    return dq, dctx, dz


# ------------------------------------------------------------------------------------------ LSTM
def lstm_cell_fwd(gates, c_prev, save=False):
    B, G4 = gates.shape
    H = G4 // 4
    h = torch.empty(B, H, dtype=torch.float32, device=gates.device)
    c = torch.empty_like(h)
    act = torch.empty_like(gates) if save else None
    _call("dasa_lstm_cell_fwd", "lstm_cell", _lib.lib().dasa_lstm_cell_fwd, _p(gates.contiguous()), _p(c_prev.contiguous()), _p(h), _p(c), _p(act), B, H,
          _stream(), nbytes=4.0 * B * (4 * H + H + 2 * H + (4 * H if act is not None else 0)))
    return h, c, act


def lstm_cell_bwd(act, c_prev, c, dh, dc):
    B, G4 = act.shape
    H = G4 // 4
    dgates = torch.empty_like(act)
    dc_prev = torch.empty(B, H, dtype=torch.float32, device=act.device)
    _call("dasa_lstm_cell_bwd", "lstm_cell", _lib.lib().dasa_lstm_cell_bwd, _p(act), _p(c_prev.contiguous()), _p(c), _p(dh.contiguous() if dh is not None else None),
                                        _p(dc.contiguous() if dc is not None else None), _p(dgates), _p(dc_prev), B, H,
          _stream(), nbytes=4.0 * B * (4 * H + 4 * H + H + 3 * H))
    return dgates, dc_prev


_ERR = {}


def _error_word(dev):
    """The device error word of `dev` (include/dasa_hip.h dasa_set_error_word): persistent kernels
    OR a bit into it when their inter-workgroup barrier times out (and poison their outputs)."""
    w = _ERR.get(dev.index)
    if w is None:
        w = torch.zeros(1, dtype=torch.int32, device=dev)
        _ERR[dev.index] = w
        _lib.check(_lib.lib().dasa_set_error_word(w.data_ptr()), "dasa_set_error_word")
    return w


_ERR_BITS = {1: "persistent bi-LSTM forward: inter-workgroup barrier timed out (outputs poisoned with NaN)",
             2: "persistent bi-LSTM BPTT: inter-workgroup barrier timed out (gate gradients poisoned with NaN)",
             4: "D-split attention: group barrier timed out (outputs poisoned with NaN)"}


def check_device_errors():
    """Raise DasaError if a kernel reported a device-side failure since the last check. Reads the
    error word(s) from the device (a host sync: call it where the caller syncs anyway)."""
    for idx, w in _ERR.items():
        v = int(w.item())
        if v:
            w.zero_()
            # a timed-out barrier may leave the inter-workgroup counters of the workspaces non-zero:
            # drop the cached workspaces (re-allocated zeroed on next use)
            _WS_OLD.extend(_AWS.values())     # captured graphs may still point at them
            _AWS.clear()
            msgs = [m for bit, m in _ERR_BITS.items() if v & bit] or [f"error word 0x{v:x}"]
            raise _lib.DasaError(f"device-side failure on cuda:{idx}: " + "; ".join(msgs))


def force_persist_timeout(on):
    """Test hook: every persistent-kernel barrier takes its timeout path."""
    _lib.check(_lib.lib().dasa_persist_force_timeout(1 if on else 0), "dasa_persist_force_timeout")


_CONCURRENT = []


def register_concurrent_stream(st):
    """A stream that may run kernels beside the main stream (the train-mode language pipe). The
    persistent bi-LSTM kernels need every CU, so their launches first join every such stream."""
    if all(st is not s for s in _CONCURRENT):
        _CONCURRENT.append(st)


def _exclusive(dev):
    if torch.cuda.is_current_stream_capturing():
        return      # a captured region is joined before its replay (Seq2SeqAgent's step graph)
    cur = torch.cuda.current_stream(dev)
    for st in _CONCURRENT:
        if st.device == dev and st != cur:
            cur.wait_stream(st)


def bilstm_fwd(xproj, whh_f, whh_b, lengths_i32, H, save=False):
    """xproj [B, L, 2, 4H]; whh_f/whh_b [4H, H]; lengths int32 [B] (device). Returns out [B, L, 2H],
    h_n [2, B, H], c_n [2, B, H], saved (act, c) or None."""
    B, L = xproj.shape[0], xproj.shape[1]
    dev = xproj.device
    out = torch.empty(B, L, 2 * H, dtype=torch.float32, device=dev)
    h_n = torch.empty(2, B, H, dtype=torch.float32, device=dev)
    c_n = torch.empty_like(h_n)
    sa = sc = None
    if save:
        sa = torch.empty(L, 2, B, 4 * H, dtype=torch.float32, device=dev)
        sc = torch.empty(L, 2, B, H, dtype=torch.float32, device=dev)
    L_ = _lib.lib()
    ws = torch.empty(L_.dasa_bilstm_workspace(B, H) // 4, dtype=torch.float32, device=dev)
    _error_word(dev)
    _exclusive(dev)
    _call("dasa_bilstm_fwd", "bilstm", L_.dasa_bilstm_fwd, _p(xproj.contiguous()), _p(whh_f.contiguous()),
          _p(whh_b.contiguous()), _p(lengths_i32), _p(out), _p(h_n), _p(c_n), _p(sa), _p(sc), B, L, H, _p(ws), _stream(),
          flops=2.0 * 2 * L * B * 4 * H * H, nbytes=4.0 * L * 2 * 4 * H * H)
    return out, h_n, c_n, ((sa, sc) if save else None)


def bilstm_bwd(whh_f, whh_b, lengths_i32, saved, dout, dh_n, dc_n, H):
    sa, sc = saved
    L, _, B, _ = sa.shape
    dev = sa.device
    dgates = torch.empty(B, L, 2, 4 * H, dtype=torch.float32, device=dev)
    ws = torch.empty(_lib.lib().dasa_bilstm_bwd_workspace(B, H) // 4 + 4, dtype=torch.float32, device=dev)
    _error_word(dev)
    _exclusive(dev)
    _call("dasa_bilstm_bwd", "bilstm_bptt", _lib.lib().dasa_bilstm_bwd, _p(whh_f.contiguous()), _p(whh_b.contiguous()),
          _p(lengths_i32), _p(sa), _p(sc), _p(dout.contiguous()),
          _p(dh_n.contiguous() if dh_n is not None else None),
          _p(dc_n.contiguous() if dc_n is not None else None), _p(dgates), B, L, H, _p(ws), _stream(),
          flops=2.0 * 2 * L * B * 4 * H * H, nbytes=4.0 * L * 2 * 4 * H * H)
    return dgates


def bilstm_hprev(out, H):
    B, L, _ = out.shape
    hprev = torch.empty(2, B, L, H, dtype=torch.float32, device=out.device)
    _call("dasa_bilstm_hprev", "elementwise", _lib.lib().dasa_bilstm_hprev, _p(out.contiguous()), _p(hprev), B, L, H, _stream(),
          nbytes=16.0 * B * L * H)
    return hprev


def bilstm_dw_hh(dgates, out, d, H):
    """dW_hh of direction d of a packed bi-LSTM (r2rmodel.py:2339-2343, nn.LSTM's weight_hh gradient):
    sum over (sequence, t) of dgates[., t, d]ᵀ h_prev(t), with h_prev the direction's previous output —
    fwd out[., t-1, :H], bwd out[., t+1, H:], zero at the sequence ends — read IN PLACE from `out` (VERDICT
    r05 #6: no shifted copy; bilstm_hprev wrote 0.9 GB per flush for it). One TN GEMM over all rows with the
    two operands offset by one row, then one small GEMM (alpha = -1, beta = 1) removing the NB - 1 pairs that
    offset pairs across a sequence boundary (fwd: dgates[n, 0] with out[n-1, L-1]; bwd: dgates[n, L-1] with
    out[n+1, 0]). Rows past a sequence's length carry zero dgates, as with the copy. dgates [NB, L, 2, 4H],
    out [NB, L, 2H] (contiguous); returns [4H, H]."""
    NB, L = dgates.shape[0], dgates.shape[1]
    G = dgates.shape[-1]
    assert dgates.is_contiguous() and out.is_contiguous() and tuple(out.shape) == (NB, L, 2 * H) and G == 4 * H
    res = torch.empty(G, H, dtype=torch.float32, device=dgates.device)
    if NB * L < 2:
        return res.zero_()
    dg = dgates.view(NB * L, 2, G)[:, d, :]           # [NB*L, 4H], row stride 8H
    h = out.view(NB * L, 2 * H)[:, d * H:(d + 1) * H]  # [NB*L, H], row stride 2H
    if d == 0:
        matmul_tn(dg[1:], h[:-1], out=res)
        if NB > 1:
            A, B = dgates[1:, 0, 0, :], out[:-1, L - 1, :H]
    else:
        matmul_tn(dg[:-1], h[1:], out=res)
        if NB > 1:
            A, B = dgates[:-1, L - 1, 1, :], out[1:, 0, H:]
    if NB > 1:
        gemm(A, B, res, M=G, N=H, K=NB - 1, opA=1, opB=0, lda=A.stride(0), ldb=B.stride(0), ldc=H,
             alpha=-1.0, beta=1.0)
    return res


def reverse_valid(x, lengths_i32):
    B, L, H = x.shape
    out = torch.empty_like(x)
    _call("dasa_reverse_valid", "elementwise", _lib.lib().dasa_reverse_valid, _p(x.contiguous()), _p(lengths_i32), _p(out), B, L, H, _stream(),
          nbytes=8.0 * B * L * H)
    return out


def adain_musigma(content, style, out=None, eps=1e-5):
    """adaptive_instance_normalization (model.py:1832-1840) over the last dim of [..., N] blocks."""
    M, ldc = _rows(content)
    _, lds = _rows(style)
    N = content.shape[-1]
    if out is None:
        out = torch.empty(content.shape, dtype=torch.float32, device=content.device)
    _, ldo = _rows(out)
    _call("dasa_adain_musigma_fwd", "adain_musigma", _lib.lib().dasa_adain_musigma_fwd, _p(content), ldc, _p(style), lds, _p(out), ldo, None, M, N, float(eps),
                                            _stream(), nbytes=12.0 * M * N)
    return out


def adain_musigma_bwd(content, style, dout, want_dcontent=True, want_dstyle=True, eps=1e-5):
    """Gradients of adain_musigma w.r.t. content and style (dasa_adain_musigma_bwd)."""
    M, ldc = _rows(content)
    _, lds = _rows(style)
    _, ldg = _rows(dout)
    N = content.shape[-1]
    dc = torch.empty(content.shape, dtype=torch.float32, device=content.device) if want_dcontent else None
    ds = torch.empty(style.shape, dtype=torch.float32, device=style.device) if want_dstyle else None
    _call("dasa_adain_musigma_bwd", "adain_musigma", _lib.lib().dasa_adain_musigma_bwd, _p(content), ldc, _p(style),
          lds, _p(dout), ldg, _p(dc), N, _p(ds), N, M, N, float(eps), _stream(), nbytes=4.0 * M * N * 5)
    return dc, ds


def gather_rows(ta, ia, tb, ib, out):
    """out[r] = [ta[ia[r]] | tb[ib[r]]] (zeros for negative indices); ta [Na, Fa], tb [Nb, Fb]."""
    R = ia.numel()
    Fa = ta.shape[-1]
    Fb = tb.shape[-1] if tb is not None else out.shape[-1] - Fa
    _call("dasa_gather_rows", "gather", _lib.lib().dasa_gather_rows, _p(ta), _p(ia), Fa, _p(tb), _p(ib), Fb, _p(out),
          R, _stream(), nbytes=8.0 * R * (Fa + Fb))
    return out


# DASA_CHECK_FINITE=1|strict: every tensor-producing entry point above checks its outputs (dasa_amd/debug.py)
from . import debug as _debug  # noqa: E402
if _debug.active():
    import sys as _sys
    _debug.install(_sys.modules[__name__])
