"""ctypes binding of libdasa_hip.so (C-ABI: include/dasa_hip.h).

This is the product's only path to compute: there is no CPU fallback. If the library is missing
or cannot be loaded, `lib()` raises — callers on a GPU box therefore fail loudly instead of silently
running something else.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DASA_DEBUG=1: the debug library (device input checks compiled in; dasa_amd/build.py --debug)
LIB_PATH = os.path.join(_HERE, "libdasa_hip_debug.so" if os.environ.get("DASA_DEBUG", "0") not in ("", "0")
                        else "libdasa_hip.so")
# DASA_LIB=<path>: an alternate build of the same sources (A/B diagnosis builds, e.g. tools/build_variant.sh)
LIB_PATH = os.environ.get("DASA_LIB") or LIB_PATH

f32p = C.c_void_p  # device pointers travel as integers
i64 = C.c_int64
i32 = C.c_int32
u64 = C.c_uint64
f32 = C.c_float
vp = C.c_void_p

ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3, 4


class GemmDesc(C.Structure):
    _fields_ = [
        ("M", i32), ("N", i32), ("K", i32), ("batch", i32),
        ("opA", i32), ("opB", i32),
        ("A", vp), ("lda", i64), ("strideA", i64),
        ("B", vp), ("ldb", i64), ("strideB", i64),
        ("C", vp), ("ldc", i64), ("strideC", i64),
        ("bias", vp),
        ("act", i32),
        ("aux", vp), ("ld_aux", i64), ("strideAux", i64),
        ("colscale", vp),
        ("alpha", f32), ("beta", f32),
    ]


class CopySeg(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("n0", i64), ("n1", i64), ("row_bytes", i64),
                ("src_s0", i64), ("src_s1", i64), ("dst_s0", i64), ("dst_s1", i64)]


COPY_MAX_SEGS = 16


# name -> (restype, argtypes)
SIGNATURES = {
    "dasa_version": (i32, []),
    "dasa_build_info": (C.c_char_p, []),
    "dasa_error_string": (C.c_char_p, [i32]),
    "dasa_gemm_f32_workspace": (i64, [C.POINTER(GemmDesc)]),
    "dasa_gemm_f32": (i32, [C.POINTER(GemmDesc), vp, i64, vp]),
    "dasa_gemm_bf16": (i32, [C.POINTER(GemmDesc), vp]),
    "dasa_copy_segments": (i32, [C.POINTER(CopySeg), i32, vp]),
    "dasa_gemm_bf16_ex": (i32, [C.POINTER(GemmDesc), i32, vp]),
    "dasa_gemm_bf16_dma": (i32, [i32]),
    "dasa_f32_to_bf16": (i32, [vp, vp, i64, vp]),
    "dasa_gemm_f32x6": (i32, [C.POINTER(GemmDesc), i64, vp]),
    "dasa_gemm_f32x6_workspace": (i64, [C.POINTER(GemmDesc)]),
    "dasa_gemm_f32x6_ws": (i32, [C.POINTER(GemmDesc), i64, vp, i64, vp]),
    "dasa_gemm_f32x6_kernels": (i32, [vp, i64]),
    "dasa_gemm_f32x6_tn": (i32, [C.POINTER(GemmDesc), vp, i64, vp]),
    "dasa_gemm_f32x6_tn_workspace": (i64, [C.POINTER(GemmDesc)]),
    "dasa_gemm_x6_tn_config": (i32, [i32, i32]),
    "dasa_gemm_f32x6_pp": (i32, [C.POINTER(GemmDesc), i64, i64, i32, vp]),
    "dasa_gemm_f32x6_k64": (i32, [C.POINTER(GemmDesc), i64, i32, vp]),
    "dasa_f32_split3_bf16": (i32, [vp, i64, vp, i32, i32, vp]),
    "dasa_gemm_force_config": (i32, [i32]),
    "dasa_gemm_x6_set_balance": (i32, [i32]),
    "dasa_gemm_x6_set_tail": (i32, [i32]),
    "dasa_gemm_skinny_tune": (i32, [i32, i32]),
    "dasa_layernorm_fwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, u64, vp]),
    "dasa_layernorm_fwd_bf16": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, u64, vp]),
    "dasa_layernorm_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp]),
    "dasa_bert_embed_fwd": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, u64, vp]),
    "dasa_mha_fwd": (i32, [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, f32, f32, u64, vp]),
    "dasa_mha_fwd_bf16": (i32, [vp, i64, vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32, f32, f32, u64, vp]),
    "dasa_mha_bwd": (i32, [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, vp, vp, i32, i32, i32, i32, i32, f32, f32, u64,
                           vp]),
    "dasa_softdot_fwd": (i32, [vp, vp, i64, vp, vp, vp, vp, i32, i32, i32, vp, vp]),
    "dasa_attn_workspace": (i64, [i32, i32, i32]),
    "dasa_attn_set_mode": (i32, [i32]),
    "dasa_attn_debug_buffer": (i32, [vp, i64]),
    "dasa_attn_debug_record_floats": (i64, []),
    "dasa_softdot_bwd": (i32, [vp, vp, i64, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp]),
    "dasa_shift_attn_fwd": (i32, [vp, vp, i64, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp]),
    "dasa_shift_attn_bwd": (i32, [vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp]),
    "dasa_lstm_cell_fwd": (i32, [vp, vp, vp, vp, vp, i32, i32, vp]),
    "dasa_lstm_cell_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, vp]),
    "dasa_bilstm_workspace": (i64, [i32, i32]),
    "dasa_bilstm_fwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp]),
    "dasa_bilstm_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp]),
    "dasa_bilstm_hprev": (i32, [vp, vp, i32, i32, i32, vp]),
    "dasa_bilstm_set_mode": (i32, [i32]),
    "dasa_bilstm_bptt_x6": (i32, [i32]),
    "dasa_bilstm_bptt_one_tile": (i32, [i32]),
    "dasa_mha_bwd_split": (i32, [i32]),
    "dasa_mha_bwd_stamps": (i32, [vp]),
    "dasa_bilstm_fwd_x6": (i32, [i32]),
    "dasa_bilstm_fwd_bf16": (i32, [i32]),
    "dasa_set_error_word": (i32, [vp]),
    "dasa_persist_force_timeout": (i32, [i32]),
    "dasa_persist_stamps": (i32, [vp]),
    "dasa_bilstm_bwd_workspace": (i64, [i32, i32]),
    "dasa_adain_musigma_fwd": (i32, [vp, i64, vp, i64, vp, i64, vp, i32, i32, f32, vp]),
    "dasa_adain_musigma_bwd": (i32, [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, i32, i32, f32, vp]),
    "dasa_reverse_valid": (i32, [vp, vp, vp, i32, i32, i32, vp]),
    "dasa_dropout_fwd": (i32, [vp, i64, vp, i64, i32, i32, f32, u64, vp]),
    "dasa_set_seed_source": (i32, [vp]),
    "dasa_policy_head_fwd": (i32, [vp, i64, vp, vp, i32, i32, i32, i32, u64, vp, vp, vp, vp, vp, vp, vp]),
    "dasa_policy_head_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, vp]),
    "dasa_seed_bump": (i32, [vp, vp]),
    "dasa_ada_gate_fwd": (i32, [vp, i64, vp, i64, vp, vp, i64, i32, i32, vp]),
    "dasa_ada_gate_bwd": (i32, [vp, i64, vp, i64, vp, i64, vp, vp, i64, i32, i32, vp]),
    "dasa_act_bwd": (i32, [vp, vp, vp, i64, i32, vp]),
    "dasa_act_fwd": (i32, [vp, vp, i64, i32, vp]),
    "dasa_add2d": (i32, [vp, i64, vp, i64, vp, i64, i32, i32, vp]),
    "dasa_copy2d": (i32, [vp, i64, vp, i64, i32, i32, vp]),
    "dasa_colscale": (i32, [vp, i64, vp, vp, i64, i32, i32, vp]),
    "dasa_gather_rows": (i32, [vp, vp, i32, vp, vp, i32, vp, i32, vp]),
}

_LIB = None


class DasaError(RuntimeError):
    pass


def lib():
    """Load libdasa_hip.so (once). Raises DasaError if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise DasaError(
            f"libdasa_hip.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback for the DASA hot path)")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def check(rc, what):
    if rc != 0:
        msg = lib().dasa_error_string(rc)
        raise DasaError(f"{what} failed: hip error {rc} ({msg.decode() if msg else '?'})")
