// SoftDotAttention / ShiftSoftDotAttention forward + backward for gfx950 (model.py:253-353).
//
// HBM-bound: the compulsory traffic is one read of ctx [B][N][D] (+ one write of dctx in backward).
// At the policy's shapes a call moves 3-13 MB, so the kernels are built for latency: every
// workgroup issues all of its loads in ONE round trip and there is no grid-wide wait.
//
// Row-split layout: workgroup (j, b) owns rows [j*RB, j*RB + RB) of batch row b (RB = 12 for the
// panorama: one elevation ring of 12 headings, so the K-tap circular shift stays inside the
// workgroup; RB = 16 otherwise) and thread t owns float4 column t of those rows (D = 2176 -> 576
// threads, 2048 -> 512), holding the RB float4 in registers for both passes over them.
//   forward   scores of its rows (4-wide partial dots, reduce-scattered over the wave with 17
//             shuffles, wave partials meet in LDS), a LOCAL softmax (max m_j, sum l_j, e_r =
//             exp(s_r - m_j)), the shift of e within the ring, and the partial context
//             sum_r e'_r ctx_r; the last workgroup of b to finish (arrival counter, release/acquire
//             write-through stores, nothing ever waits) rescales the partials by exp(m_j - M) / Z and writes
//             wctx, probs and the shifted weights (the online-softmax merge).
//   backward  launch 1: dp_r = ctx_r . dwctx per row block; the last arriver forms the softmax /
//             shift backward for all N rows (ds, the weights pw, dshift). Launch 2: dctx rows and a
//             partial dq per row block; the last arriver sums the dq partials.
// Workspace: dasa_attn_workspace(); its first 2 x 32768 words are arrival counters that must be zero
// on entry and are left zero.
#include <stdlib.h>

#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

constexpr int kMaxN = 256;   // max attended rows (instruction <= 80, views 36, candidates)
constexpr int kMaxK = 15;    // max shift taps
constexpr int kMaxW = 16;    // waves per workgroup (1024 threads)
constexpr int kMaxBlk = kMaxN / 12 + 1;

__device__ __forceinline__ float dot4(const float4 a, const float4 b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}

__device__ __forceinline__ void fma4(float s, const float4 x, float4& acc) {
  acc.x = fmaf(s, x.x, acc.x);
  acc.y = fmaf(s, x.y, acc.y);
  acc.z = fmaf(s, x.z, acc.z);
  acc.w = fmaf(s, x.w, acc.w);
}

// Reduce-scatter of 16 per-lane partials over the 64-lane wave: returns on every lane the full-wave
// sum of partial (lane >> 2) & 15. Exchange on lane bits 5..2 halves the live values each step
// (8 + 4 + 2 + 1 shuffles), then bits 1..0 finish the sum (2 more).
__device__ __forceinline__ float reduce_scatter16(const float (&v)[16], int lane) {
  float u[8], w4[4], w2[2];
  {
    const bool up = lane & 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float send = up ? v[i] : v[i + 8], keep = up ? v[i + 8] : v[i];
      u[i] = keep + __shfl_xor(send, 32, 64);
    }
  }
  {
    const bool up = lane & 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float send = up ? u[i] : u[i + 4], keep = up ? u[i + 4] : u[i];
      w4[i] = keep + __shfl_xor(send, 16, 64);
    }
  }
  {
    const bool up = lane & 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float send = up ? w4[i] : w4[i + 2], keep = up ? w4[i + 2] : w4[i];
      w2[i] = keep + __shfl_xor(send, 8, 64);
    }
  }
  const bool up = lane & 4;
  float s = (up ? w2[1] : w2[0]) + __shfl_xor(up ? w2[0] : w2[1], 4, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 1, 64);
  return s;
}

// Partials handed to another workgroup of the same launch are stored write-through (sc1) and every
// load of them is sc1, so the hand-off needs no L2-wide release / acquire fence (gfx950's L2 is
// per XCD): writers drain vmcnt, then one lane takes a relaxed agent-scope ticket.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(float* ws) {
  return __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void pub1(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 16);
}
__device__ __forceinline__ void pub4(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 16);
}
__device__ __forceinline__ float get1(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}
__device__ __forceinline__ float4 get4(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}

__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
}

// Row dots of the workgroup's rows with vec, summed over the workgroup: returns on lane r < nr of
// wave 0 (valid after the internal __syncthreads) the dot of row r; thread t < D/4 keeps its float4
// of each row in x (D <= 4096, so one column per thread).
// Diagnosis dump (dasa_attn_debug_buffer; r05): per workgroup a record of kDbgRec floats —
// [0] HW_ID, [1] XCC_ID, [2] blockIdx.x, [3] blockIdx.y (as raw bits), then per thread its 16 row
// partials v[] (blockDim x 16), a checksum of its q float4 (blockDim), the 16 x 16 wave partials as
// written to red[w][r], and the 16 row dots wave 0 summed. Diagnosis only: written beside, never read.
constexpr int kDbgHdr = 4, kDbgMaxT = 1024;
constexpr int kDbgRec = kDbgHdr + kDbgMaxT * 16 + kDbgMaxT + kMaxW * 16 + 16;

//
// Loads (r05): every row of the block is read by ONE buffer_load_dwordx4 with the same per-thread byte
// offset VGPR (column t) and the row's offset in an SGPR (soffset), so no load's address lives in
// registers that a younger load's data return overwrites. The r04 form (LEG = true: a 64-bit VGPR
// address per row; the compiler reused the address registers of in-flight loads as the destinations of
// younger ones, one even overlapping its own address) returned wrong data on lanes 48-63 of one row's
// load in 10-60 % of calls while a bf16x6 form-20 GEMM started on another stream
// (tools/rowsplit_diag.py, profiles/r05/rowsplit_diag_a.log: every bad workgroup's per-thread partials
// already differ — the loads, not the reduction); the whole-row kernel, whose loads all share one offset
// VGPR, never did. LEG stays for the diagnosis (dasa_attn_set_mode(3)).
template <int RB, bool DBG = false, bool LEG = false>
__device__ __forceinline__ float block_row_dots(const float* rows, long ldn, int nr, const float* vec, int D4,
                                                float4 (&x)[RB], float (*red)[16], float* dbg = nullptr) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, W = blockDim.x >> 6;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  float qsum = 0.f;
  if (t < D4) {   // D4 <= blockDim: one float4 column per thread
    const float4 qv = reinterpret_cast<const float4*>(vec)[t];
    if (LEG) {
#pragma unroll
      for (int i = 0; i < RB; ++i) x[i] = reinterpret_cast<const float4*>(rows + (long)min(i, nr - 1) * ldn)[t];
    } else {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows), 0, 0x7fffffff,
                                                                          0x00020000);
      const int voff = t * 16;
#pragma unroll
      for (int i = 0; i < RB; ++i)
        x[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rr, voff, __builtin_amdgcn_readfirstlane(min(i, nr - 1) * (int)ldn * 4), 0));
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) v[i] = dot4(x[i], qv);
    if (DBG) qsum = (qv.x + qv.y) + (qv.z + qv.w);
  }
  if (DBG) {
#pragma unroll
    for (int i = 0; i < 16; ++i) dbg[kDbgHdr + t * 16 + i] = v[i];
    dbg[kDbgHdr + kDbgMaxT * 16 + t] = qsum;
    if (t == 0) {
      dbg[0] = __uint_as_float(__builtin_amdgcn_s_getreg(0xF804));   // HW_REG_HW_ID, 32 bits
      dbg[1] = __uint_as_float(__builtin_amdgcn_s_getreg(0xF814));   // HW_REG_XCC_ID
      dbg[2] = __uint_as_float(blockIdx.x);
      dbg[3] = __uint_as_float(blockIdx.y);
    }
  }
  const float s = reduce_scatter16(v, lane);
  const int r = (lane >> 2) & 15;
  if ((lane & 3) == 0 && r < RB) red[w][r] = s;
  if (DBG && (lane & 3) == 0) dbg[kDbgHdr + kDbgMaxT * 17 + w * 16 + r] = s;
  __syncthreads();
  float tot = 0.f;
  if (t < 64 && lane < nr)
    for (int i = 0; i < W; ++i) tot += red[i][lane];
  if (DBG && t < 16) dbg[kDbgHdr + kDbgMaxT * 17 + kMaxW * 16 + t] = tot;
  return tot;
}

// Announce this workgroup's (sc1-stored) partials for batch row b; true in exactly one workgroup,
// the last to arrive, which then reads every partial with sc1 loads.
__device__ __forceinline__ bool last_arriver(unsigned* cnt, int nblk, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its write-through stores landed
  __syncthreads();
  if (threadIdx.x == 0)
    *s_flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nblk - 1);
  __syncthreads();
  if (!*s_flag) return false;
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-arm
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep the sc1 loads below the ticket
  return true;
}

// Softmax weights over K shift taps (model.py:336) into sw[0..K), computed by wave 0.
__device__ __forceinline__ void shift_taps(const float* logits, int K, float* sw, int lane) {
  const float z = lane < K ? logits[lane] : -INFINITY;
  const float zm = wave_max(z);
  const float e = lane < K ? __expf(z - zm) : 0.f;
  const float es = wave_sum(e);
  if (lane < K) sw[lane] = e / es;
}

struct FwdArgs {
  const float* q; const float* ctx; long ldn;
  const uint8_t* mask;
  const float* shift_logits; int K;
  float* scores; float* probs; float* shifted; float* wsm; float* wctx;
  int N, D, nblk;
  unsigned* cnt; float* ws; int o_part, o_ml, o_ee;   // workspace: counters + byte offsets of partials
  float* dbg;                                          // row-split diagnosis dump (DBG instantiation only)
};

template <int RB, bool DBG = false, bool LEG = false>
__global__ __launch_bounds__(1024) void attn_fwd_kernel(FwdArgs a) {
  __shared__ float red[kMaxW][16];
  __shared__ float se[16], sep[16], sw[kMaxK + 1], ssc[kMaxBlk];
  __shared__ int s_flag;
  const int j = blockIdx.x, b = blockIdx.y, t = threadIdx.x, lane = t & 63;
  const int N = a.N, D4 = a.D >> 2, r0 = j * RB, nr = min(RB, N - r0), nblk = a.nblk;
  DASA_DCHECK((int)blockDim.x >= D4 && nr >= 1 && (int)gridDim.x == nblk, 128);   // one column per thread
  const bool shift = a.shift_logits != nullptr;
  const float* rows = a.ctx + ((long)b * N + r0) * a.ldn;
  float4 x[RB];
  const float s = block_row_dots<RB, DBG, LEG>(rows, a.ldn, nr, a.q + (long)b * a.D, D4, x, red,
                                               DBG ? a.dbg + (long)(b * nblk + j) * kDbgRec : nullptr);
  const bool combine = a.wctx || a.probs || a.shifted;
  const __amdgpu_buffer_rsrc_t wr = ws_rsrc(a.ws);
  if (t < 64) {
    float sm = -INFINITY;
    if (lane < nr) {
      if (a.scores) a.scores[(long)b * N + r0 + lane] = s;
      sm = (a.mask && a.mask[(long)b * N + r0 + lane]) ? -INFINITY : s;
    }
    const float m = wave_max(sm);
    const float e = (sm == -INFINITY) ? 0.f : __expf(sm - m);
    const float l = wave_sum(e);
    if (lane < 16) se[lane] = e;
    if (shift) shift_taps(a.shift_logits + (long)b * a.K, a.K, sw, lane);
    lds_wave_sync();
    float ep = e;
    if (shift && lane < nr) {   // RB = 12: this workgroup is one elevation ring (model.py:337-344)
      const int P = a.K / 2;
      ep = 0.f;
      for (int k = 0; k < a.K; ++k) {
        int jj = lane + k - P;
        jj = ((jj % 12) + 12) % 12;
        ep = fmaf(sw[k], se[jj], ep);
      }
    }
    if (lane < 16) sep[lane] = lane < nr ? ep : 0.f;
    if (combine && nblk > 1) {
      if (lane < nr) {
        pub1(wr, a.o_ee + ((b * N + r0 + lane) * 2) * 4, e);
        pub1(wr, a.o_ee + ((b * N + r0 + lane) * 2 + 1) * 4, ep);
      }
      if (lane == 0) {
        pub1(wr, a.o_ml + ((b * nblk + j) * 2) * 4, m);
        pub1(wr, a.o_ml + ((b * nblk + j) * 2 + 1) * 4, l);
      }
    } else if (combine) {   // single workgroup: normalise here
      const float inv = 1.f / l;
      if (lane < nr) {
        if (a.probs) a.probs[(long)b * N + lane] = e * inv;
        if (a.shifted) a.shifted[(long)b * N + lane] = ep * inv;
      }
      if (shift && a.wsm && lane < a.K) a.wsm[(long)b * a.K + lane] = sw[lane];
      if (lane == 0) ssc[0] = inv;
    }
  }
  __syncthreads();
  if (!combine) return;
  if (a.wctx && t < D4) {   // partial (or, with one workgroup, final) context from the rows in VGPRs
    const float sc = nblk == 1 ? ssc[0] : 1.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < RB; ++i) fma4(i < nr ? sep[i] * sc : 0.f, x[i], acc);
    if (nblk == 1) reinterpret_cast<float4*>(a.wctx + (long)b * a.D)[t] = acc;
    else pub4(wr, a.o_part + (((b * nblk + j) * a.D) + 4 * t) * 4, acc);
  }
  if (nblk == 1) return;
  if (!last_arriver(a.cnt + b, nblk, &s_flag)) return;
  // merge: M = max_j m_j, Z = sum_j exp(m_j - M) l_j; weight of block j = exp(m_j - M) / Z
  if (t < 64) {
    const int ob = a.o_ml + (b * nblk * 2) * 4;
    const float mj = lane < nblk ? get1(wr, ob + (2 * lane) * 4) : -INFINITY;
    const float lj = lane < nblk ? get1(wr, ob + (2 * lane + 1) * 4) : 0.f;
    const float M = wave_max(mj);
    const float sj = lane < nblk ? __expf(mj - M) : 0.f;
    const float Z = wave_sum(sj * lj);
    if (lane < nblk) ssc[lane] = sj / Z;
    if (shift) {
      shift_taps(a.shift_logits + (long)b * a.K, a.K, sw, lane);
      if (a.wsm && lane < a.K) a.wsm[(long)b * a.K + lane] = sw[lane];
    }
  }
  __syncthreads();
  for (int n = t; n < N; n += blockDim.x) {
    const float sc = ssc[n / RB];
    const int en = a.o_ee + ((b * N + n) * 2) * 4;
    if (a.probs) a.probs[(long)b * N + n] = get1(wr, en) * sc;
    if (a.shifted) a.shifted[(long)b * N + n] = get1(wr, en + 4) * sc;
  }
  if (a.wctx && t < D4) {
    const int pb = a.o_part + (b * nblk * a.D + 4 * t) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < nblk; i0 += 8) {   // 8 partial loads in flight (clamped, unconditional)
      float4 pv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) pv[k] = get4(wr, pb + min(i0 + k, nblk - 1) * a.D * 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) fma4(i0 + k < nblk ? ssc[i0 + k] : 0.f, pv[k], acc);
    }
    reinterpret_cast<float4*>(a.wctx + (long)b * a.D)[t] = acc;
  }
}

// ---- whole-row form: one workgroup per batch row, rows streamed ring by ring -----------------------
// No cross-workgroup hand-off at all (each costs several microseconds on MI355X: MI355X_MICROARCH.md
// "handoff-flag", "barrier-counter"): thread t owns float4 column t of every row. The rows come in
// slices of 12 (for the panorama: the three elevation rings), two slices in registers at a time: a
// slice's row dots are reduce-scattered over the wave and meet in LDS, wave 0 turns them into
// exp(s - m) weights against the running max m (and shifts them within the ring: the K-tap
// correlation is linear and never leaves a ring, model.py:337-344), and every thread folds the slice
// into its running context column (online softmax: earlier slices rescaled when m grows). At the end
// the exact softmax / shifted weights are written from the saved scores, and wctx = acc / Z. A
// workgroup streams its 313 KB panorama through one CU: at B = 20 that beats the row-split kernel's
// launch + merge latency, and at B = 256 its 256 workgroups stream at HBM rate.
template <int NS>
__global__ __launch_bounds__(576) void attn_rows_fwd_kernel(FwdArgs a) {
  __shared__ float red[kMaxW][16];
  __shared__ float ssc[12 * NS], swt[12], sw[kMaxK + 1], sscale;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6, W = blockDim.x >> 6;
  const int N = a.N, D4 = a.D >> 2;
  DASA_DCHECK((int)blockDim.x >= D4 && N <= 12 * NS, 128);   // one column per thread, N rows in NS slices
  const bool shift = a.shift_logits != nullptr, col = t < D4;
  const float* rows = a.ctx + (long)b * N * a.ldn;
  float4 xa[12], xb[12];
  float4 qv = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](float4 (&x)[12], int s0) {
    if (col) {
#pragma unroll
      for (int i = 0; i < 12; ++i) x[i] = reinterpret_cast<const float4*>(rows + (long)min(s0 + i, N - 1) * a.ldn)[t];
    }
  };
  load(xa, 0);
  if (NS > 1) load(xb, 12);
  if (col) qv = reinterpret_cast<const float4*>(a.q + (long)b * a.D)[t];
  if (shift && t < 64) shift_taps(a.shift_logits + (long)b * a.K, a.K, sw, lane);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float m_run = -INFINITY, z_run = 0.f;   // wave 0's running max / sum (lane-uniform)
  auto slice = [&](const float4 (&x)[12], int s0) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = (i < 12 && col) ? dot4(x[i], qv) : 0.f;
    const float sum = reduce_scatter16(v, lane);
    const int r = (lane >> 2) & 15;
    if ((lane & 3) == 0 && r < 12) red[w][r] = sum;
    __syncthreads();
    if (t < 64) {
      float sv = -INFINITY;
      if (lane < 12 && s0 + lane < N) {
        float tot = 0.f;
        for (int i = 0; i < W; ++i) tot += red[i][lane];
        ssc[s0 + lane] = tot;
        sv = (a.mask && a.mask[(long)b * N + s0 + lane]) ? -INFINITY : tot;
      }
      const float m_new = fmaxf(m_run, wave_max(sv));
      const float e = sv == -INFINITY ? 0.f : __expf(sv - m_new);
      const float sc = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
      z_run = z_run * sc + wave_sum(e);
      m_run = m_new;
      float we = e;
      if (shift) {   // the ring's shifted weights, exp(s - m_new) scale
        if (lane < 12) swt[lane] = e;
        lds_wave_sync();
        const int P = a.K / 2;
        we = 0.f;
        if (lane < 12)
          for (int k = 0; k < a.K; ++k) {
            int jj = lane + k - P;
            jj = ((jj % 12) + 12) % 12;
            we = fmaf(sw[k], swt[jj], we);
          }
        lds_wave_sync();
      }
      if (lane < 12) swt[lane] = we;
      if (lane == 0) sscale = sc;
    }
    __syncthreads();
    if (col) {
      const float sc = sscale;
      acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc;
#pragma unroll
      for (int i = 0; i < 12; ++i) fma4(swt[i], x[i], acc);
    }
    __syncthreads();   // red / swt are rewritten by the next slice
  };
  // slices s = 0 .. NS-1 alternate between the two register buffers; the buffer a slice has just
  // been folded from is reloaded with slice s + 2 (NS <= 7: N <= 84, the instruction SoftDot's 80 rows)
  slice(xa, 0);
  if (NS > 2) load(xa, 24);
  if (NS > 1) slice(xb, 12);
  if (NS > 3) load(xb, 36);
  if (NS > 2) slice(xa, 24);
  if (NS > 4) load(xa, 48);
  if (NS > 3) slice(xb, 36);
  if (NS > 5) load(xb, 60);
  if (NS > 4) slice(xa, 48);
  if (NS > 6) load(xa, 72);
  if (NS > 5) slice(xb, 60);
  if (NS > 6) slice(xa, 72);
  if (t < 64) {   // the exact softmax / shifted weights from the saved scores
    const float M = m_run, inv = 1.f / z_run;
    if (lane == 0) sscale = inv;
    for (int n = lane; n < N; n += 64) {
      const bool masked = a.mask && a.mask[(long)b * N + n];
      const float p = masked ? 0.f : __expf(ssc[n] - M) * inv;
      if (a.scores) a.scores[(long)b * N + n] = ssc[n];
      if (a.probs) a.probs[(long)b * N + n] = p;
      ssc[n] = p;
    }
    lds_wave_sync();
    if (shift) {
      const int P = a.K / 2;
      for (int n = lane; n < N; n += 64) {
        const int r = n / 12, j = n % 12;
        float wgt = 0.f;
        for (int k = 0; k < a.K; ++k) {
          int jj = j + k - P;
          jj = ((jj % 12) + 12) % 12;
          wgt = fmaf(sw[k], ssc[r * 12 + jj], wgt);
        }
        if (a.shifted) a.shifted[(long)b * N + n] = wgt;
      }
      if (a.wsm && lane < a.K) a.wsm[(long)b * a.K + lane] = sw[lane];
    }
  }
  __syncthreads();
  if (a.wctx && col) {
    const float inv = sscale;
    reinterpret_cast<float4*>(a.wctx + (long)b * a.D)[t] = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
  }
}

struct BwdArgs {
  const float* q; const float* ctx; long ldn;
  const float* probs;     // softmax a [B][N]
  const float* shifted;   // a' [B][N] (shift only)
  const float* wsm;       // w [B][K] (shift only)
  int K;
  const float* dwctx;     // [B][D] or NULL
  const float* dscores;   // [B][N] or NULL
  float* dq; float* dctx; int accumulate;
  float* dshift;          // [B][K] (shift only)
  int N, D, nblk;
  unsigned* cnt1; unsigned* cnt2; float* ds; float* pw;   // workspace (ds / pw: read by the next launch)
  float* ws; int o_dp, o_part;                            // byte offsets of the in-launch partials
};

// Launch 1: dp = ctx . dwctx per row block; the last arriver does the softmax / shift backward.
template <int RB>
__global__ __launch_bounds__(1024) void attn_bwd_dp_kernel(BwdArgs a) {
  __shared__ float red[kMaxW][16];
  __shared__ float sdp[kMaxN], sda[kMaxN], sp[kMaxN], swt[kMaxK + 1];
  __shared__ int s_flag;
  const int j = blockIdx.x, b = blockIdx.y, t = threadIdx.x, lane = t & 63;
  const int N = a.N, D4 = a.D >> 2, r0 = j * RB, nr = min(RB, N - r0);
  const float* rows = a.ctx + ((long)b * N + r0) * a.ldn;
  float4 x[RB];
  const float s = block_row_dots<RB>(rows, a.ldn, nr, a.dwctx + (long)b * a.D, D4, x, red);
  const __amdgpu_buffer_rsrc_t wr = ws_rsrc(a.ws);
  if (t < 64 && lane < nr) pub1(wr, a.o_dp + (b * N + r0 + lane) * 4, s);
  if (!last_arriver(a.cnt1 + b, a.nblk, &s_flag)) return;
  if (t >= 64) return;
  // stage dp, the softmax and the taps in LDS (every load issued before any is used: the loops below
  // would otherwise wait out one global round trip per element)
  for (int n = lane; n < N; n += 64) {
    sdp[n] = get1(wr, a.o_dp + (b * N + n) * 4);
    sp[n] = a.probs[(long)b * N + n];
  }
  if (a.wsm && lane < a.K) swt[lane] = a.wsm[(long)b * a.K + lane];
  lds_wave_sync();
  const float* p = sp;
  if (a.wsm) {
    // da[v] = sum_k w_k dp'[r][(i - k + P) mod 12] (transpose of the forward correlation);
    // dw[k] = sum_v dp'[v] a[r][(j + k - P) mod 12]; softmax backward over the K taps.
    const float* w = swt;
    const int P = a.K / 2;
    for (int v = lane; v < N; v += 64) {
      const int r = v / 12, i = v % 12;
      float acc = 0.f;
      for (int k = 0; k < a.K; ++k) {
        int jj = i - k + P;
        jj = ((jj % 12) + 12) % 12;
        acc = fmaf(w[k], sdp[r * 12 + jj], acc);
      }
      sda[v] = acc;
      a.pw[(long)b * N + v] = a.shifted[(long)b * N + v];
    }
    float dwk = 0.f;
    if (lane < a.K) {
      for (int v = 0; v < N; ++v) {
        const int r = v / 12, jx = v % 12;
        int jj = jx + lane - P;
        jj = ((jj % 12) + 12) % 12;
        dwk = fmaf(sdp[v], p[r * 12 + jj], dwk);
      }
    }
    const float wk = lane < a.K ? w[lane] : 0.f;
    const float dot = wave_sum(wk * dwk);
    if (lane < a.K) a.dshift[(long)b * a.K + lane] = wk * (dwk - dot);
  } else {
    for (int v = lane; v < N; v += 64) {
      sda[v] = sdp[v];
      a.pw[(long)b * N + v] = p[v];
    }
  }
  lds_wave_sync();
  float dot = 0.f;
  for (int v = lane; v < N; v += 64) dot = fmaf(p[v], sda[v], dot);
  dot = wave_sum(dot);
  for (int v = lane; v < N; v += 64) {
    float g = p[v] * (sda[v] - dot);
    if (a.dscores) g += a.dscores[(long)b * N + v];
    a.ds[(long)b * N + v] = g;
  }
}

// Launch 2: dctx rows (+)= pw dwctx + ds q and a partial dq = sum_r ds_r ctx_r per row block; the
// last arriver sums the partials. ds / pw come from launch 1 (or ds = dscores, pw unused, when the
// caller has no dwctx: the candidate-logit backward).
template <int RB>
__global__ __launch_bounds__(1024) void attn_bwd_apply_kernel(BwdArgs a) {
  __shared__ float sds[16], spw[16];
  __shared__ int s_flag;
  const int j = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int N = a.N, D4 = a.D >> 2, r0 = j * RB, nr = min(RB, N - r0), nblk = a.nblk;
  const float* rows = a.ctx + ((long)b * N + r0) * a.ldn;
  const bool gdw = a.dwctx != nullptr;
  if (t < RB) {
    const int n = r0 + min(t, nr - 1);
    const float* dsp = gdw ? a.ds : a.dscores;
    sds[t] = t < nr ? dsp[(long)b * N + n] : 0.f;
    spw[t] = (t < nr && gdw) ? a.pw[(long)b * N + n] : 0.f;
  }
  __syncthreads();
  float* drows = a.dctx ? a.dctx + ((long)b * N + r0) * a.ldn : nullptr;
  const __amdgpu_buffer_rsrc_t wr = ws_rsrc(a.ws);
  if (t < D4) {
    const int c = t;
    float4 x[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) x[i] = reinterpret_cast<const float4*>(rows + (long)min(i, nr - 1) * a.ldn)[c];
    const float4 qv = reinterpret_cast<const float4*>(a.q + (long)b * a.D)[c];
    const float4 gv = gdw ? reinterpret_cast<const float4*>(a.dwctx + (long)b * a.D)[c]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < RB; ++i) fma4(sds[i], x[i], acc);
    if (drows) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (i < nr) {
          float4* d4 = reinterpret_cast<float4*>(drows + (long)i * a.ldn) + c;
          float4 g;
          g.x = fmaf(spw[i], gv.x, sds[i] * qv.x);
          g.y = fmaf(spw[i], gv.y, sds[i] * qv.y);
          g.z = fmaf(spw[i], gv.z, sds[i] * qv.z);
          g.w = fmaf(spw[i], gv.w, sds[i] * qv.w);
          if (a.accumulate) {
            const float4 o = *d4;
            g.x += o.x; g.y += o.y; g.z += o.z; g.w += o.w;
          }
          *d4 = g;
        }
      }
    }
    if (a.dq) {
      if (nblk == 1) reinterpret_cast<float4*>(a.dq + (long)b * a.D)[c] = acc;
      else pub4(wr, a.o_part + ((b * nblk + j) * a.D + 4 * c) * 4, acc);
    }
  }
  if (nblk == 1 || !a.dq) return;
  if (!last_arriver(a.cnt2 + b, nblk, &s_flag)) return;
  if (t < D4) {
    const int pb = a.o_part + (b * nblk * a.D + 4 * t) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < nblk; i0 += 8) {   // 8 partial loads in flight (clamped, unconditional)
      float4 pv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) pv[k] = get4(wr, pb + min(i0 + k, nblk - 1) * a.D * 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) fma4(i0 + k < nblk ? 1.f : 0.f, pv[k], acc);
    }
    reinterpret_cast<float4*>(a.dq + (long)b * a.D)[t] = acc;
  }
}

// ---- D-split backward (small batches: the decision step at B = 20) --------------------------------
// The row-split backward gives a batch row ceil(N / RB) workgroups (60 / 100 / 20 at B = 20) and two
// launches. Here a batch row gets G = D / 128 workgroups instead (17 for D = 2176, 16 for 2048), each
// owning a 128-float column chunk of ALL N rows (N <= 80): thread (row lane rl = t / 32, column t % 32)
// holds rows rl, rl + 8, ... of its float4 column in registers. One launch: partial dp = ctx . dwctx
// over the chunk, published write-through; the G workgroups meet at a group barrier (bounded spin on an
// agent-scope counter); every workgroup sums the G partials in the same order, forms ds / the shift
// backward for the N rows, then writes its chunk of dctx and of dq directly (no dq partial merge).
// Without dwctx (candidate logits) there is no barrier. (The forward takes the whole-row form above:
// a cross-workgroup hand-off costs more than streaming the whole row through one CU.)
// Co-residency: the spin form is used only while B x G <= kSplitMaxWG (4 small workgroups per CU);
// workgroups are dispatched in order, so a group whose first member runs is completed by workgroups
// that are either running or next in line. A wait that exceeds kAttnSpinTicks anyway NaN-poisons the
// workgroup's outputs and sets bit 4 of the library error word (raised by ops.check_device_errors).
constexpr int kCW = 32;                          // float4 columns per workgroup
constexpr int kSplitMaxN = 80;
constexpr long kSplitMaxWG = 1024;
constexpr long long kAttnSpinTicks = 20000000;   // 200 ms of the 100 MHz wall clock
constexpr unsigned kErrAttnBarrier = 4u;

struct SplitArgs {
  const float* q; const float* ctx; long ldn;
  const uint8_t* mask;                            // fwd [B][N] or NULL
  const float* shift_logits; int K;               // fwd, shift attention
  float* scores; float* probs; float* shifted; float* wsm; float* wctx;   // fwd outputs (each optional)
  const float* a_probs; const float* a_shifted; const float* a_wsm;       // bwd: saved forward values
  const float* dwctx; const float* dscores;       // bwd inputs (either may be NULL, not both)
  float* dq; float* dctx; int accumulate; float* dshift;                  // bwd outputs
  int N, D, G;
  unsigned* cnt; unsigned* bar; float* ws; int o_part;   // workspace: last-arriver / barrier counters, partials
  unsigned* err; int force;
};

// The G workgroups of batch row b meet on a monotonic counter (one per (G, b), never reset): every
// launch adds exactly G arrivals, so an arrival's ticket tk says which launch it belongs to and the
// wait ends at (tk / G + 1) * G. One atomic round trip plus the poll; no departure count, and a
// timed-out workgroup still arrives, so the counters stay consistent. False on timeout (error word).
__device__ bool group_barrier(unsigned* cnt, int G, unsigned* err, int force, int* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its write-through stores landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (tk / (unsigned)G + 1u) * (unsigned)G;
    int ok = force ? 0 : 1;
    const long long t0 = wall_clock64();
    while (ok && (int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > kAttnSpinTicks) ok = 0;
    }
    if (!ok && err) __hip_atomic_fetch_or(err, kErrAttnBarrier, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_ok = ok;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep the sc1 loads below
  return *s_ok != 0;
}

// Row dots of the thread's RPT rows with vec over its float4 column, summed over the 32 columns of the
// half-wave: lane col == 0 ends with the chunk's partial dot of row rl + 8 i in v[i].
template <int RPT>
__device__ __forceinline__ void chunk_row_dots(const float4 (&x)[RPT], float4 vec, float (&v)[RPT]) {
#pragma unroll
  for (int i = 0; i < RPT; ++i) v[i] = dot4(x[i], vec);
#pragma unroll
  for (int o = 16; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < RPT; ++i) v[i] += __shfl_xor(v[i], o, 64);
}

// The G x N published partials of a batch row into LDS spart[g * N + n]: every load is issued before
// the first is used (clamped, unconditional addresses: a guarded load would make the compiler wait for
// each one in turn — a dependent round trip per partial), then the caller sums them in LDS.
constexpr int kMaxPartPerThread = 10;   // G * N <= 32 * 80 over 256 threads
__device__ __forceinline__ void gather_partials(__amdgpu_buffer_rsrc_t wr, int pbase, int GN, float* spart) {
  const int t = threadIdx.x;
  float tmp[kMaxPartPerThread];
#pragma unroll
  for (int k = 0; k < kMaxPartPerThread; ++k) tmp[k] = get1(wr, pbase + min(t + 256 * k, GN - 1) * 4);
#pragma unroll
  for (int k = 0; k < kMaxPartPerThread; ++k)
    if (t + 256 * k < GN) spart[t + 256 * k] = tmp[k];
  __syncthreads();
}

// Sum over the 8 row lanes of the per-thread float4 (LDS), returned on threads t < 32 (column t).
__device__ __forceinline__ float4 rowlane_sum(float4 acc, float4 (*red4)[kCW]) {
  const int t = threadIdx.x;
  red4[t >> 5][t & 31] = acc;
  __syncthreads();
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < kCW) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 p = red4[i][t];
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
  }
  return s;
}

template <int RPT>
__global__ __launch_bounds__(256) void attn_split_bwd_kernel(SplitArgs a) {
  __shared__ float4 red4[8][kCW];
  __shared__ float spart[256 * kMaxPartPerThread];
  __shared__ float sdp[kSplitMaxN], sds[kSplitMaxN], spw[kSplitMaxN], sp[kSplitMaxN], swk[kMaxK + 1];
  __shared__ int s_flag;
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x, lane = t & 63, col = t & 31, rl = t >> 5;
  const int N = a.N, G = a.G, c = g * kCW + col;
  const float* base = a.ctx + (long)b * N * a.ldn;
  float4 x[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) x[i] = reinterpret_cast<const float4*>(base + (long)min(rl + 8 * i, N - 1) * a.ldn)[c];
  const float4 qv = reinterpret_cast<const float4*>(a.q + (long)b * a.D)[c];
  const bool gdw = a.dwctx != nullptr;
  const float4 gv = gdw ? reinterpret_cast<const float4*>(a.dwctx + (long)b * a.D)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  if (gdw) {
    float v[RPT];
    chunk_row_dots<RPT>(x, gv, v);
    const __amdgpu_buffer_rsrc_t wr = ws_rsrc(a.ws);
    const int pbase = a.o_part + (int)((long)b * G * N) * 4;
    if (col == 0) {
#pragma unroll
      for (int i = 0; i < RPT; ++i)
        if (rl + 8 * i < N) pub1(wr, pbase + (g * N + rl + 8 * i) * 4, v[i]);
    }
    if (!group_barrier(a.bar + b, G, a.err, a.force, &s_flag)) {
      const float qnan = __builtin_nanf("");
      const float4 q4 = make_float4(qnan, qnan, qnan, qnan);
      if (t < kCW && a.dq) reinterpret_cast<float4*>(a.dq + (long)b * a.D)[g * kCW + t] = q4;
      if (a.dctx)
#pragma unroll
        for (int i = 0; i < RPT; ++i)
          if (rl + 8 * i < N) reinterpret_cast<float4*>(a.dctx + ((long)b * N + rl + 8 * i) * a.ldn)[c] = q4;
      return;
    }
    gather_partials(wr, pbase, G * N, spart);
    if (t < N) {
      float s = 0.f;
      for (int gg = 0; gg < G; ++gg) s += spart[gg * N + t];
      sdp[t] = s;
      sp[t] = a.a_probs[(long)b * N + t];
      if (a.a_shifted) spw[t] = a.a_shifted[(long)b * N + t];
    }
    if (a.a_wsm && t < a.K) swk[t] = a.a_wsm[(long)b * a.K + t];
    __syncthreads();
    if (t < 64) {
      const float* p = sp;
      float da0 = 0.f, da1 = 0.f;
      if (a.a_wsm) {   // shift backward (transpose of the forward correlation; softmax over the taps)
        const float* w = swk;
        const int P = a.K / 2;
        if (lane < N) {
          const int r = lane / 12, i = lane % 12;
          for (int k = 0; k < a.K; ++k) {
            int jj = i - k + P;
            jj = ((jj % 12) + 12) % 12;
            da0 = fmaf(w[k], sdp[r * 12 + jj], da0);
          }
        }
        float dwk = 0.f;
        if (lane < a.K) {
          for (int vv = 0; vv < N; ++vv) {
            const int r = vv / 12, jx = vv % 12;
            int jj = jx + lane - P;
            jj = ((jj % 12) + 12) % 12;
            dwk = fmaf(sdp[vv], p[r * 12 + jj], dwk);
          }
        }
        const float wk = lane < a.K ? w[lane] : 0.f;
        const float dot = wave_sum(wk * dwk);
        if (g == 0 && lane < a.K && a.dshift) a.dshift[(long)b * a.K + lane] = wk * (dwk - dot);
      } else {
        if (lane < N) { da0 = sdp[lane]; spw[lane] = p[lane]; }
        if (lane + 64 < N) { da1 = sdp[lane + 64]; spw[lane + 64] = p[lane + 64]; }
      }
      const float p0 = lane < N ? p[lane] : 0.f, p1 = lane + 64 < N ? p[lane + 64] : 0.f;
      const float dot = wave_sum(p0 * da0 + p1 * da1);
      if (lane < N) sds[lane] = p0 * (da0 - dot) + (a.dscores ? a.dscores[(long)b * N + lane] : 0.f);
      if (lane + 64 < N) sds[lane + 64] = p1 * (da1 - dot) + (a.dscores ? a.dscores[(long)b * N + lane + 64] : 0.f);
    }
  } else {
    if (t < N) {
      sds[t] = a.dscores[(long)b * N + t];
      spw[t] = 0.f;
    }
  }
  __syncthreads();
  if (a.dctx) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = rl + 8 * i;
      if (r < N) {
        float4* d4 = reinterpret_cast<float4*>(a.dctx + ((long)b * N + r) * a.ldn) + c;
        const float pw = spw[r], ds = sds[r];
        float4 o;
        o.x = fmaf(pw, gv.x, ds * qv.x);
        o.y = fmaf(pw, gv.y, ds * qv.y);
        o.z = fmaf(pw, gv.z, ds * qv.z);
        o.w = fmaf(pw, gv.w, ds * qv.w);
        if (a.accumulate) {
          const float4 old = *d4;
          o.x += old.x; o.y += old.y; o.z += old.z; o.w += old.w;
        }
        *d4 = o;
      }
    }
  }
  if (!a.dq) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = rl + 8 * i;
    fma4(r < N ? sds[r] : 0.f, x[i], acc);
  }
  const float4 o = rowlane_sum(acc, red4);
  if (t < kCW) reinterpret_cast<float4*>(a.dq + (long)b * a.D)[g * kCW + t] = o;
}

// ---- two-launch D-split forward (small batches: the decision step at B = 20) ------------------------
// A cross-workgroup hand-off inside one launch costs 3-5 us on MI355X (MI355X_MICROARCH.md price table,
// "handoff-flag", "fanin"); a dependent kernel boundary 1.5-1.9 us ("boundary"). So the forward splits
// the row dots from the softmax at a launch boundary instead of a group barrier, and both launches put
// B x G workgroups (G = D / 128: 340 for the panorama at B = 20) on the chip, each holding a 128-float
// column chunk of all N rows (thread: row lane rl = t / 32, float4 column t % 32, rows rl + 8 i).
//   launch 1  partial row dots over the chunk -> part[b][g][n] (plain stores; the boundary publishes)
//   launch 2  the chunk's rows re-read (L2 / MALL: launch 1 just streamed them) with their loads issued
//             BEFORE the G x N partial loads, so the two round trips overlap; the G partials of each row
//             summed in fixed order g = 0..G-1 (every workgroup of b gets bitwise the same scores),
//             masked softmax, the ring shift, and the chunk of wctx = sum_n w_n ctx_n; workgroup g = 0
//             also writes scores / probs / shifted / the tap weights.
// Measured (profiles/r03/attn_forms_b.txt, B = 20): shift attention 8.55 us vs 8.89 for the row-split
// kernel's in-launch merge, so the shift forward takes it; the instruction SoftDot (N = 80) ran 12.1 vs
// 10.8 us on it and stays there (r04 moved it here while the row-split kernel was not reproducible beside
// bf16x6 form-20 GEMMs; r05 found and removed the cause: dasa_softdot_fwd).
template <int RPT>
__global__ __launch_bounds__(256) void attn_split_dots_kernel(SplitArgs a) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x, col = t & 31, rl = t >> 5;
  const int N = a.N, c = g * kCW + col;
  const float* base = a.ctx + (long)b * N * a.ldn;
  float4 x[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) x[i] = reinterpret_cast<const float4*>(base + (long)min(rl + 8 * i, N - 1) * a.ldn)[c];
  const float4 qv = reinterpret_cast<const float4*>(a.q + (long)b * a.D)[c];
  float v[RPT];
  chunk_row_dots<RPT>(x, qv, v);
  if (col == 0) {
    float* part = a.ws + (a.o_part >> 2) + ((long)b * a.G + g) * N;
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      if (rl + 8 * i < N) part[rl + 8 * i] = v[i];
  }
}

template <int RPT>
__global__ __launch_bounds__(256) void attn_split_ctx_kernel(SplitArgs a) {
  __shared__ float4 red4[8][kCW];
  __shared__ float spart[256 * kMaxPartPerThread];
  __shared__ float ssc[kSplitMaxN], sw[kSplitMaxN], swk[kMaxK + 1];
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x, lane = t & 63, col = t & 31, rl = t >> 5;
  const int N = a.N, G = a.G, c = g * kCW + col;
  const bool shift = a.shift_logits != nullptr;
  const float* base = a.ctx + (long)b * N * a.ldn;
  float4 x[RPT];
  if (a.wctx) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) x[i] = reinterpret_cast<const float4*>(base + (long)min(rl + 8 * i, N - 1) * a.ldn)[c];
  }
  gather_partials(ws_rsrc(a.ws), a.o_part + (int)((long)b * G * N) * 4, G * N, spart);
  if (t < 64) {
    float s0 = 0.f, s1 = 0.f;
    for (int gg = 0; gg < G; ++gg) {   // fixed order: the same scores in all G workgroups of b
      if (lane < N) s0 += spart[gg * N + lane];
      if (lane + 64 < N) s1 += spart[gg * N + lane + 64];
    }
    const bool v0 = lane < N, v1 = lane + 64 < N;
    const bool m0 = v0 && a.mask && a.mask[(long)b * N + lane], m1 = v1 && a.mask && a.mask[(long)b * N + lane + 64];
    const float z0 = (v0 && !m0) ? s0 : -INFINITY, z1 = (v1 && !m1) ? s1 : -INFINITY;
    const float M = wave_max(fmaxf(z0, z1));
    const float e0 = z0 == -INFINITY ? 0.f : __expf(z0 - M), e1 = z1 == -INFINITY ? 0.f : __expf(z1 - M);
    const float inv = 1.f / wave_sum(e0 + e1);
    const float p0 = e0 * inv, p1 = e1 * inv;
    if (v0) ssc[lane] = p0;
    if (v1) ssc[lane + 64] = p1;
    if (g == 0) {
      if (v0 && a.scores) a.scores[(long)b * N + lane] = s0;
      if (v1 && a.scores) a.scores[(long)b * N + lane + 64] = s1;
      if (v0 && a.probs) a.probs[(long)b * N + lane] = p0;
      if (v1 && a.probs) a.probs[(long)b * N + lane + 64] = p1;
    }
    if (shift) {   // N = 36: three rings of 12, the K-tap circular correlation within each (model.py:337-344)
      shift_taps(a.shift_logits + (long)b * a.K, a.K, swk, lane);
      lds_wave_sync();
      const int P = a.K / 2;
      float wgt = 0.f;
      if (v0) {
        const int r = lane / 12, j = lane % 12;
        for (int k = 0; k < a.K; ++k) {
          int jj = j + k - P;
          jj = ((jj % 12) + 12) % 12;
          wgt = fmaf(swk[k], ssc[r * 12 + jj], wgt);
        }
        sw[lane] = wgt;
      }
      if (g == 0) {
        if (v0 && a.shifted) a.shifted[(long)b * N + lane] = wgt;
        if (a.wsm && lane < a.K) a.wsm[(long)b * a.K + lane] = swk[lane];
      }
    } else {
      if (v0) sw[lane] = p0;
      if (v1) sw[lane + 64] = p1;
    }
  }
  if (!a.wctx) return;   // uniform: no workgroup reaches the barrier below
  __syncthreads();
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = rl + 8 * i;
    fma4(r < N ? sw[r] : 0.f, x[i], acc);
  }
  const float4 o = rowlane_sum(acc, red4);
  if (t < kCW) reinterpret_cast<float4*>(a.wctx + (long)b * a.D)[g * kCW + t] = o;
}

// Scores only (the candidate logits, model.py:276-280): one workgroup per (row, batch row), the row's
// float4 loads all in flight at once, a block reduction, no hand-off of any kind. B < 128 only: 2.5 vs
// 3.9 us at B = 20, but 9.4 vs 6.9 us at B = 256 (profiles/r03/attn_forms_b.txt).
__global__ __launch_bounds__(256) void attn_dot_rows_kernel(const float* __restrict__ q, const float* __restrict__ ctx,
                                                            long ldn, float* __restrict__ scores, int N, int D) {
  __shared__ float red[4];
  const int n = blockIdx.x, b = blockIdx.y, t = threadIdx.x, D4 = D >> 2;
  const float4* row = reinterpret_cast<const float4*>(ctx + ((long)b * N + n) * ldn);
  const float4* qv = reinterpret_cast<const float4*>(q + (long)b * D);
  float4 x[4], y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = min(t + 256 * i, D4 - 1);
    x[i] = row[k];
    y[i] = qv[k];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (t + 256 * i < D4) s += dot4(x[i], y[i]);
  s = block_sum<4>(s, red);
  if (t == 0) scores[(long)b * N + n] = s;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

inline int block_threads(int D) {
  const int D4 = D >> 2;
  int T = ((D4 + 63) / 64) * 64;
  return T > 1024 ? 1024 : (T < 64 ? 64 : T);
}

inline int rows_per_block(int N, bool shift) { return shift ? 12 : 16; }

// Workspace layout (32-bit words): [cnt1 kMaxB][cnt2 kMaxB] at fixed offsets (so the zero-on-entry
// counters never overlap another call's data, whatever its shape), the D-split group-barrier counters
// [kBarSlots][kSplitMaxWG] (monotonic, slot = G), then [dp B*N][ds B*N][pw B*N][ml B*nblk*2]
// [ee B*N*2][part B*nblk*D], the partial blocks 16-B aligned.
constexpr long kMaxB = 32768;
constexpr long kBarSlots = 33;   // G = D / 128 <= 32
struct WsLayout {
  unsigned* cnt1; unsigned* cnt2; unsigned* bar; float* ds; float* pw;
  int o_dp, o_ml, o_ee, o_part;   // byte offsets from the workspace base
  int64_t bytes;
};

inline WsLayout ws_layout(void* ws, int B, int N, int D) {
  const long nblk = (N + 11) / 12;   // the larger block count of the two row splits
  long off = 0;
  auto take = [&](long n) { long o = off; off += (n + 3) & ~3L; return o; };
  const long o1 = take(kMaxB), o2 = take(kMaxB), ob = take(kBarSlots * kSplitMaxWG), o3 = take((long)B * N),
             o4 = take((long)B * N), o5 = take((long)B * N), o6 = take((long)B * nblk * 2), o7 = take((long)B * N * 2),
             o8 = take((long)B * nblk * D);
  // pointers only into a real buffer (a size query passes ws = nullptr: no arithmetic on a null pointer)
  float* f = (float*)ws;
  auto at = [&](long o) { return f ? f + o : nullptr; };
  WsLayout L{(unsigned*)at(o1), (unsigned*)at(o2), (unsigned*)at(ob), at(o4), at(o5), (int)(o3 * 4),
             (int)(o6 * 4), (int)(o7 * 4), (int)(o8 * 4), (int64_t)off * 4};
  return L;
}

int g_attn_mode = -1;   // dasa_attn_set_mode: 0 automatic, 1 row-split only, 2 = 0 + the two-launch
                        // D-split forward for SoftDot too (tests); -1 = not read from the env yet
float* g_attn_dbg = nullptr;   // dasa_attn_debug_buffer: the next row-split forward dumps here
int64_t g_attn_dbg_bytes = 0;

template <int RB>
int launch_fwd(FwdArgs a, int B, void* ws, hipStream_t st) {
  a.nblk = (a.N + RB - 1) / RB;
  WsLayout L = ws_layout(ws, B, a.N, a.D);
  a.cnt = L.cnt1; a.ws = (float*)ws; a.o_part = L.o_part; a.o_ml = L.o_ml; a.o_ee = L.o_ee;
  const dim3 grid(a.nblk, B), block(block_threads(a.D));
  const bool leg = g_attn_mode == 3;   // diagnosis: the r04 per-row-address loads
  if (g_attn_dbg && (int64_t)a.nblk * B * kDbgRec * 4 <= g_attn_dbg_bytes) {
    a.dbg = g_attn_dbg;
    g_attn_dbg = nullptr;   // one launch per armed buffer
    if (leg) hipLaunchKernelGGL((attn_fwd_kernel<RB, true, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<RB, true>), grid, block, 0, st, a);
  } else {
    if (leg) hipLaunchKernelGGL((attn_fwd_kernel<RB, false, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL(attn_fwd_kernel<RB>, grid, block, 0, st, a);
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

template <int RB>
int launch_bwd(BwdArgs a, int B, void* ws, hipStream_t st) {
  a.nblk = (a.N + RB - 1) / RB;
  WsLayout L = ws_layout(ws, B, a.N, a.D);
  a.cnt1 = L.cnt1; a.cnt2 = L.cnt2; a.ds = L.ds; a.pw = L.pw; a.ws = (float*)ws; a.o_dp = L.o_dp;
  a.o_part = L.o_part;
  const dim3 grid(a.nblk, B), block(block_threads(a.D));
  if (a.dwctx) {
    hipLaunchKernelGGL(attn_bwd_dp_kernel<RB>, grid, block, 0, st, a);
    DASA_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(attn_bwd_apply_kernel<RB>, grid, block, 0, st, a);
  DASA_CHECK_LAUNCH();
  return 0;
}

// D-split eligibility (0 = use the row-split kernels): rows per thread for N <= 80, D a multiple of 128,
// and B x G within kSplitMaxWG when the call needs the group barrier. DASA_ATTN_SPLIT=0 disables it.

int split_rpt(int B, int N, int D, bool spin) {
  if (g_attn_mode < 0) {
    const char* e = getenv("DASA_ATTN_SPLIT");
    g_attn_mode = (e && e[0] == '0') ? 1 : 0;
  }
  if (g_attn_mode == 1 || g_attn_mode == 3 || N < 1 || N > kSplitMaxN || D % (4 * kCW) != 0) return 0;
  if (spin && (long)B * (D / (4 * kCW)) > kSplitMaxWG) return 0;
  return N <= 16 ? 2 : (N <= 40 ? 5 : 10);
}

template <int RPT>
void split_launch(const SplitArgs& a, int B, hipStream_t st) {
  hipLaunchKernelGGL(attn_split_bwd_kernel<RPT>, dim3(a.G, B), dim3(256), 0, st, a);
}

// Whole-row forward: N <= 36 rows, D4 = D / 4 <= 576 columns (one per thread), mode 0, and at least
// 128 batch rows. One CU streams a row at ~35-40 GB/s (the loads one CU keeps in flight), so the form
// pays at large B — B = 256: shift 0.44 -> 0.57 of HBM peak — and loses at B = 20, where the row-split
// kernel's 60 workgroups win despite their merge (9.2 vs 10.6 us; profiles/r03/attn_forms.txt).
constexpr int kRowsMinB = 128;
bool rows_ok(int B, int N, int D, bool shift = true) {
  if (g_attn_mode < 0) split_rpt(1, 1, 128, false);   // reads DASA_ATTN_SPLIT once
  // the shift attention's rings need N <= 36; SoftDot takes up to seven 12-row slices (N <= 84)
  return g_attn_mode != 1 && g_attn_mode != 3 && B >= kRowsMinB && N >= 1 && N <= (shift ? 36 : 84) && D <= 4 * 576;
}

int launch_rows(const FwdArgs& a, int B, hipStream_t st) {
  const int ns = (a.N + 11) / 12;
  const dim3 grid(B), block(block_threads(a.D));
  switch (ns) {
    case 1: hipLaunchKernelGGL(attn_rows_fwd_kernel<1>, grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL(attn_rows_fwd_kernel<2>, grid, block, 0, st, a); break;
    case 3: hipLaunchKernelGGL(attn_rows_fwd_kernel<3>, grid, block, 0, st, a); break;
    case 4: hipLaunchKernelGGL(attn_rows_fwd_kernel<4>, grid, block, 0, st, a); break;
    case 5: hipLaunchKernelGGL(attn_rows_fwd_kernel<5>, grid, block, 0, st, a); break;
    case 6: hipLaunchKernelGGL(attn_rows_fwd_kernel<6>, grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL(attn_rows_fwd_kernel<7>, grid, block, 0, st, a); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

int launch_split_bwd(SplitArgs a, int rpt, int B, void* ws, hipStream_t st) {
  WsLayout L = ws_layout(ws, B, a.N, a.D);
  a.G = a.D / (4 * kCW);
  a.cnt = L.cnt1; a.bar = L.bar + (long)a.G * kSplitMaxWG; a.ws = (float*)ws; a.o_part = L.o_part;
  a.err = dasa_err_word_host(); a.force = dasa_force_timeout_host();
  switch (rpt) {
    case 2: split_launch<2>(a, B, st); break;
    case 5: split_launch<5>(a, B, st); break;
    default: split_launch<10>(a, B, st); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

// Two-launch D-split forward: mode 0, fewer than kRowsMinB batch rows (the whole-row form takes the large
// batches), N <= 80, D a multiple of 128 (G <= 32 chunks).
bool split2_ok(int B, int N, int D) {
  if (g_attn_mode < 0) split_rpt(1, 1, 128, false);
  return g_attn_mode != 1 && g_attn_mode != 3 && B < kRowsMinB && N >= 1 && N <= kSplitMaxN && D % (4 * kCW) == 0 &&
         D <= 4 * kCW * 32;
}

template <int RPT>
void split2_launch(const SplitArgs& a, int B, hipStream_t st) {
  hipLaunchKernelGGL(attn_split_dots_kernel<RPT>, dim3(a.G, B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_split_ctx_kernel<RPT>, dim3(a.G, B), dim3(256), 0, st, a);
}

int launch_split2_fwd(const FwdArgs& f, int B, void* ws, hipStream_t st) {
  WsLayout L = ws_layout(ws, B, f.N, f.D);
  SplitArgs a{};
  a.q = f.q; a.ctx = f.ctx; a.ldn = f.ldn; a.mask = f.mask; a.shift_logits = f.shift_logits; a.K = f.K;
  a.scores = f.scores; a.probs = f.probs; a.shifted = f.shifted; a.wsm = f.wsm; a.wctx = f.wctx;
  a.N = f.N; a.D = f.D; a.G = f.D / (4 * kCW); a.ws = (float*)ws; a.o_part = L.o_part;
  const int rpt = f.N <= 16 ? 2 : (f.N <= 40 ? 5 : 10);
  switch (rpt) {
    case 2: split2_launch<2>(a, B, st); break;
    case 5: split2_launch<5>(a, B, st); break;
    default: split2_launch<10>(a, B, st); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

bool bad_common(const float* q, const float* ctx, int64_t ldn, int B, int N, int D, const void* ws) {
  return N > kMaxN || D > 4096 || B > kMaxB || ws_layout(nullptr, B, N, D).bytes >= (1L << 31) || (D & 3) || (ldn & 3) || ldn < D || !aligned16(q) || !aligned16(ctx) || !ws ||
         !aligned16(ws);
}

}  // namespace

extern "C" int dasa_attn_set_mode(int32_t mode) {
  if (mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  g_attn_mode = mode;
  return 0;
}

extern "C" int dasa_attn_debug_buffer(float* buf, int64_t bytes) {
  if (buf && (bytes < (int64_t)kDbgRec * 4 || ((uintptr_t)buf & 15))) return (int)hipErrorInvalidValue;
  g_attn_dbg = buf;
  g_attn_dbg_bytes = buf ? bytes : 0;
  return 0;
}

extern "C" int64_t dasa_attn_debug_record_floats() { return kDbgRec; }

extern "C" int64_t dasa_attn_workspace(int32_t B, int32_t N, int32_t D) {
  if (B <= 0 || N <= 0 || D <= 0) return 16;
  return ws_layout(nullptr, B, N, D).bytes;
}

extern "C" int dasa_softdot_fwd(const float* q, const float* ctx, int64_t ldn, const uint8_t* mask,
                                float* scores, float* probs, float* wctx,
                                int32_t B, int32_t N, int32_t D, float* ws, void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (bad_common(q, ctx, ldn, B, N, D, ws) || (wctx && !aligned16(wctx))) return (int)hipErrorInvalidValue;
  FwdArgs a{q, ctx, (long)ldn, mask, nullptr, 0, scores, probs, nullptr, nullptr, wctx, N, D};
  if (g_attn_mode < 0) split_rpt(1, 1, 128, false);   // reads DASA_ATTN_SPLIT once
  if ((probs || wctx) && rows_ok(B, N, D, false)) return launch_rows(a, B, (hipStream_t)stream);
  if (!probs && !wctx && scores && g_attn_mode != 1 && g_attn_mode != 3 && D <= 4 * 1024) {   // scores only (every B: see below)
    hipLaunchKernelGGL(attn_dot_rows_kernel, dim3(N, B), dim3(256), 0, (hipStream_t)stream, q, ctx, (long)ldn,
                       scores, N, D);
    DASA_CHECK_LAUNCH();
    return 0;
  }
  // Every B the whole-row form does not take: the row-split kernel (1.2-1.3 us faster per call than the
  // two-launch D-split form at B = 20, profiles/r03/attn_forms_b.txt); mode 2 takes the D-split form. r04
  // routed SoftDot away from the row-split kernel because it returned wrong row dots beside starting bf16x6
  // form-20 GEMMs; r05 found the cause — packed-FP32 VALU results (the compiler's v_pk_fma_f32 row pairs)
  // corrupted on lanes 48-63 beside a starting MFMA-dense workgroup — and builds every kernel without packed
  // FP32 (dasa_amd/build.py), after which the kernel is bitwise reproducible under the same stress
  // (profiles/r05/rowsplit_diag_c_noslp_m1.log, stress_c_noslp_all_mode1.log).
  if (g_attn_mode == 2 && N <= kSplitMaxN && D % (4 * kCW) == 0 && D <= 4 * kCW * 32)
    return launch_split2_fwd(a, B, ws, (hipStream_t)stream);
  return launch_fwd<16>(a, B, ws, (hipStream_t)stream);
}

extern "C" int dasa_softdot_bwd(const float* q, const float* ctx, int64_t ldn, const float* probs,
                                const float* dwctx, const float* dscores, float* dq, float* dctx,
                                int32_t accumulate, int32_t B, int32_t N, int32_t D, float* ws,
                                void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (bad_common(q, ctx, ldn, B, N, D, ws) || !probs || (!dwctx && !dscores) || (dwctx && !aligned16(dwctx)) ||
      (dq && !aligned16(dq)) || (dctx && !aligned16(dctx)))
    return (int)hipErrorInvalidValue;
  const int rpt = split_rpt(B, N, D, dwctx != nullptr);
  if (rpt) {
    SplitArgs sa{};
    sa.q = q; sa.ctx = ctx; sa.ldn = ldn; sa.a_probs = probs; sa.dwctx = dwctx; sa.dscores = dscores;
    sa.dq = dq; sa.dctx = dctx; sa.accumulate = accumulate; sa.N = N; sa.D = D;
    return launch_split_bwd(sa, rpt, B, ws, (hipStream_t)stream);
  }
  BwdArgs a{q, ctx, (long)ldn, probs, nullptr, nullptr, 0, dwctx, dscores, dq, dctx, accumulate, nullptr, N, D};
  return launch_bwd<16>(a, B, ws, (hipStream_t)stream);
}

extern "C" int dasa_shift_attn_fwd(const float* q, const float* ctx, int64_t ldn, const float* shift_logits,
                                   float* attn, float* shifted, float* wsm, float* wctx,
                                   int32_t B, int32_t D, int32_t K, float* ws, void* stream) {
  const int N = 36;
  if (B <= 0) return 0;
  if (K < 1 || K > kMaxK || bad_common(q, ctx, ldn, B, N, D, ws) || !shift_logits || !wctx || !aligned16(wctx))
    return (int)hipErrorInvalidValue;
  FwdArgs a{q, ctx, (long)ldn, nullptr, shift_logits, K, nullptr, attn, shifted, wsm, wctx, N, D};
  if (rows_ok(B, N, D)) return launch_rows(a, B, (hipStream_t)stream);
  // (A/B) 4: the row-split kernel instead of the two-launch D-split form
  if (g_attn_mode != 4 && split2_ok(B, N, D)) return launch_split2_fwd(a, B, ws, (hipStream_t)stream);
  return launch_fwd<12>(a, B, ws, (hipStream_t)stream);
}

extern "C" int dasa_shift_attn_bwd(const float* q, const float* ctx, int64_t ldn, const float* attn,
                                   const float* shifted, const float* wsm, const float* dwctx,
                                   float* dq, float* dctx, float* dshift_logits, int32_t accumulate,
                                   int32_t B, int32_t D, int32_t K, float* ws, void* stream) {
  const int N = 36;
  if (B <= 0) return 0;
  if (K < 1 || K > kMaxK || bad_common(q, ctx, ldn, B, N, D, ws) || !attn || !shifted || !wsm || !dwctx ||
      !dshift_logits || !aligned16(dwctx) || (dq && !aligned16(dq)) || (dctx && !aligned16(dctx)))
    return (int)hipErrorInvalidValue;
  const int rpt = split_rpt(B, N, D, true);
  if (rpt) {
    SplitArgs sa{};
    sa.q = q; sa.ctx = ctx; sa.ldn = ldn; sa.K = K; sa.a_probs = attn; sa.a_shifted = shifted; sa.a_wsm = wsm;
    sa.dwctx = dwctx; sa.dq = dq; sa.dctx = dctx; sa.accumulate = accumulate; sa.dshift = dshift_logits;
    sa.N = N; sa.D = D;
    return launch_split_bwd(sa, rpt, B, ws, (hipStream_t)stream);
  }
  BwdArgs a{q, ctx, (long)ldn, attn, shifted, wsm, K, dwctx, nullptr, dq, dctx, accumulate,
            dshift_logits, N, D};
  return launch_bwd<12>(a, B, ws, (hipStream_t)stream);
}
