// SoftDotAttention / ShiftSoftDotAttention forward + backward for gfx950 (model.py:253-353).
//
// Both are HBM-bound: one pass over ctx [B][N][D] for the scores and one for the weighted sum
// (the second mostly L2/MALL-served). Kernel split:
//   scores_kernel : one wave per (b, n) row, float4 coalesced dot over D, wave-shuffle reduction.
//   apply_kernel  : grid (B, D/256); each block recomputes the tiny N-wide softmax (+ the 3x12
//                   circular shift for the panorama) in LDS, then its 4 waves split the N rows of a
//                   256-column slab (float4 per lane) and reduce across waves through LDS.
// The backward reuses scores_kernel for dp = ctx.dwctx and fuses dq and dctx in one slab pass.
#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

constexpr int kMaxN = 256;   // max attended rows (instruction <= 80, views 36, candidates)
constexpr int kMaxK = 15;    // max shift taps

// scores[b][n] = sum_d ctx[b][n][d] * q[b][d]; one wave per row.
__global__ __launch_bounds__(256) void scores_kernel(const float* __restrict__ q, long ldq,
                                                     const float* __restrict__ ctx, long ldn,
                                                     float* __restrict__ out, int B, int N, int D) {
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave >= B * N) return;
  const int b = wave / N, n = wave % N;
  const float4* c4 = reinterpret_cast<const float4*>(ctx + ((long)b * N + n) * ldn);
  const float4* q4 = reinterpret_cast<const float4*>(q + (long)b * ldq);
  float s = 0.f;
  const int D4 = D >> 2;
  for (int i = lane; i < D4; i += 64) {
    const float4 c = c4[i], v = q4[i];
    s = fmaf(c.x, v.x, s);
    s = fmaf(c.y, v.y, s);
    s = fmaf(c.z, v.z, s);
    s = fmaf(c.w, v.w, s);
  }
  s = wave_sum(s);
  if (lane == 0) out[(long)b * N + n] = s;
}

// Softmax over n of scores[b][:N] with optional mask (-inf), written to sp[0..N).
// Called by all 256 threads of the block; wave 0 does the work.
__device__ void block_softmax(const float* sc, const uint8_t* mask, int N, float* sp) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    float m = -INFINITY;
    for (int n = lane; n < N; n += 64) {
      float v = sc[n];
      if (mask && mask[n]) v = -INFINITY;
      sp[n] = v;
      m = fmaxf(m, v);
    }
    m = wave_max(m);
    float s = 0.f;
    for (int n = lane; n < N; n += 64) {
      const float e = (sp[n] == -INFINITY) ? 0.f : __expf(sp[n] - m);
      sp[n] = e;
      s += e;
    }
    s = wave_sum(s);
    const float inv = 1.f / s;
    for (int n = lane; n < N; n += 64) sp[n] *= inv;
  }
}

// 3 elevation rows x 12 headings circular correlation (model.py:337-344).
__device__ __forceinline__ float shift_at(const float* a, const float* w, int K, int v) {
  const int r = v / 12, j = v % 12, p = K / 2;
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    int jj = j + k - p;
    jj = ((jj % 12) + 12) % 12;
    s = fmaf(w[k], a[r * 12 + jj], s);
  }
  return s;
}

struct ApplyArgs {
  const float* q; const float* ctx; long ldn;
  const float* scores; const uint8_t* mask;
  const float* shift_logits; int K;
  float* probs; float* shifted; float* wsm; float* wctx;
  int B, N, D;
};

// Forward slab kernel: softmax (+shift) then wctx[b][slab] = sum_n p'[n] ctx[b][n][slab].
__global__ __launch_bounds__(256) void apply_fwd_kernel(ApplyArgs a) {
  __shared__ float sp[kMaxN];
  __shared__ float sw[kMaxK];
  __shared__ float sa2[kMaxN];
  __shared__ float4 red[4][64];
  const int b = blockIdx.x;
  const int N = a.N;
  block_softmax(a.scores + (long)b * N, a.mask ? a.mask + (long)b * N : nullptr, N, sp);
  __syncthreads();
  const float* pw = sp;
  if (a.shift_logits) {
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      float z = lane < a.K ? a.shift_logits[(long)b * a.K + lane] : -INFINITY;
      const float m = wave_max(z);
      const float e = lane < a.K ? __expf(z - m) : 0.f;
      const float s = wave_sum(e);
      if (lane < a.K) sw[lane] = e / s;
    }
    __syncthreads();
    for (int v = threadIdx.x; v < N; v += 256) sa2[v] = shift_at(sp, sw, a.K, v);
    __syncthreads();
    pw = sa2;
  }
  if (blockIdx.y == 0) {
    for (int n = threadIdx.x; n < N; n += 256) {
      if (a.probs) a.probs[(long)b * N + n] = sp[n];
      if (a.shifted && a.shift_logits) a.shifted[(long)b * N + n] = sa2[n];
    }
    if (a.wsm && a.shift_logits && threadIdx.x < a.K) a.wsm[(long)b * a.K + threadIdx.x] = sw[threadIdx.x];
  }
  if (!a.wctx) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d4 = blockIdx.y * 64 + lane;  // float4 index within the row
  const int D4 = a.D >> 2;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (d4 < D4) {
    const float* base = a.ctx + (long)b * N * a.ldn;
    for (int n = w; n < N; n += 4) {
      const float pn = pw[n];
      const float4 c = reinterpret_cast<const float4*>(base + (long)n * a.ldn)[d4];
      acc.x = fmaf(pn, c.x, acc.x);
      acc.y = fmaf(pn, c.y, acc.y);
      acc.z = fmaf(pn, c.z, acc.z);
      acc.w = fmaf(pn, c.w, acc.w);
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && d4 < D4) {
    float4 s = red[0][lane];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      s.x += red[i][lane].x; s.y += red[i][lane].y; s.z += red[i][lane].z; s.w += red[i][lane].w;
    }
    reinterpret_cast<float4*>(a.wctx + (long)b * a.D)[d4] = s;
  }
}

struct BwdArgs {
  const float* q; const float* ctx; long ldn;
  const float* probs;     // softmax a [B][N]
  const float* shifted;   // a' [B][N] (shift only)
  const float* wsm;       // w [B][K] (shift only)
  int K;
  const float* dp;        // ctx.dwctx [B][N] or NULL
  const float* dwctx;     // [B][D] or NULL
  const float* dscores;   // [B][N] or NULL
  float* dq; float* dctx; int accumulate;
  float* dshift;          // [B][K] (shift only)
  int B, N, D;
};

// Backward slab kernel: ds (softmax / shift backward, recomputed per block), then
// dq[slab] = sum_n ds[n] ctx[n][slab]; dctx[n][slab] (+)= pw[n]*dwctx[slab] + ds[n]*q[slab].
__global__ __launch_bounds__(256) void apply_bwd_kernel(BwdArgs a) {
  __shared__ float sds[kMaxN];
  __shared__ float spw[kMaxN];
  __shared__ float sda[kMaxN];
  __shared__ float sdw[kMaxK];
  __shared__ float4 red[4][64];
  const int b = blockIdx.x, N = a.N;
  const float* p = a.probs + (long)b * N;
  const bool shift = a.wsm != nullptr;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    // da = grad wrt the (pre-shift) softmax output
    if (shift) {
      const float* w = a.wsm + (long)b * a.K;
      const float* dap = a.dp + (long)b * N;  // grad wrt a'
      const int P = a.K / 2;
      for (int v = lane; v < N; v += 64) {
        const int r = v / 12, i = v % 12;
        float s = 0.f;
        for (int k = 0; k < a.K; ++k) {
          int j = i - k + P;
          j = ((j % 12) + 12) % 12;
          s = fmaf(w[k], dap[r * 12 + j], s);
        }
        sda[v] = s;
        spw[v] = a.shifted[(long)b * N + v];
      }
      // dw[k] = sum_{r,j} da'[r][j] * a[r][(j+k-P) mod 12]; softmax backward over K taps.
      float dwk = 0.f;
      if (lane < a.K) {
        for (int v = 0; v < N; ++v) {
          const int r = v / 12, j = v % 12;
          int jj = j + lane - P;
          jj = ((jj % 12) + 12) % 12;
          dwk = fmaf(dap[v], p[r * 12 + jj], dwk);
        }
      }
      const float wk = lane < a.K ? w[lane] : 0.f;
      const float dot = wave_sum(wk * dwk);
      if (lane < a.K) {
        sdw[lane] = wk * (dwk - dot);
        a.dshift[(long)b * a.K + lane] = sdw[lane];
      }
    } else {
      for (int v = lane; v < N; v += 64) {
        sda[v] = a.dp ? a.dp[(long)b * N + v] : 0.f;
        spw[v] = p[v];
      }
    }
    float dot = 0.f;
    for (int v = lane; v < N; v += 64) dot = fmaf(p[v], sda[v], dot);
    dot = wave_sum(dot);
    for (int v = lane; v < N; v += 64) {
      float ds = p[v] * (sda[v] - dot);
      if (a.dscores) ds += a.dscores[(long)b * N + v];
      sds[v] = ds;
    }
  }
  __syncthreads();
  (void)sdw;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d4 = blockIdx.y * 64 + lane;
  const int D4 = a.D >> 2;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (d4 < D4) {
    const float* base = a.ctx + (long)b * N * a.ldn;
    float* dbase = a.dctx ? a.dctx + (long)b * N * a.ldn : nullptr;
    const float4 qv = reinterpret_cast<const float4*>(a.q + (long)b * a.D)[d4];
    const float4 gv = a.dwctx ? reinterpret_cast<const float4*>(a.dwctx + (long)b * a.D)[d4]
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int n = w; n < N; n += 4) {
      const float ds = sds[n], pn = spw[n];
      const float4 c = reinterpret_cast<const float4*>(base + (long)n * a.ldn)[d4];
      acc.x = fmaf(ds, c.x, acc.x);
      acc.y = fmaf(ds, c.y, acc.y);
      acc.z = fmaf(ds, c.z, acc.z);
      acc.w = fmaf(ds, c.w, acc.w);
      if (dbase) {
        float4* dp4 = reinterpret_cast<float4*>(dbase + (long)n * a.ldn) + d4;
        float4 g;
        g.x = pn * gv.x + ds * qv.x;
        g.y = pn * gv.y + ds * qv.y;
        g.z = pn * gv.z + ds * qv.z;
        g.w = pn * gv.w + ds * qv.w;
        if (a.accumulate) {
          const float4 o = *dp4;
          g.x += o.x; g.y += o.y; g.z += o.z; g.w += o.w;
        }
        *dp4 = g;
      }
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && d4 < D4 && a.dq) {
    float4 s = red[0][lane];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      s.x += red[i][lane].x; s.y += red[i][lane].y; s.z += red[i][lane].z; s.w += red[i][lane].w;
    }
    reinterpret_cast<float4*>(a.dq + (long)b * a.D)[d4] = s;
  }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int dasa_softdot_fwd(const float* q, const float* ctx, int64_t ldn, const uint8_t* mask,
                                float* scores, float* probs, float* wctx,
                                int32_t B, int32_t N, int32_t D, void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (N > kMaxN || (D & 3) || (ldn & 3) || ldn < D || !scores || !aligned16(q) || !aligned16(ctx))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(scores_kernel, dim3((B * N + 3) / 4), dim3(256), 0, st, q, (long)D, ctx, (long)ldn,
                     scores, B, N, D);
  DASA_CHECK_LAUNCH();
  if (probs || wctx) {
    ApplyArgs a{q, ctx, (long)ldn, scores, mask, nullptr, 0, probs, nullptr, nullptr, wctx, B, N, D};
    dim3 grid(B, wctx ? (D / 4 + 63) / 64 : 1);
    hipLaunchKernelGGL(apply_fwd_kernel, grid, dim3(256), 0, st, a);
    DASA_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int dasa_softdot_bwd(const float* q, const float* ctx, int64_t ldn, const float* probs,
                                const float* dwctx, const float* dscores, float* dq, float* dctx,
                                int32_t accumulate, int32_t B, int32_t N, int32_t D, float* ws,
                                void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (N > kMaxN || (D & 3) || (ldn & 3) || ldn < D || !probs || (dwctx && !ws))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dwctx) {  // dp = ctx . dwctx -> ws[B][N]
    hipLaunchKernelGGL(scores_kernel, dim3((B * N + 3) / 4), dim3(256), 0, st, dwctx, (long)D, ctx,
                       (long)ldn, ws, B, N, D);
    DASA_CHECK_LAUNCH();
  }
  BwdArgs a{q, ctx, (long)ldn, probs, nullptr, nullptr, 0, dwctx ? ws : nullptr, dwctx, dscores,
            dq, dctx, accumulate, nullptr, B, N, D};
  hipLaunchKernelGGL(apply_bwd_kernel, dim3(B, (D / 4 + 63) / 64), dim3(256), 0, st, a);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_shift_attn_fwd(const float* q, const float* ctx, int64_t ldn, const float* shift_logits,
                                   float* attn, float* shifted, float* wsm, float* wctx,
                                   int32_t B, int32_t D, int32_t K, float* ws, void* stream) {
  const int N = 36;
  if (B <= 0) return 0;
  if (K < 1 || K > kMaxK || (D & 3) || (ldn & 3) || ldn < D || !shift_logits || !wctx || !ws)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(scores_kernel, dim3((B * N + 3) / 4), dim3(256), 0, st, q, (long)D, ctx, (long)ldn,
                     ws, B, N, D);
  DASA_CHECK_LAUNCH();
  ApplyArgs a{q, ctx, (long)ldn, ws, nullptr, shift_logits, K, attn, shifted, wsm, wctx, B, N, D};
  hipLaunchKernelGGL(apply_fwd_kernel, dim3(B, (D / 4 + 63) / 64), dim3(256), 0, st, a);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_shift_attn_bwd(const float* q, const float* ctx, int64_t ldn, const float* attn,
                                   const float* shifted, const float* wsm, const float* dwctx,
                                   float* dq, float* dctx, float* dshift_logits, int32_t accumulate,
                                   int32_t B, int32_t D, int32_t K, float* ws, void* stream) {
  const int N = 36;
  if (B <= 0) return 0;
  if (K < 1 || K > kMaxK || (D & 3) || (ldn & 3) || ldn < D || !attn || !shifted || !wsm || !dwctx ||
      !dshift_logits || !ws)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(scores_kernel, dim3((B * N + 3) / 4), dim3(256), 0, st, dwctx, (long)D, ctx,
                     (long)ldn, ws, B, N, D);
  DASA_CHECK_LAUNCH();
  BwdArgs a{q, ctx, (long)ldn, attn, shifted, wsm, K, ws, dwctx, nullptr, dq, dctx, accumulate,
            dshift_logits, B, N, D};
  hipLaunchKernelGGL(apply_bwd_kernel, dim3(B, (D / 4 + 63) / 64), dim3(256), 0, st, a);
  DASA_CHECK_LAUNCH();
  return 0;
}
