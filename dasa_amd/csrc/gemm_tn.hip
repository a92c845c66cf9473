// bf16x6 (fp32-accurate) TN GEMM for the backward's long-K weight gradients: C = alpha * A^T B + beta * C
// with A fp32 [K][lda] (M contiguous) and B fp32 [K][ldb] (N contiguous) — dW = dYᵀ X of the batched
// bi-LSTM BPTT (agent_dg.py:1389-1405 optim_step's backward through r2rmodel.py:2339-2343: weight_ih /
// weight_hh gradients over K = steps x batch x tokens = 112000 rows at the cfg2 headline) and of the
// deferred decoder / critic weight gradients (functional.flush_weight_grads).
//
// Same numerics as the NT bf16x6 kernel of gemm.hip (form 8): both operands split exactly into three bf16
// planes (hi + mid + lo), the six products hh, hm, mh, hl, lh, mm on v_mfma_f32_16x16x32_bf16, hh in its own
// accumulator; the error against fp64 is at most the native fp32 MFMA kernel's (tests/test_kernels_gpu.py
// test_gemm_f32x6_tn). The difference is the staging: here BOTH operands arrive K-major (a row of A holds
// consecutive m at one k), while the MFMA fragment wants 8 consecutive k of one row. Each loader thread reads
// 8 k-rows x 2 adjacent columns (one 8-byte load per k-row; 64 lanes of a wave = 512 contiguous bytes of
// one k-row), so after the loads it holds, per column, the 8 consecutive k of one 16-B LDS unit: the
// transpose is register renaming, the split is form 8's split3_quad, and the LDS image is form 8's
// quad-major [plane][q][row] — the MFMA loop is form 8's loop. Threads 0-255 stage A, 256-511 stage B.
// A native fp32 TN kernel (gemm_f32_kernel) ran these at 0.6-0.8 of the 157 TF fp32 roof; the transposes
// the NT bf16x6 kernel would need cost more than it saved (profiles/r02/ab_x6_tn_rejected.txt).
//
// Rows k >= K of the last K step are read clamped and zeroed before the split (no per-element branch around
// a load). Few-tile problems (4096 x 768: 192 tiles) split K over workgroups; the last split to arrive sums
// the write-through slabs in split order (deterministic), as gemm.hip's X6Split form.
#include "gemm_common.h"

namespace {

struct TnSplit { unsigned* cnt; float* slab; int splitk, kchunk; };

constexpr int kTnCntBytes = 64 << 10;   // per-tile arrival counters at the head of the workspace
constexpr int kTnCntWords = kTnCntBytes / 4;

// ONE_STAGE: one LDS stage and one register stage in <= 128 VGPRs, two workgroups per CU (gemm.hip form 20's
// layout); otherwise two LDS stages, two register stages, one workgroup per CU (form 8's).
template <int BM, int BN, int WAVES_M, int WAVES_N, bool ONE_STAGE>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
__attribute__((amdgpu_waves_per_eu(ONE_STAGE ? 4 : 1, ONE_STAGE ? 4 : 2)))
void gemm_f32x6_tn_kernel(GemmP p, TnSplit xs) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  static_assert(NT == 512 && BM == 128 && BN == 128, "loader mapping: 256 threads per 128-column operand");
  constexpr int PA = BM * 4, PB = BN * 4;        // uint4 per plane image (4 k-quads x rows)
  constexpr int STAGE = 3 * (PA + PB);
  __shared__ uint4 smem[(ONE_STAGE ? 1 : 2) * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  // tile order: the column panels of B (N) of one row panel of A (M) on consecutive ids -> one XCD, so the
  // A panel they share streams once per XCD
  const int tiles_n = gridDim.x;
  const int wgid = xcd_remap(blockIdx.y * tiles_n + blockIdx.x, tiles_n * gridDim.y);
  const int m0 = (wgid / tiles_n) * BM, n0 = (wgid % tiles_n) * BN;
  const int split = blockIdx.z;
  const int kb = split * xs.kchunk, kend = min(p.K, kb + xs.kchunk);

  // loader: operand (A for tid < 256), column pair cp (2 columns), k-quad q
  const bool isA = tid < 256;
  const int li = tid & 255, cp = li & 63, q = li >> 6;
  const float* src = isA ? p.A : p.B;
  const long ld = isA ? p.lda : p.ldb;
  const int c0 = isA ? m0 : n0, lim = isA ? p.M : p.N;
  const int col = min(c0 + 2 * cp, lim - 2);      // clamped (M, N even): rows past the edge are never stored

  floatx4 big[TM][TN], small[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] = small[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  struct Stage {
    float2 v[8];
    int k0;
    __device__ __forceinline__ void load(const float* src, long ld, int col, int kq, int kend) {
      k0 = kq;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float2*>(src + (long)min(kq + j, kend - 1) * ld + col);
    }
    __device__ __forceinline__ void store(uint4* S, bool isA, int cp, int q, int kend) const {
      float2 w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = (k0 + j < kend) ? v[j] : float2{0.f, 0.f};   // rows past K: zero
      uint4 h, m, l;
      uint4* base = S + (isA ? 0 : 3 * PA);
      const int P = isA ? PA : PB, R = isA ? BM : BN;
      split3_quad(float4{w[0].x, w[1].x, w[2].x, w[3].x}, float4{w[4].x, w[5].x, w[6].x, w[7].x}, h, m, l);
      base[0 * P + q * R + 2 * cp] = h;
      base[1 * P + q * R + 2 * cp] = m;
      base[2 * P + q * R + 2 * cp] = l;
      split3_quad(float4{w[0].y, w[1].y, w[2].y, w[3].y}, float4{w[4].y, w[5].y, w[6].y, w[7].y}, h, m, l);
      base[0 * P + q * R + 2 * cp + 1] = h;
      base[1 * P + q * R + 2 * cp + 1] = m;
      base[2 * P + q * R + 2 * cp + 1] = l;
    }
  } stg, stg2;

  // form 8's K step: fragments of the three planes from LDS, the six products, hh in `big`
  auto compute = [&](const uint4* S) {
    const int qq = lane >> 4;
    bf16x8_t bf[3][TN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[pl][j] = __builtin_bit_cast(bf16x8_t, S[3 * PA + pl * PB + qq * BN + wn + 16 * j + (lane & 15)]);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      bf16x8_t af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        af[pl] = __builtin_bit_cast(bf16x8_t, S[pl * PA + qq * BM + wm + 16 * i + (lane & 15)]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        floatx4& sm = small[i][j];
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[1][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[2][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], bf[0][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[1][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[0][j], sm, 0, 0, 0);
        big[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[0][j], big[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = (kend - kb + 31) / 32;
  auto kq = [&](int t) { return kb + 32 * min(t, nk - 1) + 8 * q; };   // clamped re-read past the last step
  stg.load(src, ld, col, kq(0), kend);
  if (ONE_STAGE) {
    stg.store(smem, isA, cp, q, kend);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      stg.load(src, ld, col, kq(t + 1), kend);
      compute(smem);
      __syncthreads();
      stg.store(smem, isA, cp, q, kend);
      __syncthreads();
    }
  } else {
    stg2.load(src, ld, col, kq(1), kend);
    stg.store(smem, isA, cp, q, kend);
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {
      stg.load(src, ld, col, kq(t + 2), kend);
      compute(smem);
      stg2.store(smem + STAGE, isA, cp, q, kend);
      __syncthreads();
      if (t + 1 >= nk) break;
      stg2.load(src, ld, col, kq(t + 3), kend);
      compute(smem + STAGE);
      stg.store(smem, isA, cp, q, kend);
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] += small[i][j];

  if (xs.splitk > 1) {
    __shared__ int s_last;
    const int tile = (m0 / BM) * tiles_n + n0 / BN;
    constexpr int SLAB_B = BM * BN * 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(xs.slab, 0, 0x7fffffff, 0x00020000);
    const long tbase = (long)tile * xs.splitk;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int off = (int)((tbase + split) * SLAB_B) + ((i * TN + j) * NT + tid) * 16;
        const u32x4 u = {__float_as_uint(big[i][j][0]), __float_as_uint(big[i][j][1]),
                         __float_as_uint(big[i][j][2]), __float_as_uint(big[i][j][3])};
        __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);   // sc1: write-through
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      s_last = __hip_atomic_fetch_add(xs.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)(xs.splitk - 1);
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) __hip_atomic_store(xs.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: sc1 loads below the ticket
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) big[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < xs.splitk; ++s2) {     // fixed order: deterministic whoever arrives last
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int off = (int)((tbase + s2) * SLAB_B) + ((i * TN + j) * NT + tid) * 16;
          const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);   // sc1
          big[i][j][0] += __uint_as_float(u.x);
          big[i][j][1] += __uint_as_float(u.y);
          big[i][j][2] += __uint_as_float(u.z);
          big[i][j][3] += __uint_as_float(u.w);
        }
    }
  }
  store_tile_mf<16, TM, TN, BM, BN>(p, big, 0, 0, m0, n0, wm, wn, lane);
}

struct TnPlan { int form, splitk, kchunk; int64_t ws; };

static int g_tn_form = -1, g_tn_split = -1;   // dasa_gemm_x6_tn_config (sweeps / tests)

static TnPlan tn_plan(const dasa_gemm_desc* d) {
  const long tiles = cdiv(d->M, 128) * cdiv(d->N, 128);
  TnPlan pl{1, 1, d->K, 0};
  // fill >= 3 rounds of one workgroup per CU (192 tiles of the 4096 x 768 weight_ih gradient: 4 splits) while
  // every split keeps >= 64 K steps
  int s = tiles >= 256 ? 1 : (int)cdiv(768, tiles);
  if (g_tn_split > 0) s = g_tn_split;
  while (s > 1 && (long)d->K / s < 2048) --s;
  if (s > 16) s = 16;
  if (tiles * s > kTnCntWords) s = 1;
  if (g_tn_form >= 0) pl.form = g_tn_form;
  if (s > 1) {
    pl.kchunk = (int)(cdiv(cdiv(d->K, s), 32) * 32);
    pl.splitk = (int)cdiv(d->K, pl.kchunk);
    pl.ws = kTnCntBytes + tiles * pl.splitk * (int64_t)128 * 128 * (int64_t)sizeof(float);
  }
  return pl;
}

}  // namespace

extern "C" int dasa_gemm_x6_tn_config(int32_t form, int32_t splitk) {
  if (form < -1 || form > 1 || splitk < -1 || splitk > 16) return (int)hipErrorInvalidValue;
  g_tn_form = form;
  g_tn_split = splitk;
  return 0;
}

extern "C" int64_t dasa_gemm_f32x6_tn_workspace(const dasa_gemm_desc* d) {
  if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0) return 0;
  return tn_plan(d).ws;
}

extern "C" int dasa_gemm_f32x6_tn(const dasa_gemm_desc* d, void* ws, int64_t ws_bytes, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K;
  if (M < 0 || N < 0 || K < 0 || d->opA != 1 || d->opB != 0 || (d->batch > 1)) return (int)hipErrorInvalidValue;
  if ((M & 1) || (N & 1) || M < 2 || N < 2 || (d->lda & 1) || (d->ldb & 1) || d->lda < M || d->ldb < N || d->ldc < N)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)d->A & 7) || ((uintptr_t)d->B & 7)) return (int)hipErrorInvalidValue;
  if (K == 0) return (int)hipErrorInvalidValue;          // (callers handle the empty sum)
  TnPlan pl = tn_plan(d);
  if (pl.splitk > 1 && (ws == nullptr || ws_bytes < pl.ws)) { pl.splitk = 1; pl.kchunk = K; }
  GemmP p{};
  p.M = M; p.N = N; p.K = K; p.batch = 1; p.splitk = 1; p.kchunk = K;
  p.A = d->A; p.lda = d->lda;
  p.B = d->B; p.ldb = d->ldb;
  p.C = d->C; p.ldc = d->ldc;
  p.bias = d->bias; p.act = d->act;
  p.aux = d->aux; p.ld_aux = d->ld_aux;
  p.colscale = d->colscale; p.alpha = d->alpha; p.beta = d->beta;
  TnSplit xs{};
  xs.splitk = pl.splitk;
  xs.kchunk = pl.kchunk;
  if (pl.splitk > 1) {
    xs.cnt = (unsigned*)ws;
    xs.slab = (float*)((char*)ws + kTnCntBytes);
  }
  const dim3 grid((unsigned)cdiv(N, 128), (unsigned)cdiv(M, 128), (unsigned)pl.splitk);
  hipStream_t st = (hipStream_t)stream;
  if (pl.form == 0)
    hipLaunchKernelGGL((gemm_f32x6_tn_kernel<128, 128, 4, 2, true>), grid, dim3(512), 0, st, p, xs);
  else
    hipLaunchKernelGGL((gemm_f32x6_tn_kernel<128, 128, 4, 2, false>), grid, dim3(512), 0, st, p, xs);
  DASA_CHECK_LAUNCH();
  return 0;
}
