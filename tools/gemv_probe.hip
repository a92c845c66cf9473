// Probe (r06): fp32 weight-streaming GEMV forms for the decision step's M <= 32 projections
// (Y[M,N] = X[M,K] . W[N,K]^T, nn.Linear at B = 20), against the library's gemm_skinny_nt_kernel.
//   mode 0  floor: the same W loads as mode 1, summed and written per lane (no X, no MFMA)
//   mode 1  no split-K: workgroup = 16 W rows x the whole K, split over the workgroup's waves
//           (contiguous K ranges), partials summed in LDS; MT 16-column MFMA tiles of X rows
//   mode 2  mode 1 with rows 16..M-1 (M <= 20) on the VALU from X staged in LDS (hybrid)
//   mode 3  mode 1's loads (W and X), summed on the VALU instead of the MFMAs (diagnosis)
//   mode 4  mode 1's MFMAs with W loaded and X a register constant (no X loads; diagnosis)
// Lane (r = lane & 15, g = lane >> 4) of a wave loads W[n0 + r][k + 8g .. +7] per 32-deep step, all
// steps issued before the first MFMA.
#include <hip/hip_runtime.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float f4get(const float4 v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ float4 sel4(bool ok, float4 v) { return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f); }

template <int S>
__global__ __launch_bounds__(1024) void floor_kernel(const float* __restrict__ W, float* __restrict__ out, int N, int K) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W_ = blockDim.x >> 6, r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16, kq = K - 4;
  const float* wrow = W + (long)min(n0 + r, N - 1) * K;
  const int kbase = w * S * 32 + 8 * g;
  float4 wv[S][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = kbase + 32 * s;
    wv[s][0] = ldg4(wrow + min(k, kq));
    wv[s][1] = ldg4(wrow + min(k + 4, kq));
  }
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) acc += wv[s][h].x + wv[s][h].y + wv[s][h].z + wv[s][h].w;
  out[(long)blockIdx.x * blockDim.x + threadIdx.x] = acc;
  (void)W_;
}

template <int S, int MT, int XR, int DIAG = 0>
__global__ __launch_bounds__(1024) void gemv_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                    float* __restrict__ Y, int M, int N, int K) {
  extern __shared__ floatx4 red[];   // [waves - 1][MT + 1][64]; hybrid: X rows 16.. staged after it
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, NW = blockDim.x >> 6, r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16, kq = K - 4;
  const float* wrow = W + (long)min(n0 + r, N - 1) * K;
  const float* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xrow[t] = X + (long)min(16 * t + r, M - 1) * K;
  const int kbase = w * S * 32 + 8 * g;
  float4* xs = reinterpret_cast<float4*>(red + (NW - 1) * (MT + 1) * 64);
  if constexpr (XR > 0) {   // rows 16 .. 16 + XR - 1 of this wave's K range into LDS (the wave's own slice)
    const int kw = w * S * 32;
#pragma unroll
    for (int i = 0; i < (XR * S * 8 + 63) / 64; ++i) {
      const int idx = lane + 64 * i, q = idx / (S * 8), kk = kw + 4 * (idx % (S * 8));
      if (idx >= XR * S * 8) break;
      const float z = (16 + q < M && kk < K) ? 1.f : 0.f;
      const float4 v = ldg4(X + (long)min(16 + q, M - 1) * K + min(kk, kq));
      xs[(w * XR + q) * S * 8 + idx % (S * 8)] = make_float4(z * v.x, z * v.y, z * v.z, z * v.w);
    }
    __builtin_amdgcn_wave_barrier();
  }
  float4 wv[S][2], xv[S][MT][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = kbase + 32 * s;
    wv[s][0] = ldg4(wrow + min(k, kq));
    wv[s][1] = ldg4(wrow + min(k + 4, kq));
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if (DIAG == 4) {
        xv[s][t][0] = make_float4(1.f, 1.f, 1.f, 1.f);
        xv[s][t][1] = xv[s][t][0];
      } else {
        xv[s][t][0] = ldg4(xrow[t] + min(k, kq));
        xv[s][t][1] = ldg4(xrow[t] + min(k + 4, kq));
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (DIAG == 3) {
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        sum += wv[s][h].x + wv[s][h].y + wv[s][h].z + wv[s][h].w;
#pragma unroll
        for (int t = 0; t < MT; ++t) sum += xv[s][t][h].x + xv[s][t][h].y + xv[s][t][h].z + xv[s][t][h].w;
      }
    Y[(long)blockIdx.x * blockDim.x + threadIdx.x] = sum;
    return;
  }
  floatx4 acc[MT + 1];
#pragma unroll
  for (int t = 0; t <= MT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = kbase + 32 * s;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool ok = k + 4 * h < K;
      const float4 a = sel4(ok, wv[s][h]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < MT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, e), f4get(sel4(ok, xv[s][t][h]), e), acc[t], 0, 0, 0);
      if constexpr (XR > 0) {
        const int kl = (32 * s + 8 * g) / 4 + h;
#pragma unroll
        for (int q = 0; q < XR; ++q) {
          const float4 x = xs[(w * XR + q) * S * 8 + kl];
          float v = acc[MT][q];
          v = fmaf(a.x, x.x, v);
          v = fmaf(a.y, x.y, v);
          v = fmaf(a.z, x.z, v);
          v = fmaf(a.w, x.w, v);
          acc[MT][q] = v;
        }
      }
    }
  }
  if constexpr (XR > 0) {
#pragma unroll
    for (int q = 0; q < XR; ++q) {
      float v = acc[MT][q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[MT][q] = v;
    }
  }
  constexpr int NA = MT + (XR ? 1 : 0);
  if (w > 0) {
#pragma unroll
    for (int a = 0; a < NA; ++a) red[((w - 1) * (MT + 1) + a) * 64 + lane] = acc[a];
  }
  __syncthreads();
  if (w > 0) return;
  for (int v = 0; v < NW - 1; ++v)
#pragma unroll
    for (int a = 0; a < NA; ++a) acc[a] += red[(v * (MT + 1) + a) * 64 + lane];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * t + r, n = n0 + 4 * g + j;
      if (m < M && n < N) Y[(long)m * N + n] = acc[t][j];
    }
  if constexpr (XR > 0) {
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < XR; ++q)
        if (16 + q < M && n0 + r < N) Y[(long)(16 + q) * N + n0 + r] = acc[MT][q];
    }
  }
}


// mode 5: workgroup = 4 waves = RW row waves (16 W rows each) x (4 / RW) K waves; X rows [0, M) of the
// workgroup's K range staged ONCE in LDS (one coalesced pass through the TA instead of one X fragment
// per W fragment: the r06 probe measured the per-wave X loads as the form's cost); split-K partials
// (one slab per (column block, split, wave)) summed in fixed split order by the last arriver.
template <int S, int RW>
__global__ __launch_bounds__(256) void gemv_xlds_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                        float* __restrict__ Y, int M, int N, int K,
                                                        float* __restrict__ slab, unsigned* __restrict__ cnt) {
  constexpr int KW = 4 / RW, KWG = KW * S * 32, LDX = KWG + 4;   // LDX: padded row stride (floats)
  __shared__ float xs[32 * LDX];
  __shared__ floatx4 red[KW > 1 ? 3 : 1][2][64];
  __shared__ int s_last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int rw = w % RW, kw = w / RW;
  const int col = blockIdx.x, split = blockIdx.y, splits = gridDim.y;
  const int n0 = col * 16 * RW + 16 * rw, k0 = split * KWG, kq = K - 4;
  // X staging loads first (M rows x KWG), then every W load of the wave
  constexpr int XQ = 32 * KWG / 4, XI = (XQ + 255) / 256;
  float4 xe[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int idx = threadIdx.x + 256 * i, m = idx / (KWG / 4), kk = k0 + 4 * (idx % (KWG / 4));
    xe[i] = ldg4(X + (long)min(m, M - 1) * K + min(kk, kq));
  }
  const float* wrow = W + (long)min(n0 + r, N - 1) * K;
  const int kb = k0 + kw * S * 32 + 8 * g;
  float4 wv[S][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    wv[s][0] = ldg4(wrow + min(kb + 32 * s, kq));
    wv[s][1] = ldg4(wrow + min(kb + 32 * s + 4, kq));
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int idx = threadIdx.x + 256 * i, m = idx / (KWG / 4), kl = 4 * (idx % (KWG / 4));
    if (idx < XQ) {
      const bool ok = m < M && k0 + kl < K;
      *reinterpret_cast<float4*>(&xs[m * LDX + kl]) = sel4(ok, xe[i]);
    }
  }
  __syncthreads();
  const bool two = M > 16;
  floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kl = kw * S * 32 + 32 * s + 8 * g + 4 * h;
      const bool ok = k0 + kl < K;
      const float4 a = sel4(ok, wv[s][h]);
      const float4 x0 = *reinterpret_cast<const float4*>(&xs[r * LDX + kl]);
      const float4 x1 = *reinterpret_cast<const float4*>(&xs[(16 + r) * LDX + kl]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, e), f4get(x0, e), acc[0], 0, 0, 0);
        if (two) acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, e), f4get(x1, e), acc[1], 0, 0, 0);
      }
    }
  }
  if constexpr (KW > 1) {   // the K waves of a row wave meet in LDS (fixed order)
    if (kw > 0) {
      red[(kw - 1) * RW + rw][0][lane] = acc[0];
      red[(kw - 1) * RW + rw][1][lane] = acc[1];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int v = 1; v < KW; ++v) {
      acc[0] += red[(v - 1) * RW + rw][0][lane];
      acc[1] += red[(v - 1) * RW + rw][1][lane];
    }
  }
  if (splits > 1) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int off = (int)(((((long)col * splits + split) * RW + rw) * 2 + a) * 64 + lane) * 16;
      const u32x4 u = {__float_as_uint(acc[a][0]), __float_as_uint(acc[a][1]), __float_as_uint(acc[a][2]),
                       __float_as_uint(acc[a][3])};
      __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (RW > 1) __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(cnt + col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(splits - 1);
    if constexpr (RW > 1) __syncthreads(); else __builtin_amdgcn_wave_barrier();
    if (!s_last) return;
    if (threadIdx.x == 0) __hip_atomic_store(cnt + col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    acc[0] = acc[1] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < splits; ++s2) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int off = (int)(((((long)col * splits + s2) * RW + rw) * 2 + a) * 64 + lane) * 16;
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
        acc[a][0] += __uint_as_float(u.x);
        acc[a][1] += __uint_as_float(u.y);
        acc[a][2] += __uint_as_float(u.z);
        acc[a][3] += __uint_as_float(u.w);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * t + r, n = n0 + 4 * g + j;
      if (m < M && n < N) Y[(long)m * N + n] = acc[t][j];
    }
}

float* g_slab = nullptr;      // split-K partials (gemv_set_ws)
unsigned* g_cnt = nullptr;   // arrival counters, zero

template <int S>
int launch_s(int mode, const float* X, const float* W, float* Y, int M, int N, int K, int waves, hipStream_t st) {
  const dim3 grid((N + 15) / 16), block(64 * waves);
  if (mode == 0) {
    hipLaunchKernelGGL((floor_kernel<S>), grid, block, 0, st, W, Y, N, K);
  } else if (mode == 1) {
    const size_t lds = (size_t)(waves - 1) * 3 * 64 * 16;
    if (M <= 16)
      hipLaunchKernelGGL((gemv_kernel<S, 1, 0>), grid, block, lds, st, X, W, Y, M, N, K);
    else
      hipLaunchKernelGGL((gemv_kernel<S, 2, 0>), grid, block, lds, st, X, W, Y, M, N, K);
  } else if (mode >= 50) {   // 5x: gemv_xlds_kernel, RW = mode - 50, K split to cover K
    const int rw = mode - 50, kwg = (4 / rw) * S * 32, splits = (K + kwg - 1) / kwg;
    const dim3 g5((N + 16 * rw - 1) / (16 * rw), splits);
    if ((long)g5.x * splits > 16384 || splits > 64) return -5;
    if (rw == 1) hipLaunchKernelGGL((gemv_xlds_kernel<S, 1>), g5, dim3(256), 0, st, X, W, Y, M, N, K, g_slab, g_cnt);
    else if (rw == 2) hipLaunchKernelGGL((gemv_xlds_kernel<S, 2>), g5, dim3(256), 0, st, X, W, Y, M, N, K, g_slab, g_cnt);
    else hipLaunchKernelGGL((gemv_xlds_kernel<S, 4>), g5, dim3(256), 0, st, X, W, Y, M, N, K, g_slab, g_cnt);
  } else if (mode == 3 || mode == 4) {
    const size_t lds = (size_t)(waves - 1) * 3 * 64 * 16;
    if (mode == 3)
      hipLaunchKernelGGL((gemv_kernel<S, 2, 0, 3>), grid, block, lds, st, X, W, Y, M, N, K);
    else
      hipLaunchKernelGGL((gemv_kernel<S, 2, 0, 4>), grid, block, lds, st, X, W, Y, M, N, K);
  } else {
    if (M <= 16 || M > 20) return -2;
    const size_t lds = (size_t)(waves - 1) * 2 * 64 * 16 + (size_t)waves * 4 * S * 8 * 16;
    hipLaunchKernelGGL((gemv_kernel<S, 1, 4>), grid, block, lds, st, X, W, Y, M, N, K);
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" void gemv_set_ws(float* slab, unsigned* cnt) {
  g_slab = slab;
  g_cnt = cnt;
}

extern "C" int gemv_launch(int mode, const float* X, const float* W, float* Y, int M, int N, int K, int waves,
                           int S, void* stream) {
  if (waves < 1 || waves > 16 || (K & 3) || M < 1 || M > 32) return -1;
  if (mode < 50 && (long)waves * S * 32 < K) return -3;   // the workgroup must cover K
  hipStream_t st = (hipStream_t)stream;
  switch (S) {
    case 1: return launch_s<1>(mode, X, W, Y, M, N, K, waves, st);
    case 2: return launch_s<2>(mode, X, W, Y, M, N, K, waves, st);
    case 4: return launch_s<4>(mode, X, W, Y, M, N, K, waves, st);
    case 8: return launch_s<8>(mode, X, W, Y, M, N, K, waves, st);
    default: return -4;
  }
}
