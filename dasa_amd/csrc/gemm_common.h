// Shared by the GEMM translation units (gemm.hip, gemm_tn.hip): the GEMM parameter block, the fused
// epilogue of MFMA accumulator tiles, the XCD-aware workgroup remap and the exact fp32 -> 3 x bf16 split of
// the bf16x6 kernels. Everything sits in an anonymous namespace: each unit gets its own copy.
#pragma once
#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

struct GemmP {
  int M, N, K, batch, splitk, kchunk;
  const float* A; long lda, sA;
  const float* B; long ldb, sB;
  float* C; long ldc, sC;
  const float* bias; int act;
  const float* aux; long ld_aux, sAux;
  const float* colscale;
  float alpha, beta;
  float* ws;
  int group_m;   // > 1: L2-grouped tile order (64-deep K kernels, non-stream-K)
  unsigned* cnt; // split-K of gemm_f32_kernel: per-tile arrival counters (last arriver reduces in-kernel), or
                 // null: partials to ws in [split][b][M][N] for splitk_reduce_kernel
};

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case DASA_ACT_RELU: return fmaxf(v, 0.f);
    case DASA_ACT_GELU: return gelu_erf(v);
    case DASA_ACT_TANH: return tanhf(v);
    case DASA_ACT_SIGMOID: return sigmoidf_(v);
    default: return v;
  }
}

__device__ __forceinline__ void epilogue_store(const GemmP& p, int b, int row, int col, float acc) {
  float v = p.alpha * acc;
  if (p.bias) v += p.bias[col];
  v = apply_act(v, p.act);
  if (p.aux) v *= p.aux[(long)b * p.sAux + (long)row * p.ld_aux + col];
  if (p.colscale) v *= p.colscale[col];
  float* c = p.C + (long)b * p.sC + (long)row * p.ldc + col;
  if (p.beta != 0.f) v += p.beta * (*c);
  *c = v;
}

// Fused epilogue of one wave's TM x TN accumulators of MF x MF MFMA tiles (MF = 32: floatx16,
// MF = 16: floatx4) at block origin (m0, n0), wave offset (wm, wn). C/D map: col = lane & (MF-1);
// row = (r&3) + 8*(r>>2) + 4*(lane>>5) for 32x32, row = 4*(lane>>4) + r for 16x16.
// Every optional operand is fetched with unconditional clamped loads inside ONE uniform branch per
// operand (a per-element branch around a load makes hipcc wait vmcnt(0) per element).
template <int MF, int TM, int TN, int BM, int BN, typename AccT>
__device__ __forceinline__ void store_tile_mf(const GemmP& p, AccT (&acc)[TM][TN], int b, int split, int m0,
                                              int n0, int wm, int wn, int lane) {
  constexpr int NR = MF == 32 ? 16 : 4;
  const bool full_tile = (m0 + BM <= p.M) && (n0 + BN <= p.N);
  auto rowof = [&](int rbase, int r) { return MF == 32 ? rbase + (r & 3) + 8 * (r >> 2) : rbase + r; };
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + j * MF + (lane & (MF - 1));
    const int colc = min(col, p.N - 1);
    float bj = 0.f, cs = 1.f;
    if (p.splitk == 1) {
      if (p.bias) bj = p.bias[colc];
      if (p.colscale) cs = p.colscale[colc];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rbase = m0 + wm + i * MF + (MF == 32 ? 4 * (lane >> 5) : 4 * (lane >> 4));
      if (p.splitk > 1) {
        float* ws = p.ws + ((long)split * p.batch + b) * p.M * p.N;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int row = rowof(rbase, r);
          if (full_tile || (row < p.M && col < p.N)) ws[(long)row * p.N + col] = acc[i][j][r];
        }
        continue;
      }
      float v[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) v[r] = p.alpha * acc[i][j][r] + bj;
      switch (p.act) {   // one uniform branch per tile, not per element
        case DASA_ACT_RELU:
#pragma unroll
          for (int r = 0; r < NR; ++r) v[r] = fmaxf(v[r], 0.f);
          break;
        case DASA_ACT_GELU:
#pragma unroll
          for (int r = 0; r < NR; ++r) v[r] = gelu_erf(v[r]);
          break;
        case DASA_ACT_TANH:
#pragma unroll
          for (int r = 0; r < NR; ++r) v[r] = tanhf(v[r]);
          break;
        case DASA_ACT_SIGMOID:
#pragma unroll
          for (int r = 0; r < NR; ++r) v[r] = sigmoidf_(v[r]);
          break;
        default:
          break;
      }
      if (p.aux) {
        const float* ab = p.aux + (long)b * p.sAux;
        float av[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) av[r] = ab[(long)min(rowof(rbase, r), p.M - 1) * p.ld_aux + colc];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] *= av[r];
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) v[r] *= cs;
      float* cb = p.C + (long)b * p.sC;
      if (p.beta != 0.f) {
        float cv[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) cv[r] = cb[(long)min(rowof(rbase, r), p.M - 1) * p.ldc + colc];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] += p.beta * cv[r];
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int row = rowof(rbase, r);
        if (full_tile || (row < p.M && col < p.N)) cb[(long)row * p.ldc + col] = v[r];
      }
    }
  }
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

inline long cdiv(long a, long b) { return (a + b - 1) / b; }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  const f32x2_t w = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(w, bf16x2_t));
}

__device__ __forceinline__ void split3_pair(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  h = pack_bf16x2(a, b);
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  m = pack_bf16x2(ra, rb);
  l = pack_bf16x2(ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u));
}

__device__ __forceinline__ void split3_quad(const float4& x, const float4& y, uint4& h, uint4& m, uint4& l) {
  split3_pair(x.x, x.y, h.x, m.x, l.x);
  split3_pair(x.z, x.w, h.y, m.y, l.y);
  split3_pair(y.x, y.y, h.z, m.z, l.z);
  split3_pair(y.z, y.w, h.w, m.w, l.w);
}

}  // namespace
