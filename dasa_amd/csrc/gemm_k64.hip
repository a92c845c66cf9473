// bf16x6 NT GEMM with a 64-deep K step.
//
// gemm.hip's forms 8 / 20 advance K 32 at a time: per step every wave runs 48 MFMAs (its 32 x 64 wave tile
// times six products) and then the workgroup meets at the split + ds_write + barrier phase; the r05 PMC
// breakdown (profiles/r05/x6_pmc/) puts 38-49 % of wave time at waitcnt / barrier. Here one LDS stage holds
// a 64-deep K slab (two 32-deep sub-slabs in form 8's quad-major [plane][q][row] layout), so every wave
// runs 96 MFMAs between barriers — half the barrier / split phases per MAC.
// The 64-deep slab of a 128 x 128 tile is 96 KB of LDS (three bf16 planes per operand), so two of them do
// not fit a CU's 160 KB: form 1 keeps 128 x 128 tiles at one workgroup per CU (the next slab is prefetched
// into registers during the MFMAs, as form 20 does); forms 2 / 3 halve one tile side (72 KB) so that two
// workgroups share a CU and overlap each other's split / ds_write phase with their MFMAs, as form 20 does.
//   form 1: 128 x 128, 8 waves of 32 x 64 (form 20's wave tile), 96 KB, one workgroup per CU
//   form 2: 128 x  64, 4 waves of 64 x 32, 72 KB, two workgroups per CU
//   form 3:  64 x 128, 4 waves of 32 x 64, 72 KB, two workgroups per CU
// Every form runs form 8's products in form 8's order (each 32-deep sub-slab in K order, hh in its own
// accumulator): bitwise equal to form 8. A is split on its way into LDS; W arrives pre-split.
// MEASURED AND REJECTED (probe entry only; profiles/r06/k64/probe.log, graph-timed, bitwise equal to form 8 on
// all ten shapes): 0.70-0.80x the planned forms everywhere — 12800 x 3072 x 768 476 / 488 / 496 us (forms 1 / 2 /
// 3) vs 356 us form 20, 12800 x 768 x 3072 486-510 vs 357 default, 1600 x 4096 x 768 93-106 vs 75. Halving the
// barriers per MAC does not pay: with one 96 KB stage per CU (form 1) the whole workgroup's split / ds_write
// phase runs with no MFMA beside it, and the two-per-CU half tiles (forms 2 / 3) run 2 waves per SIMD instead of
// form 20's 4 — the barrier count is not what bounds forms 8 / 20, the overlap of the store phase is.
#include "gemm_common.h"

namespace {

template <int BM, int BN, int WAVES_M, int WAVES_N, int OCC>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) __attribute__((amdgpu_waves_per_eu(1, OCC)))
void gemm_f32x6_k64_kernel(GemmP p, long plane) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;     // 16-B K quads per thread per plane (8 quads per row)
  static_assert(NA * NT == BM * 8 && NB * NT == BN * 8, "tile quads must split evenly");
  constexpr int PA = BM * 4, PB = BN * 4;               // uint4 per plane image of one 32-deep sub-slab
  constexpr int SUB = 3 * (PA + PB);
  __shared__ uint4 smem[2 * SUB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m < -1) {   // groups of -group_m W column panels, A streaming under them (form 8's order)
    const int gn = -p.group_m, per = gn * gridDim.y, grp = wgid / per;
    const int cols = min(gn, (int)gridDim.x - grp * gn), r = wgid - grp * per;
    n0 = (grp * gn + r % cols) * BN;
    m0 = (r / cols) * BM;
  } else {
    n0 = (wgid % gridDim.x) * BN;
    m0 = (wgid / gridDim.x) * BM;
  }
  const int b = blockIdx.z;
  const float* A = p.A + (long)b * p.sA;
  const unsigned short* W = reinterpret_cast<const unsigned short*>(p.B) + (long)b * p.sB;

  floatx4 big[TM][TN], small[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] = small[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // unit u -> (row, quad q of 8): 8 consecutive lanes take 8 consecutive rows of one quad, a wave covers
  // 8 rows x 256 B of A (coalesced); LDS sub-slab q >> 2, quad q & 3: conflict-free ds_write_b128 groups
  auto unit = [](int u, int& row, int& q) {
    q = (u >> 3) & 7;
    row = (u & 7) + 8 * (u >> 6);
  };
  u32x4 ra[NA][2], rw[3][NB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int row, q;
      unit(tid + NT * i, row, q);
      const float* src = A + (long)min(m0 + row, p.M - 1) * p.lda + k0 + 8 * q;
      ra[i][0] = *reinterpret_cast<const u32x4*>(src);
      ra[i][1] = *reinterpret_cast<const u32x4*>(src + 4);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int row, q;
      unit(tid + NT * i, row, q);
      const unsigned short* src = W + (long)min(n0 + row, p.N - 1) * p.ldb + k0 + 8 * q;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) rw[pl][i] = *reinterpret_cast<const u32x4*>(src + pl * plane);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int row, q;
      unit(tid + NT * i, row, q);
      uint4* S = smem + (q >> 2) * SUB;
      uint4 h, m, l;
      split3_quad(__builtin_bit_cast(float4, ra[i][0]), __builtin_bit_cast(float4, ra[i][1]), h, m, l);
      S[0 * PA + (q & 3) * BM + row] = h;
      S[1 * PA + (q & 3) * BM + row] = m;
      S[2 * PA + (q & 3) * BM + row] = l;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int row, q;
      unit(tid + NT * i, row, q);
      uint4* S = smem + (q >> 2) * SUB;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) S[3 * PA + pl * PB + (q & 3) * BN + row] = __builtin_bit_cast(uint4, rw[pl][i]);
    }
  };
  auto compute = [&](const uint4* S) {   // form 8's 32-deep step
    const int q = lane >> 4;
    bf16x8_t bf[3][TN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[pl][j] = __builtin_bit_cast(bf16x8_t, S[3 * PA + pl * PB + q * BN + wn + 16 * j + (lane & 15)]);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      bf16x8_t af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        af[pl] = __builtin_bit_cast(bf16x8_t, S[pl * PA + q * BM + wm + 16 * i + (lane & 15)]);
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

  const int nk = p.K / 64;
  load(0);
  store();
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    load(64 * min(t + 1, nk - 1));   // unconditional (clamped re-read on the last slab)
    compute(smem);
    compute(smem + SUB);
    __syncthreads();
    store();
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] += small[i][j];
  store_tile_mf<16, TM, TN, BM, BN>(p, big, b, 0, m0, n0, wm, wn, lane);
}

}  // namespace

// C = epilogue(A . W^T) at fp32 accuracy with 64-deep K steps; W pre-split (dasa_f32_split3_bf16: d->B = hi
// plane, planes `plane` bf16 elements apart), A fp32. K % 64 == 0, lda % 4, ldb / plane % 8, 16-B aligned
// A / W. form 1 / 2 / 3 as above. Probe entry only (measured slower above: no plan routes here).
extern "C" int dasa_gemm_f32x6_k64(const dasa_gemm_desc* d, int64_t plane, int32_t form, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  if (M < 0 || N < 0 || K <= 0 || d->opA != 0 || d->opB != 1 || (K & 63) || (d->lda & 3) || (d->ldb & 7) ||
      (plane & 7) || d->lda < K || d->ldb < K || d->ldc < N || ((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15) ||
      (batch > 1 && ((d->strideA & 3) || (d->strideB & 7))) || form < 1 || form > 3)
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  GemmP p{};
  p.M = M; p.N = N; p.K = K; p.batch = batch; p.splitk = 1; p.kchunk = K;
  p.A = d->A; p.lda = d->lda; p.sA = d->strideA;
  p.B = d->B; p.ldb = d->ldb; p.sB = d->strideB;
  p.C = d->C; p.ldc = d->ldc; p.sC = d->strideC;
  p.bias = d->bias; p.act = d->act;
  p.aux = d->aux; p.ld_aux = d->ld_aux; p.sAux = d->strideAux;
  p.colscale = d->colscale; p.alpha = d->alpha; p.beta = d->beta;
  const int bm = form == 3 ? 64 : 128, bn = form == 2 ? 64 : 128;
  p.group_m = cdiv(M, bm) >= 8 ? -8 : 1;
  const dim3 grid((unsigned)cdiv(N, bn), (unsigned)cdiv(M, bm), batch);
  hipStream_t st = (hipStream_t)stream;
  switch (form) {
    case 1: hipLaunchKernelGGL((gemm_f32x6_k64_kernel<128, 128, 4, 2, 2>), grid, dim3(512), 0, st, p, (long)plane); break;
    case 2: hipLaunchKernelGGL((gemm_f32x6_k64_kernel<128, 64, 2, 2, 2>), grid, dim3(256), 0, st, p, (long)plane); break;
    default: hipLaunchKernelGGL((gemm_f32x6_k64_kernel<64, 128, 2, 2, 2>), grid, dim3(256), 0, st, p, (long)plane); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}
