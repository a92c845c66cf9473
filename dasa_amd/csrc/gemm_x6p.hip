// bf16x6 NT GEMM with BOTH operands pre-split into bf16 planes (probe form "P").
//
// gemm.hip's forms 8 / 20 stage A (fp32) through VGPRs, split it, and ds_write the planes: every wave of a
// workgroup reaches that split + ds_write + barrier phase together after each K step, 38-49 % of wave time
// parks at waitcnt / barrier and the MFMA pipe is 47-53 % busy (profiles/r05/x6_pmc/). Form 16 moved both
// operands to LDS-DMA but split A at fragment-read time (2x the split VALU, between the MFMAs): 0.80-0.90x.
// Here A arrives already split (the producer writes the planes: 6 B per element instead of 4), so a K step is
// a pure bf16 GEMM step over three planes per operand: every byte goes HBM / L2 -> LDS by
// global_load_lds_dwordx4 (no VGPR staging, no ds_write, no split VALU), one s_barrier per K step, and the
// MFMA loop is form 8's — same products, same order, same two accumulators: bitwise equal to form 8.
//   NSTAGE = 3: 128 x 128 tile, a ring of three 48 KB stages, DMAs two steps ahead (the guide's "glds with
//               stages in flight across the barrier": counted vmcnt, raw s_barrier);
//   NSTAGE = 2: 256 x 128 tile (form 7's 64 x 64 wave tiles), two 72 KB stages, one step ahead.
// LDS image per stage and operand: [plane][q][row] 16-B units (q = 8-bf16 K group), A planes then W planes:
// a DMA wave-instruction fills 64 consecutive rows of one (plane, q), the fragment read of lane l is unit
// (q = l >> 4, row l & 15) — conflict-free, as form 8.
#include "gemm_common.h"

namespace {

__device__ __forceinline__ void dma16(const void* g, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_base)
               : "memory", "m0");
}
__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(size_t)((const __attribute__((address_space(3))) void*)p);
}

// IMG = 1 (r06, forms 4 / 5): each plane image row-major, 128-row x 64-B rows of four 16-B K groups, group q
// of row r at slot q ^ ((r >> 2) & 3): a DMA wave-instruction fills 16 whole 64-B row slices (16 lines
// instead of 64), the fragment reads of a 16-lane group still hit 16 distinct bank slots.
__device__ __forceinline__ int pswz(int row) { return (row >> 2) & 3; }

template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTAGE, int IMG = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) __attribute__((amdgpu_waves_per_eu(1, 2)))
void gemm_f32x6_pp_kernel(GemmP p, long wplane, long aplane) {
  constexpr int NWV = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int PA = BM * 4, PB = BN * 4;                      // 16-B units per plane image
  constexpr int STAGE = 3 * (PA + PB);
  constexpr int IA = 3 * PA / 64 / NWV, IW = 3 * PB / 64 / NWV; // DMA wave-instructions per wave per stage
  static_assert(IA * 64 * NWV == 3 * PA && IW * 64 * NWV == 3 * PB && BM % 64 == 0 && BN % 64 == 0,
                "stage units must split evenly over the waves, 64 rows per instruction");
  static_assert(NSTAGE == 2 || IA + IW == 6, "the 3-stage vmcnt immediate below counts 6 DMAs per stage");
  __shared__ uint4 smem[NSTAGE * STAGE];   // ONE shared array (a second one can de-pipeline the DMA waits)

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
  const unsigned short* A = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* W = reinterpret_cast<const unsigned short*>(p.B);

  floatx4 big[TM][TN], small[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] = small[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-lane DMA sources (rows past M / N re-read the last row; their outputs are dropped) and the
  // wave-uniform LDS bases of its DMA slots in stage 0
  const unsigned short* asrc[IA];
  unsigned adst[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int u = (wave * IA + j) * 64 + lane, pl = u / PA, rem = u % PA;
    const int row = IMG ? rem / 4 : rem % BM, q = IMG ? (rem % 4) ^ pswz(row) : rem / BM;
    asrc[j] = A + pl * aplane + (long)min(m0 + row, p.M - 1) * p.lda + 8 * q;
    adst[j] = __builtin_amdgcn_readfirstlane(lds_u32(&smem[(wave * IA + j) * 64]));
  }
  const unsigned short* wsrc[IW];
  unsigned wdst[IW];
#pragma unroll
  for (int j = 0; j < IW; ++j) {
    const int u = (wave * IW + j) * 64 + lane, pl = u / PB, rem = u % PB;
    const int row = IMG ? rem / 4 : rem % BN, q = IMG ? (rem % 4) ^ pswz(row) : rem / BN;
    wsrc[j] = W + pl * wplane + (long)min(n0 + row, p.N - 1) * p.ldb + 8 * q;
    wdst[j] = __builtin_amdgcn_readfirstlane(lds_u32(&smem[3 * PA + (wave * IW + j) * 64]));
  }
  const int nk = p.K / 32;
  auto dma = [&](int stage, int t) {   // stage t's slice of this wave, unconditional (clamped re-read)
    const int k0 = 32 * min(t, nk - 1);
#pragma unroll
    for (int j = 0; j < IA; ++j) dma16(asrc[j] + k0, adst[j] + stage * STAGE * 16);
#pragma unroll
    for (int j = 0; j < IW; ++j) dma16(wsrc[j] + k0, wdst[j] + stage * STAGE * 16);
  };
  auto compute = [&](const uint4* S) {   // form 8's K step
    const int q = lane >> 4;
    bf16x8_t bf[3][TN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + 16 * j + (lane & 15);
        bf[pl][j] = __builtin_bit_cast(bf16x8_t, S[3 * PA + pl * PB + (IMG ? row * 4 + (q ^ pswz(row)) : q * BN + row)]);
      }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      bf16x8_t af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const int row = wm + 16 * i + (lane & 15);
        af[pl] = __builtin_bit_cast(bf16x8_t, S[pl * PA + (IMG ? row * 4 + (q ^ pswz(row)) : q * BM + row)]);
      }
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
  if constexpr (NSTAGE == 3) {
    dma(0, 0);
    dma(1, 1);
    int stage = 0;
    for (int t = 0; t < nk; ++t) {
      // own stage-t DMAs landed (stage t+1's 6 may still fly), then everyone's; stage t-1 is free again
      asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      dma(stage == 0 ? 2 : stage - 1, t + 2);
      compute(smem + stage * STAGE);
      stage = stage == 2 ? 0 : stage + 1;
    }
  } else {
    dma(0, 0);
    for (int t = 0; t < nk; ++t) {
      // stage t landed (own DMAs, then everyone's); everyone is done reading stage t-1, which t+1 refills
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      dma((t + 1) & 1, t + 1);
      compute(smem + (t & 1) * STAGE);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA into LDS outlives the workgroup
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] += small[i][j];
  store_tile_mf<16, TM, TN, BM, BN>(p, big, 0, 0, m0, n0, wm, wn, lane);
}

}  // namespace

// C = epilogue(A . W^T) at fp32 accuracy, A and W both as three bf16 planes (dasa_f32_split3_bf16 layout):
// d->A / d->B = the hi planes (bf16 elements, row strides lda / ldb), the mid / lo planes aplane / wplane
// elements further on. form 3: 128 x 128 tiles, three-stage DMA ring; form 2: 256 x 128, two stages; forms 4 / 5:
// forms 3 / 2 with the row-major plane images (IMG = 1).
// K % 32 == 0; lda, ldb, planes % 8 == 0; 16-B aligned planes; batch 1. Probe entry.
extern "C" int dasa_gemm_f32x6_pp(const dasa_gemm_desc* d, int64_t wplane, int64_t aplane, int32_t form,
                                  void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K;
  if (M <= 0 || N <= 0 || K <= 0 || d->opA != 0 || d->opB != 1 || d->batch > 1 || (K & 31) || (d->lda & 7) ||
      (d->ldb & 7) || (wplane & 7) || (aplane & 7) || d->lda < K || d->ldb < K || d->ldc < N ||
      ((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15) || form < 2 || form > 5)
    return (int)hipErrorInvalidValue;
  GemmP p{};
  p.M = M; p.N = N; p.K = K; p.batch = 1; p.splitk = 1; p.kchunk = K;
  p.A = d->A; p.lda = d->lda;
  p.B = d->B; p.ldb = d->ldb;
  p.C = d->C; p.ldc = d->ldc;
  p.bias = d->bias; p.act = d->act;
  p.aux = d->aux; p.ld_aux = d->ld_aux;
  p.colscale = d->colscale; p.alpha = d->alpha; p.beta = d->beta;
  const int bm = (form == 2 || form == 5) ? 256 : 128;
  p.group_m = cdiv(M, bm) >= 8 ? -8 : 1;
  const dim3 grid((unsigned)cdiv(N, 128), (unsigned)cdiv(M, bm), 1);
  hipStream_t st = (hipStream_t)stream;
  if (form == 2)
    hipLaunchKernelGGL((gemm_f32x6_pp_kernel<256, 128, 4, 2, 2>), grid, dim3(512), 0, st, p, (long)wplane, (long)aplane);
  else if (form == 3)
    hipLaunchKernelGGL((gemm_f32x6_pp_kernel<128, 128, 4, 2, 3>), grid, dim3(512), 0, st, p, (long)wplane, (long)aplane);
  else if (form == 5)
    hipLaunchKernelGGL((gemm_f32x6_pp_kernel<256, 128, 4, 2, 2, 1>), grid, dim3(512), 0, st, p, (long)wplane, (long)aplane);
  else
    hipLaunchKernelGGL((gemm_f32x6_pp_kernel<128, 128, 4, 2, 3, 1>), grid, dim3(512), 0, st, p, (long)wplane, (long)aplane);
  DASA_CHECK_LAUNCH();
  return 0;
}
