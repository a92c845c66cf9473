// fp32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32, exact f32 fma chain).
//
// Replaces the nn.Linear / torch.bmm calls of the reference policy (model.py SoftDot/Shift/LSTMCell
// projections, vilmodel.py BERT/LXRT projections and FFN, agent_dg.py:1519 DGAdaChannel.a_fc).
//
// Structure: 256-thread workgroup = 4 waves, block tile BM x BN x 32, each wave a WM x WN sub-tile of
// 32x32 MFMA accumulators. Operand tiles are staged k-major in LDS ([k][m], [k][n]) so that the MFMA
// operand read (lane l: row l&31, k-half l>>5) is a lane-contiguous ds_read_b32; two LDS buffers,
// next tile prefetched into registers while the current one feeds the MFMAs. Epilogue is fused
// (bias, activation, gate-multiply for DGAdaChannel, column scale for env-drop, beta accumulate).
// Split-K over gridDim.z with a deterministic fixed-order reduce for skinny (M<=64) decoder GEMMs.
#include "common.h"
#include <cstdlib>
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

// Load 4 consecutive floats starting at element `e` of a row (limit = first invalid element).
// VEC: the row base is 16-B aligned, so a whole in-range quad is one dwordx4 load.
template <bool VEC>
__device__ __forceinline__ float4 load4(const float* rowp, int e, int limit) {
  if (VEC && e + 3 < limit) return *reinterpret_cast<const float4*>(rowp + e);
  if (!VEC && e + 3 < limit) return make_float4(rowp[e], rowp[e + 1], rowp[e + 2], rowp[e + 3]);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e + 0 < limit) r.x = rowp[e + 0];
  if (e + 1 < limit) r.y = rowp[e + 1];
  if (e + 2 < limit) r.z = rowp[e + 2];
  return r;
}

constexpr int BKT = 32;   // default K tile (the BK = 64 configurations set their own)

// Component-wise select (a whole-float4 ternary is lowered through scratch memory by hipcc).
__device__ __forceinline__ float4 sel4(bool c, float4 v) {
  return make_float4(c ? v.x : 0.f, c ? v.y : 0.f, c ? v.z : 0.f, c ? v.w : 0.f);
}

// KC = operand stored with K contiguous ([rows][K]); else stored [K][rows].
// LDS images: KC -> [ROWS][BK] with the 16-B quads of each row XOR-swizzled by row (BK = 32: eight
// quads, two rows per 256-B bank row, swizzle (row>>1)&7; BK = 64: sixteen quads, one row per bank
// row, swizzle row&15), so the K-permuted ds_read_b128 fragment reads below hit 16 distinct bank
// slots in each of the instruction's four 16-lane groups; !KC -> [BK][ROWS + 4] (k-major, read one
// float per lane).
template <int BK>
__device__ __forceinline__ int qswz(int row) { return BK == 32 ? ((row >> 1) & 7) : (row & 15); }

template <int ROWS, bool KC, bool VEC, int NT, int BK>
struct TileLoader {
  static constexpr int BKT = BK;
  static constexpr int PAD = KC ? 0 : 4;
  static constexpr int LDS_FL = KC ? ROWS * BKT : BKT * (ROWS + PAD);
  static constexpr int TOTAL = ROWS * BKT / 4;   // float4 per tile
  static constexpr int NF4 = (TOTAL + NT - 1) / NT;
  static constexpr bool EXACT = (TOTAL % NT) == 0;
  float4 r[NF4];
  bool ok[NF4];

  __device__ __forceinline__ void load(const float* base, long ld, int r0, int rlimit, int k0, int klimit) {
    const int tid = threadIdx.x;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < NF4; ++i) {
      const int q = EXACT ? tid + NT * i : min(tid + NT * i, TOTAL - 1);   // surplus threads re-load a valid quad
      if (VEC) {
        // Unconditional, clamped loads; the range select is applied when the tile is written to LDS
        // (after the MFMAs), so the loads stay in flight across the compute of the current tile.
        // With K % 4 == 0 (VEC) a quad is either fully in range or fully out.
        if (KC) {
          const int row = q / (BKT / 4), kq = q % (BKT / 4);
          const int gr = r0 + row, gk = k0 + 4 * kq;
          r[i] = *reinterpret_cast<const float4*>(base + (long)min(gr, rlimit - 1) * ld + min(gk, klimit - 4));
          ok[i] = gr < rlimit && gk < klimit;
        } else {
          const int kr = q / (ROWS / 4), rq = q % (ROWS / 4);
          const int gk = k0 + kr, gr = r0 + 4 * rq;
          r[i] = *reinterpret_cast<const float4*>(base + (long)min(gk, klimit - 1) * ld + min(gr, rlimit - 4));
          ok[i] = gk < klimit && gr < rlimit;
        }
      } else if (KC) {
        const int row = q / (BKT / 4), kq = q % (BKT / 4);
        const int gr = r0 + row;
        r[i] = (gr < rlimit) ? load4<VEC>(base + (long)gr * ld, k0 + 4 * kq, klimit) : z;
        ok[i] = true;
      } else {
        const int kr = q / (ROWS / 4), rq = q % (ROWS / 4);
        const int gk = k0 + kr;
        r[i] = (gk < klimit) ? load4<VEC>(base + (long)gk * ld, r0 + 4 * rq, rlimit) : z;
        ok[i] = true;
      }
    }
  }
  __device__ __forceinline__ void store(float* S) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NF4; ++i) {
      const int q = tid + NT * i;
      if (!EXACT && q >= TOTAL) continue;
      const float4 v = sel4(ok[i], r[i]);
      if (KC) {
        const int row = q / (BKT / 4), kq = q % (BKT / 4);
        *reinterpret_cast<float4*>(S + row * BKT + 4 * (kq ^ qswz<BK>(row))) = v;
      } else {
        const int kr = q / (ROWS / 4), rq = q % (ROWS / 4);
        *reinterpret_cast<float4*>(S + kr * (ROWS + PAD) + 4 * rq) = v;
      }
    }
  }
  // Fragment of K-group s (k = 8s .. 8s+7) for MFMA row `row` of the 32x32x2 layout: lane half h
  // supplies k = 8s + 4h + e to MFMA e (e = 0..3). Both operands use the same permutation, so the
  // four MFMAs together accumulate exactly k = 8s .. 8s+7.
  __device__ __forceinline__ static float4 frag(const float* S, int row, int s, int h) {
    if (KC) {
      return *reinterpret_cast<const float4*>(S + row * BKT + 4 * ((2 * s + h) ^ qswz<BK>(row)));
    } else {
      const int k = 8 * s + 4 * h;
      return make_float4(S[(k + 0) * (ROWS + PAD) + row], S[(k + 1) * (ROWS + PAD) + row],
                         S[(k + 2) * (ROWS + PAD) + row], S[(k + 3) * (ROWS + PAD) + row]);
    }
  }
};

__device__ __forceinline__ float f4get(const float4& v, int e) {
  return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

// KW > 1 splits every 32-deep K-tile between KW wave groups that own the same output sub-tiles
// (in-block split-K): more waves per block for mid-size GEMMs, reduced through LDS at the end.
template <int BM, int BN, int WM, int WN, int KW, bool AKC, bool BKC, bool VEC, int BKT>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN) * KW) void gemm_f32_kernel(GemmP p) {
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int WAVES_N = BN / WN;
  constexpr int NWG = (BM / WM) * (BN / WN);
  constexpr int NT = 64 * NWG * KW;
  constexpr int NGRP = BKT / 8;                 // K-groups of 8 per tile
  static_assert(NGRP % KW == 0, "K-split must divide the K tile");
  constexpr int GPW = NGRP / KW;                // K-groups per wave group
  constexpr int PH = GPW < 4 ? GPW : 4;         // K-groups per fragment-read phase
  using LA = TileLoader<BM, AKC, VEC, NT, BKT>;
  using LB = TileLoader<BN, BKC, VEC, NT, BKT>;
  // one LDS array: the A/B double buffers, reused by the K-split reduction after the main loop
  constexpr int A_FL = 2 * LA::LDS_FL, B_FL = 2 * LB::LDS_FL;
  constexpr int RED_FL = (KW - 1) * BM * BN;
  constexpr int SMEM_FL = (A_FL + B_FL) > RED_FL ? (A_FL + B_FL) : RED_FL;
  __shared__ __attribute__((aligned(16))) float smem[SMEM_FL];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kgrp = wave / NWG, wt = wave % NWG;
  const int wm = (wt / WAVES_N) * WM, wn = (wt % WAVES_N) * WN;
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so give each XCD a
  // contiguous run of row-major tiles (shared A row panels and B column panels in its own L2).
  // Bijective for any tile count (q = n/8 tiles per XCD, the first n%8 XCDs take one more).
  int n0, m0;
  {
    const int gx = gridDim.x, nwg = gx * gridDim.y;
    const int orig = blockIdx.y * gx + blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    n0 = (wgid % gx) * BN;
    m0 = (wgid / gx) * BM;
  }
  const int b = blockIdx.z / p.splitk, split = blockIdx.z % p.splitk;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const float* A = p.A + (long)b * p.sA;
  const float* B = p.B + (long)b * p.sB;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Two register sets in a ring: the global loads of tile t+2 are issued at the top of step t and
  // written to LDS at the end of step t+1, so each load has two MFMA phases to land.
  LA la0, la1;
  LB lb0, lb1;
  const int ntiles = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;
  if (ntiles > 0) {
    la0.load(A, p.lda, m0, p.M, kbeg, kend);
    lb0.load(B, p.ldb, n0, p.N, kbeg, kend);
    const int k1 = kbeg + min(1, ntiles - 1) * BKT;
    la1.load(A, p.lda, m0, p.M, k1, kend);
    lb1.load(B, p.ldb, n0, p.N, k1, kend);
    la0.store(smem);
    lb0.store(smem + A_FL);
    __syncthreads();
  }
  const int hl = lane >> 5, rl = lane & 31;
  // step t: X = the free register set (receives tile t+2), Y = the set holding tile t+1
  auto step = [&](int t, LA& xa, LB& xb, LA& ya, LB& yb) {
    const int buf = t & 1;
    {  // unconditional (clamped to the last tile): a conditional issue makes hipcc's vmcnt counts
       // assume the no-load path and wait for the just-issued loads before the LDS write below
      const int k0 = kbeg + min(t + 2, ntiles - 1) * BKT;
      xa.load(A, p.lda, m0, p.M, k0, kend);
      xb.load(B, p.ldb, n0, p.N, k0, kend);
    }
    const float* As = smem + buf * LA::LDS_FL;
    const float* Bs = smem + A_FL + buf * LB::LDS_FL;
    // fragments of up to 4 K-groups first, then their MFMAs (the reads overlap the MACs)
#pragma unroll
    for (int g0 = 0; g0 < GPW; g0 += PH) {
      float4 af[PH][TM], bf[PH][TN];
#pragma unroll
      for (int g = 0; g < PH; ++g) {
        const int s = kgrp * GPW + g0 + g;
#pragma unroll
        for (int i = 0; i < TM; ++i) af[g][i] = LA::frag(As, wm + i * 32 + rl, s, hl);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[g][j] = LB::frag(Bs, wn + j * 32 + rl, s, hl);
      }
      // keep the fragment reads ahead of the MFMAs: hipcc otherwise re-uses one register set and
      // serialises read -> lgkmcnt(0) -> 4 MFMAs per K-group, exposing the LDS latency each time
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < PH; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(af[g][i], e), f4get(bf[g][j], e),
                                                               acc[i][j], 0, 0, 0);
    }
    ya.store(smem + (buf ^ 1) * LA::LDS_FL);   // past the last tile this writes an unused buffer
    yb.store(smem + A_FL + (buf ^ 1) * LB::LDS_FL);
    __syncthreads();
  };
  // steps in pairs with the odd step unconditional, so both paths into the loop header carry the
  // same pending loads (a skippable odd step makes hipcc drain vmcnt(0) at the header)
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {
    step(t, la0, lb0, la1, lb1);
    step(t + 1, la1, lb1, la0, lb0);
  }
  if (t < ntiles) step(t, la0, lb0, la1, lb1);

  if (KW > 1) {   // fold the K-split wave groups into group 0 through LDS
    float* red = smem;
    __syncthreads();
    if (kgrp > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            red[((((kgrp - 1) * NWG + wt) * TM + i) * TN + j) * 1024 + r * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (kgrp > 0) return;
#pragma unroll
    for (int g = 1; g < KW; ++g)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            acc[i][j][r] += red[((((g - 1) * NWG + wt) * TM + i) * TN + j) * 1024 + r * 64 + lane];
  }
  // C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // Epilogue: every optional operand is fetched with unconditional clamped loads inside ONE uniform
  // branch per operand (a per-element branch around a load makes hipcc wait vmcnt(0) per element).
  const bool full_tile = (m0 + BM <= p.M) && (n0 + BN <= p.N);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + j * 32 + rl;
    const int colc = min(col, p.N - 1);
    float bj = 0.f, cs = 1.f;
    if (p.splitk == 1) {
      if (p.bias) bj = p.bias[colc];
      if (p.colscale) cs = p.colscale[colc];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rbase = m0 + wm + i * 32 + 4 * hl;
      if (p.splitk > 1) {
        float* ws = p.ws + ((long)split * p.batch + b) * p.M * p.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (full_tile || (row < p.M && col < p.N)) ws[(long)row * p.N + col] = acc[i][j][r];
        }
        continue;
      }
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = p.alpha * acc[i][j][r] + bj;
      switch (p.act) {   // one uniform branch per tile, not per element
        case DASA_ACT_RELU:
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = fmaxf(v[r], 0.f);
          break;
        case DASA_ACT_GELU:
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = gelu_erf(v[r]);
          break;
        case DASA_ACT_TANH:
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = tanhf(v[r]);
          break;
        case DASA_ACT_SIGMOID:
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = sigmoidf_(v[r]);
          break;
        default:
          break;
      }
      if (p.aux) {
        const float* ab = p.aux + (long)b * p.sAux;
        float av[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(rbase + (r & 3) + 8 * (r >> 2), p.M - 1);
          av[r] = ab[(long)row * p.ld_aux + colc];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= av[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] *= cs;
      float* cb = p.C + (long)b * p.sC;
      if (p.beta != 0.f) {
        float cv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(rbase + (r & 3) + 8 * (r >> 2), p.M - 1);
          cv[r] = cb[(long)row * p.ldc + colc];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] += p.beta * cv[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (full_tile || (row < p.M && col < p.N)) cb[(long)row * p.ldc + col] = v[r];
      }
    }
  }
}

__global__ void splitk_reduce_kernel(GemmP p) {
  const long total = (long)p.batch * p.M * p.N;
  const long slab = total;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < p.splitk; ++k) s += p.ws[k * slab + idx];
    const int col = (int)(idx % p.N);
    const long t = idx / p.N;
    const int row = (int)(t % p.M);
    const int b = (int)(t / p.M);
    epilogue_store(p, b, row, col, s);
  }
}

template <int BM, int BN, int WM, int WN, int KW, bool VEC, int BK = 32>
int launch_tile(const GemmP& p, int opA, int opB, hipStream_t st) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, p.batch * p.splitk);
  dim3 block(64 * (BM / WM) * (BN / WN) * KW);
  const bool akc = (opA == 0), bkc = (opB == 1);
  if (akc && bkc) hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, KW, true, true, VEC, BK>), grid, block, 0, st, p);
  else if (akc && !bkc) hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, KW, true, false, VEC, BK>), grid, block, 0, st, p);
  else if (!akc && bkc) hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, KW, false, true, VEC, BK>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, KW, false, false, VEC, BK>), grid, block, 0, st, p);
  DASA_CHECK_LAUNCH();
  return 0;
}

// Tile configurations: {BM, BN, WM, WN, KW}
struct TileCfg { int bm, bn, wm, wn, kw; };
constexpr TileCfg kCfgs[] = {
    {128, 128, 64, 64, 1},  // 0: large GEMMs
    {64, 128, 32, 64, 1},   // 1
    {64, 64, 32, 32, 1},    // 2
    {32, 128, 32, 32, 1},   // 3: skinny M
    {64, 64, 32, 32, 2},    // 4: mid-size, 8 waves
    {32, 64, 32, 32, 2},    // 5: mid-size, many small blocks
    {128, 64, 64, 32, 1},   // 6
    {64, 128, 32, 64, 2},   // 7
    {128, 128, 64, 64, 2},  // 8
    {32, 64, 32, 32, 4},    // 9
    {64, 32, 32, 32, 2},    // 10
    {64, 64, 32, 32, 2},    // 11: BK = 64
    {32, 64, 32, 32, 2},    // 12: BK = 64
    {128, 64, 64, 32, 1},   // 13: BK = 64
    {64, 128, 32, 64, 2},   // 14: BK = 64
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

int launch_cfg(int cfg, bool vec, const GemmP& p, int opA, int opB, hipStream_t st) {
  if (!vec) {
    return kCfgs[cfg].bm == 32 ? launch_tile<32, 128, 32, 32, 1, false>(p, opA, opB, st)
                               : launch_tile<64, 64, 32, 32, 1, false>(p, opA, opB, st);
  }
  switch (cfg) {
    case 0: return launch_tile<128, 128, 64, 64, 1, true>(p, opA, opB, st);
    case 1: return launch_tile<64, 128, 32, 64, 1, true>(p, opA, opB, st);
    case 2: return launch_tile<64, 64, 32, 32, 1, true>(p, opA, opB, st);
    case 3: return launch_tile<32, 128, 32, 32, 1, true>(p, opA, opB, st);
    case 4: return launch_tile<64, 64, 32, 32, 2, true>(p, opA, opB, st);
    case 5: return launch_tile<32, 64, 32, 32, 2, true>(p, opA, opB, st);
    case 6: return launch_tile<128, 64, 64, 32, 1, true>(p, opA, opB, st);
    case 7: return launch_tile<64, 128, 32, 64, 2, true>(p, opA, opB, st);
    case 8: return launch_tile<128, 128, 64, 64, 2, true>(p, opA, opB, st);
    case 9: return launch_tile<32, 64, 32, 32, 4, true>(p, opA, opB, st);
    case 10: return launch_tile<64, 32, 32, 32, 2, true>(p, opA, opB, st);
    case 11: return launch_tile<64, 64, 32, 32, 2, true, 64>(p, opA, opB, st);
    case 12: return launch_tile<32, 64, 32, 32, 2, true, 64>(p, opA, opB, st);
    case 13: return launch_tile<128, 64, 64, 32, 1, true, 64>(p, opA, opB, st);
    default: return launch_tile<64, 128, 32, 64, 2, true, 64>(p, opA, opB, st);
  }
}

inline long cdiv(long a, long b) { return (a + b - 1) / b; }

}  // namespace

struct Plan { int cfg, splitk, kchunk; int64_t ws; };

static int g_force_cfg = -2;   // DASA_GEMM_CFG=<index> pins a tile config (tuning sweeps)

static Plan make_plan(const dasa_gemm_desc* d) {
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  if (g_force_cfg == -2) {
    const char* e = getenv("DASA_GEMM_CFG");
    g_force_cfg = e ? atoi(e) : -1;
  }
  auto tiles = [&](int bm, int bn) { return cdiv(M, bm) * cdiv(N, bn) * batch; };
  Plan pl;
  // Tile choice (DESIGN.md "GEMM"), fitted to the MI355X (config x split-K) grid over the policy's
  // GEMM shapes in profiles/r01/gemm_grid_v3.txt: 8-wave 64x64 tiles (in-block K split) for large and
  // long-K problems, 32x64 tiles for mid-size ones, split-K when there are too few tiles to fill the
  // 256 CUs; the skinny decoder GEMMs (M <= 32) are weight-streaming and split K widely.
  const long t64 = tiles(64, 64);
  if (M <= 32) pl.cfg = 5;
  else if (d->opA == 1 && K >= 8192 && t64 >= 256) pl.cfg = 8;   // weight grads over many rows
  else if (t64 >= 2048) pl.cfg = 6;                              // profiles/r01/gemm_grid_v4.txt
  else if (t64 >= 800) pl.cfg = 4;
  else if (t64 >= 400) pl.cfg = (t64 >= 500 && K < 1536) ? 5 : 4;
  else if (t64 >= 250 && (K < 1536 || t64 >= 320)) pl.cfg = 5;
  else pl.cfg = 4;
  const int fcfg = g_force_cfg >= 0 ? g_force_cfg % 64 : -1, fsplit = g_force_cfg >= 0 ? g_force_cfg / 64 : 0;
  if (fcfg >= 0 && fcfg < kNumCfgs) pl.cfg = fcfg;
  const int bm = kCfgs[pl.cfg].bm, bn = kCfgs[pl.cfg].bn;
  const long blocks = tiles(bm, bn);
  int splitk = 1;
  if (M <= 32) {
    if (blocks < 160 && K >= 512) {
      splitk = (int)cdiv(256, blocks);
      const int maxs = K / 256;  // keep >= 8 K-tiles per split
      if (splitk > maxs) splitk = maxs;
      if (splitk > 16) splitk = 16;
      if (splitk < 1) splitk = 1;
    }
  } else if (blocks < 400 && K >= 1536) {
    splitk = (int)((K + 384) / 768);
    if (splitk > (blocks < 200 ? 3 : 4)) splitk = blocks < 200 ? 3 : 4;
  }
  if (fsplit > 0) splitk = fsplit;
  int kchunk = (int)(cdiv(cdiv(K, splitk), 64) * 64);   // a whole number of K tiles for BK 32 and 64
  if (kchunk < 64) kchunk = 64;
  splitk = K > 0 ? (int)cdiv(K, kchunk) : 1;
  pl.splitk = splitk;
  pl.kchunk = kchunk;
  pl.ws = splitk > 1 ? (int64_t)splitk * batch * M * N * (int64_t)sizeof(float) : 0;
  return pl;
}

extern "C" int dasa_gemm_force_config(int cfg) {
  g_force_cfg = cfg;
  return kNumCfgs;
}

extern "C" int64_t dasa_gemm_f32_workspace(const dasa_gemm_desc* d) {
  if (!d || d->M < 0 || d->N < 0 || d->K < 0) return 0;
  return make_plan(d).ws;
}

extern "C" int dasa_gemm_f32(const dasa_gemm_desc* d, void* ws, int64_t ws_bytes, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  Plan pl = make_plan(d);
  if (pl.splitk > 1 && (ws == nullptr || ws_bytes < pl.ws)) {  // no workspace: single pass
    pl.splitk = 1;
    pl.kchunk = K > 0 ? (int)(cdiv(K, 64) * 64) : 64;
  }
  if (M == 0 || N == 0) return 0;
  // float4 operand loads need 16-B aligned rows; anything else takes the scalar-load variant
  const uintptr_t am = (uintptr_t)d->A | (uintptr_t)d->B;
  // VEC also needs the contiguous extent of each operand to be a multiple of 4 (K for K-contiguous
  // operands, M / N for the transposed ones) so that quads never straddle the edge.
  const bool ext4 = (K & 3) == 0 && (d->opA == 0 || (M & 3) == 0) && (d->opB == 1 || (N & 3) == 0);
  const bool vec = ext4 && !((am & 15) || (d->lda & 3) || (d->ldb & 3) ||
                             (batch > 1 && ((d->strideA & 3) || (d->strideB & 3))));
  if (d->opA == 0 ? d->lda < K : d->lda < M) return (int)hipErrorInvalidValue;
  if (d->opB == 1 ? d->ldb < K : d->ldb < N) return (int)hipErrorInvalidValue;
  if (d->ldc < N) return (int)hipErrorInvalidValue;

  GemmP p;
  p.M = M; p.N = N; p.K = K; p.batch = batch; p.splitk = pl.splitk; p.kchunk = pl.kchunk;
  p.A = d->A; p.lda = d->lda; p.sA = d->strideA;
  p.B = d->B; p.ldb = d->ldb; p.sB = d->strideB;
  p.C = d->C; p.ldc = d->ldc; p.sC = d->strideC;
  p.bias = d->bias; p.act = d->act;
  p.aux = d->aux; p.ld_aux = d->ld_aux; p.sAux = d->strideAux;
  p.colscale = d->colscale; p.alpha = d->alpha; p.beta = d->beta;
  p.ws = (float*)ws;
  hipStream_t st = (hipStream_t)stream;
  int rc;
  rc = launch_cfg(pl.cfg, vec, p, d->opA, d->opB, st);
  if (rc) return rc;
  if (pl.splitk > 1) {
    const long total = (long)batch * M * N;
    int grid = (int)cdiv(total, 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, p);
    DASA_CHECK_LAUNCH();
  }
  return 0;
}
