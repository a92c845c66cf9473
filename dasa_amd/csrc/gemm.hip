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
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "../../include/dasa_hip.h"
#include "gemm_common.h"

namespace {


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


template <int TM, int TN, int BM, int BN>
__device__ __forceinline__ void store_tile(const GemmP& p, floatx16 (&acc)[TM][TN], int b, int split, int m0,
                                           int n0, int wm, int wn, int lane) {
  store_tile_mf<32, TM, TN, BM, BN>(p, acc, b, split, m0, n0, wm, wn, lane);
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

  const bool owner = KW == 1 || kgrp == 0;   // the waves holding the block's result after the K-split fold
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
    if (owner) {
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
  }
  if (p.splitk > 1 && p.cnt) {
    // in-kernel split-K reduction (no second launch): each split stores its raw tile write-through (sc1)
    // into its own slab; the last split to take the tile's ticket sums the slabs in split order
    // (deterministic; the same sums as splitk_reduce_kernel) and runs the fused epilogue
    __shared__ int s_last;
    constexpr int SLAB_B = BM * BN * 4, NO = 64 * NWG;
    const int tile = (b * (int)gridDim.y + m0 / BM) * (int)gridDim.x + n0 / BN;
    const int to = wt * 64 + lane;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.ws, 0, 0x7fffffff, 0x00020000);
    const long tbase = (long)tile * p.splitk;
    if (owner) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int off = (int)((tbase + split) * SLAB_B) + (((i * TN + j) * 4 + r4) * NO + to) * 16;
            const u32x4 u = {__float_as_uint(acc[i][j][4 * r4]), __float_as_uint(acc[i][j][4 * r4 + 1]),
                             __float_as_uint(acc[i][j][4 * r4 + 2]), __float_as_uint(acc[i][j][4 * r4 + 3])};
            __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);   // sc1: write-through
          }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(p.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)(p.splitk - 1);
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) __hip_atomic_store(p.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: sc1 loads below the ticket
    if (!owner) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int s2 = 0; s2 < p.splitk; ++s2) {     // fixed order: deterministic whoever arrives last
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int off = (int)((tbase + s2) * SLAB_B) + (((i * TN + j) * 4 + r4) * NO + to) * 16;
            const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);   // sc1
            acc[i][j][4 * r4] += __uint_as_float(u.x);
            acc[i][j][4 * r4 + 1] += __uint_as_float(u.y);
            acc[i][j][4 * r4 + 2] += __uint_as_float(u.z);
            acc[i][j][4 * r4 + 3] += __uint_as_float(u.w);
          }
    }
    GemmP q = p;
    q.splitk = 1;
    store_tile<TM, TN, BM, BN>(q, acc, b, 0, m0, n0, wm, wn, lane);
    return;
  }
  if (owner) store_tile<TM, TN, BM, BN>(p, acc, b, split, m0, n0, wm, wn, lane);
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

// ---- NT GEMM with LDS-DMA staging (C = A[M,K] . B[N,K]^T, both operands K-contiguous) ----------
// The nn.Linear forward shape (x . W^T), which carries most of the policy's FLOPs. Operand tiles
// (rows x 32 floats = 128-B rows) are moved HBM/L2 -> LDS by global_load_lds_dwordx4 (1 KiB per
// wave-instruction: 8 rows x 8 quads, lane-linear in LDS), so staging costs no VGPRs and no
// ds_write pass. The LDS image keeps the XOR swizzle of TileLoader<KC, BK=32> (quad q of row r at
// slot q ^ ((r>>1)&7)) by permuting the per-lane SOURCE address; the fragment reads apply the same
// involution. Two stages: tile t+1 is in flight while tile t feeds the MFMAs; one vmcnt(0) +
// barrier per 32-deep K-tile. Requires K (and the split-K chunk) % 32 == 0, 16-B aligned rows.
template <int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_nt_glds_kernel(GemmP p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int IA = BM / 8 / NW, IB = BN / 8 / NW;       // 1-KiB glds instructions per wave per stage
  static_assert(IA * 8 * NW == BM && IB * 8 * NW == BN, "tile rows must split into 8-row pieces per wave");
  constexpr int A_FL = BM * 32, B_FL = BN * 32, STAGE_FL = A_FL + B_FL;
  __shared__ __attribute__((aligned(1024))) float smem[2 * STAGE_FL];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
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
  const int ntiles = kend > kbeg ? (kend - kbeg) / 32 : 0;

  // per-lane source rows (clamped: rows past M / N re-read the last row; their outputs are dropped)
  const float* srcA[IA];
  const float* srcB[IB];
  {
    const int rsub = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int R = 8 * (wave * IA + j) + rsub;
      const int qd = slot ^ ((R >> 1) & 7);
      srcA[j] = p.A + (long)b * p.sA + (long)min(m0 + R, p.M - 1) * p.lda + kbeg + 4 * qd;
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int R = 8 * (wave * IB + j) + rsub;
      const int qd = slot ^ ((R >> 1) & 7);
      srcB[j] = p.B + (long)b * p.sB + (long)min(n0 + R, p.N - 1) * p.ldb + kbeg + 4 * qd;
    }
  }
  auto stage = [&](int st, int t) {
    float* base = smem + st * STAGE_FL;
    const int ko = 32 * t;
#pragma unroll
    for (int j = 0; j < IA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + ko),
                                       (__attribute__((address_space(3))) void*)(base + (wave * IA + j) * 256),
                                       16, 0, 0);
#pragma unroll
    for (int j = 0; j < IB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + ko),
                                       (__attribute__((address_space(3))) void*)(base + A_FL + (wave * IB + j) * 256),
                                       16, 0, 0);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int hl = lane >> 5, rl = lane & 31;
  if (ntiles > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const float* As = smem + cur * STAGE_FL;
    const float* Bs = As + A_FL;
    // every fragment of this K-tile is read BEFORE the next tile's LDS-DMA is issued: a ds_read
    // after an in-flight glds into the same array makes hipcc drain vmcnt(0) first
    float4 af[4][TM], bf[4][TN];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int q = 2 * g + hl;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm + i * 32 + rl;
        af[g][i] = *reinterpret_cast<const float4*>(As + row * 32 + 4 * (q ^ ((row >> 1) & 7)));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + j * 32 + rl;
        bf[g][j] = *reinterpret_cast<const float4*>(Bs + row * 32 + 4 * (q ^ ((row >> 1) & 7)));
      }
    }
    if (t + 1 < ntiles) stage(cur ^ 1, t + 1);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(af[g][i], e), f4get(bf[g][j], e),
                                                             acc[i][j], 0, 0, 0);
    // keep the MFMAs ahead of the wait: hipcc otherwise sinks them past the barrier, so the wait
    // for tile t+1's DMA would sit in front of tile t's MFMAs instead of behind them
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  store_tile<TM, TN, BM, BN>(p, acc, b, split, m0, n0, wm, wn, lane);
}

// ---- NT GEMM, 64-deep K tiles (C = A[M,K] . B[N,K]^T, both operands K-contiguous) --------------
// BK = 64 floats (256-B LDS rows, quad q of row r stored at slot q ^ (r & 15): the 16-lane groups
// of a ds_read_b128 fragment read hit 16 distinct slots). Tile t+1 is loaded into registers while
// tile t feeds the MFMAs; NSTAGE = 1 keeps one LDS image (write after a barrier, 2 barriers per
// tile, ~64 KiB at 128x128 so two workgroups share a CU), NSTAGE = 2 double-buffers it (1 barrier).
// MF = 16 uses v_mfma_f32_16x16x4_f32 (4 lane groups carry 4 k each: group g supplies
// k = 16s + 4g + e to MFMA e), MF = 32 uses v_mfma_f32_32x32x2_f32 (halves h: k = 8s + 4h + e).
// Requires K (and the split-K chunk) % 64 == 0 and 16-B aligned rows.
//
// SK = stream-K: a grid of G <= #CUs workgroups. The first sk_dp tiles are dealt whole (tile lw,
// lw + G, ...); the MAC iterations (64-deep K steps) of the remaining tiles are split evenly over
// the G workgroups, so every CU gets the same work whatever the tile count. A tile finished in
// one piece is stored directly; pieces of a split tile are stored write-through (sc1) to a slab per
// (workgroup, first|last piece) and the LAST piece to arrive (agent-scope ticket on the tile's
// counter, re-armed to 0) sums all pieces in workgroup order (deterministic) and runs the epilogue.
// No workgroup ever waits for another, so residency is never assumed.
struct SkP { int grid, dp, tiles, ipt, tiles_n, tiles_mn; unsigned* cnt; float* slab; };


template <int BM, int BN, int WAVES_M, int WAVES_N, int MF, int NSTAGE, bool SK, int BK = 64>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_nt_k64_kernel(GemmP p, SkP sk) {
  static_assert(BK == 64 || (BK == 32 && MF == 16), "BK 32 tiles use the 16x16x4 fragment map");
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / MF, TN = WN / MF;
  constexpr int A_FL = BM * BK, B_FL = BN * BK, STAGE_FL = A_FL + B_FL;
  constexpr int KG = MF == 32 ? BK / 8 : BK / 16;       // K-groups (one float4 per lane) per tile
  using AccT = typename std::conditional<MF == 32, floatx16, floatx4>::type;
  constexpr int NR = MF == 32 ? 16 : 4;
  __shared__ __attribute__((aligned(16))) float smem[NSTAGE * STAGE_FL];
  __shared__ int s_last;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  using LA = TileLoader<BM, true, true, NT, BK>;
  using LB = TileLoader<BN, true, true, NT, BK>;
  LA la;
  LB lb;
  AccT acc[TM][TN];
  const int fr = MF == 32 ? (lane & 31) : (lane & 15);   // fragment row within an MF tile
  const int fg = MF == 32 ? (lane >> 5) : (lane >> 4);   // lane group: which 4 k of a K-group

  auto compute = [&](const float* S) {
    const float* As = S;
    const float* Bs = S + A_FL;
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int q = (MF == 32 ? 2 : 4) * g + fg;
      float4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm + i * MF + fr;
        af[i] = *reinterpret_cast<const float4*>(As + row * BK + 4 * (q ^ qswz<BK>(row)));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + j * MF + fr;
        bf[j] = *reinterpret_cast<const float4*>(Bs + row * BK + 4 * (q ^ qswz<BK>(row)));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (MF == 32)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(af[i], e), f4get(bf[j], e), acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(af[i], e), f4get(bf[j], e), acc[i][j], 0, 0, 0);
          }
    }
  };
  // acc = A[m0.., kbeg..kbeg+64n) . B[n0.., same]^T. Starts and ends with every wave past a barrier,
  // so consecutive calls may restage the LDS image at once.
  auto mac = [&](const float* Ab, const float* Bb, int m0, int n0, int kbeg, int ntiles) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;
    if (ntiles <= 0) return;
    const int kend = kbeg + BK * ntiles;
    la.load(Ab, p.lda, m0, p.M, kbeg, kend);
    lb.load(Bb, p.ldb, n0, p.N, kbeg, kend);
    la.store(smem);
    lb.store(smem + A_FL);
    __syncthreads();
    // Unconditional staging (the last step re-loads the last tile into a buffer nobody reads): a
    // conditional load leaves the staging registers live across a branch and hipcc moves them to
    // scratch memory.
    for (int t = 0; t < ntiles; ++t) {
      {
        const int k0 = kbeg + BK * min(t + 1, ntiles - 1);
        la.load(Ab, p.lda, m0, p.M, k0, kend);
        lb.load(Bb, p.ldb, n0, p.N, k0, kend);
      }
      float* cur = smem + (NSTAGE == 2 ? (t & 1) * STAGE_FL : 0);
      compute(cur);
      if (NSTAGE == 2) {
        la.store(smem + ((t + 1) & 1) * STAGE_FL);
        lb.store(smem + ((t + 1) & 1) * STAGE_FL + A_FL);
        __syncthreads();
      } else {
        __syncthreads();
        la.store(smem);
        lb.store(smem + A_FL);
        __syncthreads();
      }
    }
  };

  if constexpr (!SK) {
    const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    int n0, m0;
    if (p.group_m > 1) {
      // L2-grouped order: consecutive tiles of one XCD walk group_m row panels column by column, so
      // the workgroups resident on an XCD share a few A row panels and B column panels in its L2
      const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
      const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
      m0 = (grp * gm + r % rows) * BM;
      n0 = (r / rows) * BN;
    } else {
      n0 = (wgid % gridDim.x) * BN;
      m0 = (wgid / gridDim.x) * BM;
    }
    const int b = blockIdx.z / p.splitk, split = blockIdx.z % p.splitk;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    mac(p.A + (long)b * p.sA, p.B + (long)b * p.sB, m0, n0, kbeg, kend > kbeg ? (kend - kbeg) / BK : 0);
    store_tile_mf<MF, TM, TN, BM, BN>(p, acc, b, split, m0, n0, wm, wn, lane);
  } else {
    const int G = sk.grid, lw = xcd_remap(blockIdx.x, G), ipt = sk.ipt;
    auto tile_at = [&](int T, int& b, int& m0, int& n0) {
      b = T / sk.tiles_mn;
      const int r = T - b * sk.tiles_mn;
      m0 = (r / sk.tiles_n) * BM;
      n0 = (r % sk.tiles_n) * BN;
    };
    for (int T = lw; T < sk.dp; T += G) {     // whole tiles
      int b, m0, n0;
      tile_at(T, b, m0, n0);
      mac(p.A + (long)b * p.sA, p.B + (long)b * p.sB, m0, n0, 0, ipt);
      store_tile_mf<MF, TM, TN, BM, BN>(p, acc, b, 0, m0, n0, wm, wn, lane);
    }
    const long I = (long)(sk.tiles - sk.dp) * ipt;     // split iterations, I >= G (host guarantees)
    auto start_of = [&](int w) { return (long)w * I / G; };
    auto owner_of = [&](long i) { return (int)(((i + 1) * G + I - 1) / I - 1); };
    long it = start_of(lw);
    const long end = start_of(lw + 1);
    const int first_tile = (int)(it / ipt);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sk.slab, 0, 0x7fffffff, 0x00020000);
    constexpr int SLAB_B = BM * BN * 4;
    while (it < end) {
      const int Ts = (int)(it / ipt), kt0 = (int)(it % ipt);
      const int kt1 = (int)min((long)ipt, kt0 + (end - it));
      int b, m0, n0;
      tile_at(sk.dp + Ts, b, m0, n0);
      mac(p.A + (long)b * p.sA, p.B + (long)b * p.sB, m0, n0, BK * kt0, kt1 - kt0);
      if (kt0 == 0 && kt1 == ipt) {
        store_tile_mf<MF, TM, TN, BM, BN>(p, acc, b, 0, m0, n0, wm, wn, lane);
      } else {
        const int slot = 2 * lw + (Ts == first_tile ? 0 : 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r4 = 0; r4 < NR / 4; ++r4) {
              const int off = slot * SLAB_B + (((i * TN + j) * (NR / 4) + r4) * NT + tid) * 16;
              const u32x4 u = {__float_as_uint(acc[i][j][4 * r4]), __float_as_uint(acc[i][j][4 * r4 + 1]),
                               __float_as_uint(acc[i][j][4 * r4 + 2]), __float_as_uint(acc[i][j][4 * r4 + 3])};
              __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);   // sc1: write-through
            }
        const long ia = (long)Ts * ipt;
        const int w0 = owner_of(ia), w1 = owner_of(ia + ipt - 1);
        // ticket: every wave's write-through stores have landed before one lane takes it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
          s_last = __hip_atomic_fetch_add(sk.cnt + Ts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (unsigned)(w1 - w0);
        __syncthreads();
        if (s_last) {
          if (tid == 0) __hip_atomic_store(sk.cnt + Ts, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: sc1 loads below the ticket
          // every piece (this workgroup's own included) is re-read from its slab and summed into the
          // accumulator registers in workgroup order
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;
          for (int w = w0; w <= w1; ++w) {      // fixed order: deterministic whoever arrives last
            const int ws = 2 * w + ((long)Ts == start_of(w) / ipt ? 0 : 1);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r4 = 0; r4 < NR / 4; ++r4) {
                  const int off = ws * SLAB_B + (((i * TN + j) * (NR / 4) + r4) * NT + tid) * 16;
                  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);   // sc1
                  acc[i][j][4 * r4] += __uint_as_float(u.x);
                  acc[i][j][4 * r4 + 1] += __uint_as_float(u.y);
                  acc[i][j][4 * r4 + 2] += __uint_as_float(u.z);
                  acc[i][j][4 * r4 + 3] += __uint_as_float(u.w);
                }
          }
          store_tile_mf<MF, TM, TN, BM, BN>(p, acc, b, 0, m0, n0, wm, wn, lane);
        }
      }
      it += kt1 - kt0;
    }
  }
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int MF, int NSTAGE, int BK = 64>
int launch_k64(const GemmP& p, const SkP* sk, hipStream_t st) {
  if (sk) {
    hipLaunchKernelGGL((gemm_nt_k64_kernel<BM, BN, WAVES_M, WAVES_N, MF, NSTAGE, true, BK>), dim3(sk->grid),
                       dim3(64 * WAVES_M * WAVES_N), 0, st, p, *sk);
  } else {
    dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, p.batch * p.splitk);
    hipLaunchKernelGGL((gemm_nt_k64_kernel<BM, BN, WAVES_M, WAVES_N, MF, NSTAGE, false, BK>), grid,
                       dim3(64 * WAVES_M * WAVES_N), 0, st, p, SkP{});
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
int launch_glds(const GemmP& p, hipStream_t st) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, p.batch * p.splitk);
  hipLaunchKernelGGL((gemm_nt_glds_kernel<BM, BN, WAVES_M, WAVES_N>), grid, dim3(64 * WAVES_M * WAVES_N), 0, st, p);
  DASA_CHECK_LAUNCH();
  return 0;
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
struct TileCfg { int bm, bn, wm, wn, kw; bool glds = false; bool sk = false; };
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
    // LDS-DMA NT kernels (gemm_nt_glds_kernel): {BM, BN, WM, WN} with kw unused
    {128, 128, 64, 64, 1, true},  // 15
    {256, 128, 64, 64, 1, true},  // 16: 8 waves
    {128, 64, 64, 32, 1, true},   // 17
    {64, 64, 32, 32, 1, true},    // 18
    {128, 128, 32, 64, 1, true},  // 19: 8 waves
    {64, 128, 32, 64, 1, true},   // 20
    // 64-deep K tiles (gemm_nt_k64_kernel): {BM, BN, WM, WN, MF | NSTAGE << 8}
    {128, 128, 64, 64, 16 | 1 << 8, true},   // 21
    {128, 128, 64, 64, 32 | 1 << 8, true},   // 22
    {128, 128, 64, 64, 16 | 2 << 8, true},   // 23
    {128, 64, 64, 32, 16 | 1 << 8, true},    // 24
    {64, 128, 32, 64, 16 | 1 << 8, true},    // 25
    {64, 64, 32, 32, 16 | 1 << 8, true},     // 26
    {128, 128, 32, 64, 16 | 1 << 8, true},   // 27: 8 waves
    {256, 128, 64, 64, 16 | 1 << 8, true},   // 28: 8 waves
    {64, 64, 32, 32, 16 | 2 << 8, true},     // 29
    {128, 64, 64, 32, 16 | 2 << 8, true},    // 30
    // stream-K forms of the 64-deep K kernels (grid = CUs x occupancy, see SkP)
    {128, 128, 64, 64, 16 | 1 << 8, true, true},   // 31
    {128, 64, 64, 32, 16 | 1 << 8, true, true},    // 32
    {64, 128, 32, 64, 16 | 1 << 8, true, true},    // 33
    {64, 64, 32, 32, 16 | 1 << 8, true, true},     // 34
    {128, 128, 32, 64, 16 | 1 << 8, true, true},   // 35: 8 waves
    // 32-deep K, double-buffered LDS (one barrier per K tile), 8 waves
    {128, 128, 32, 64, 16 | 2 << 8, true},   // 36: 64 KB LDS -> two workgroups per CU
    {256, 128, 64, 64, 16 | 2 << 8, true},   // 37: 96 KB LDS
    {128, 128, 64, 32, 16 | 2 << 8, true},   // 38: 4x2 waves of 32x64 -> 2x4 of 64x32
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

// Non-glds stand-in for a glds configuration whose operands do not qualify (same tile).
int glds_fallback(int cfg) {
  switch (cfg) {
    case 15: return 0;
    case 16: return 0;
    case 17: return 6;
    case 18: return 2;
    case 19: return 0;
    case 20: return 1;
    case 21: case 22: case 23: case 27: case 28: case 36: case 37: case 38: return 0;
    case 24: case 30: return 6;
    case 25: case 33: return 1;
    case 31: case 35: return 0;
    case 32: return 6;
    default: return 2;
  }
}

int launch_cfg(int cfg, bool vec, bool glds_ok, const GemmP& p, const SkP* sk, int opA, int opB, hipStream_t st) {
  if (kCfgs[cfg].glds) {
    if (!glds_ok) cfg = glds_fallback(cfg);
    else switch (cfg) {
      case 15: return launch_glds<128, 128, 2, 2>(p, st);
      case 16: return launch_glds<256, 128, 4, 2>(p, st);
      case 17: return launch_glds<128, 64, 2, 2>(p, st);
      case 18: return launch_glds<64, 64, 2, 2>(p, st);
      case 19: return launch_glds<128, 128, 4, 2>(p, st);
      case 20: return launch_glds<64, 128, 2, 2>(p, st);
      case 21: return launch_k64<128, 128, 2, 2, 16, 1>(p, nullptr, st);
      case 22: return launch_k64<128, 128, 2, 2, 32, 1>(p, nullptr, st);
      case 23: return launch_k64<128, 128, 2, 2, 16, 2>(p, nullptr, st);
      case 24: return launch_k64<128, 64, 2, 2, 16, 1>(p, nullptr, st);
      case 25: return launch_k64<64, 128, 2, 2, 16, 1>(p, nullptr, st);
      case 26: return launch_k64<64, 64, 2, 2, 16, 1>(p, nullptr, st);
      case 27: return launch_k64<128, 128, 4, 2, 16, 1>(p, nullptr, st);
      case 28: return launch_k64<256, 128, 4, 2, 16, 1>(p, nullptr, st);
      case 29: return launch_k64<64, 64, 2, 2, 16, 2>(p, nullptr, st);
      case 30: return launch_k64<128, 64, 2, 2, 16, 2>(p, nullptr, st);
      case 31: return launch_k64<128, 128, 2, 2, 16, 1>(p, sk, st);
      case 32: return launch_k64<128, 64, 2, 2, 16, 1>(p, sk, st);
      case 33: return launch_k64<64, 128, 2, 2, 16, 1>(p, sk, st);
      case 34: return launch_k64<64, 64, 2, 2, 16, 1>(p, sk, st);
      case 36: return launch_k64<128, 128, 4, 2, 16, 2, 32>(p, nullptr, st);
      case 37: return launch_k64<256, 128, 4, 2, 16, 2, 32>(p, nullptr, st);
      case 38: return launch_k64<128, 128, 2, 4, 16, 2, 32>(p, nullptr, st);
      default: return launch_k64<128, 128, 4, 2, 16, 1>(p, sk, st);
    }
  }
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


// ---- bf16-operand NT GEMM (BASELINE configs[4]: B = 256, bf16 with fp32 accumulation) --------------
// C = epilogue(A . W^T): A fp32 [M][lda] converted to bf16 on its way into LDS (v_cvt_pk_bf16_f32,
// round-to-nearest-even), W bf16 [N][ldb] (a weight copy converted once), v_mfma_f32_16x16x32_bf16,
// fp32 accumulators and the fp32 fused epilogue of the f32 kernels. K tiles of 64 bf16 = 128-B LDS
// rows of eight 16-B quads, quad q of row r at slot q ^ ((r >> 1) & 7) (two rows per 256-B bank row:
// each 16-lane ds_read_b128 group hits 16 distinct slots); two LDS stages, one barrier per K tile,
// next tile prefetched into registers across the MFMAs.

__device__ __forceinline__ int bswz(int row) { return (row >> 1) & 7; }

// ABF: A arrives as bf16 ([M][lda] bf16 elements: an activation a producer already rounded, e.g. the
// bf16 GELU output of the FFN-up GEMM) and is copied into LDS as is; CBF: C is written as bf16 (above).
// Rounding A in its producer's epilogue instead of on this kernel's load gives the same bf16 values.
template <int BM, int BN, int WAVES_M, int WAVES_N, int PF = 1, bool ABF = false, bool CBF = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_bf16_nt_kernel(GemmP p) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;   // 16-B bf16 quads per thread per tile
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "tile quads must split evenly");
  constexpr int STAGE = (BM + BN) * 8;                // uint4 per LDS stage
  __shared__ uint4 smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m > 1) {
    const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
    const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
    m0 = (grp * gm + r % rows) * BM;
    n0 = (r / rows) * BN;
  } else {
    n0 = (wgid % gridDim.x) * BN;
    m0 = (wgid / gridDim.x) * BM;
  }
  const int b = blockIdx.z;
  const float* A = ABF ? p.A : p.A + (long)b * p.sA;
  const unsigned short* Ab = reinterpret_cast<const unsigned short*>(p.A) + (long)b * p.sA;
  const unsigned short* W = reinterpret_cast<const unsigned short*>(p.B) + (long)b * p.sB;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // staging registers of the next K tile (a struct with member functions like TileLoader: hipcc keeps
  // it in VGPRs, where lambda-captured local arrays were promoted to LDS)
  struct Stage {
    floatx4 a[ABF ? 1 : NA][2];
    u32x4 ab[ABF ? NA : 1];
    u32x4 b[NB];
    __device__ __forceinline__ void load(const GemmP& p, const float* A, const unsigned short* Ab,
                                         const unsigned short* W, int m0, int n0, int k0, int tid) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + NT * i, row = q >> 3, kq = q & 7;
        if constexpr (ABF) {
          ab[i] = *reinterpret_cast<const u32x4*>(Ab + (long)min(m0 + row, p.M - 1) * p.lda + k0 + 8 * kq);
        } else {
          const float* src = A + (long)min(m0 + row, p.M - 1) * p.lda + k0 + 8 * kq;
          a[i][0] = *reinterpret_cast<const floatx4*>(src);
          a[i][1] = *reinterpret_cast<const floatx4*>(src + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int q = tid + NT * i, row = q >> 3, kq = q & 7;
        const unsigned short* src = W + (long)min(n0 + row, p.N - 1) * p.ldb + k0 + 8 * kq;
        b[i] = *reinterpret_cast<const u32x4*>(src);
      }
    }
    __device__ __forceinline__ void store(uint4* S, int tid) const {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + NT * i, row = q >> 3, kq = q & 7;
        if constexpr (ABF) {
          S[row * 8 + (kq ^ bswz(row))] = __builtin_bit_cast(uint4, ab[i]);
        } else {
          const floatx4 x = a[i][0], y = a[i][1];
          S[row * 8 + (kq ^ bswz(row))] = uint4{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]),
                                                pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])};
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int q = tid + NT * i, row = q >> 3, kq = q & 7;
        S[BM * 8 + row * 8 + (kq ^ bswz(row))] = __builtin_bit_cast(uint4, b[i]);
      }
    }
  } stg, stg2;
  // clamped rows: rows past M / N re-read the last valid row; the epilogue never stores them
  // lane l of a 16x16x32 MFMA holds A[row l & 15][k = 8 (l >> 4) + j]: K step s reads quad 4s + (l >> 4)
  auto compute = [&](const uint4* S) {
    const uint4* As = S;
    const uint4* Bs = S + BM * 8;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int q = 4 * st + (lane >> 4);
      bf16x8_t af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm + 16 * i + (lane & 15);
        af[i] = __builtin_bit_cast(bf16x8_t, As[row * 8 + (q ^ bswz(row))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + 16 * j + (lane & 15);
        bf[j] = __builtin_bit_cast(bf16x8_t, Bs[row * 8 + (q ^ bswz(row))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = p.K / 64;
  stg.load(p, A, Ab, W, m0, n0, 0, tid);
  if (PF == 1) {
    stg.store(smem, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      stg.load(p, A, Ab, W, m0, n0, 64 * min(t + 1, nk - 1), tid);   // unconditional (see gemm_nt_k64_kernel)
      compute(smem + (t & 1) * STAGE);
      stg.store(smem + ((t + 1) & 1) * STAGE, tid);
      __syncthreads();
    }
  } else {
    // two register stages (as gemm_f32x6_nt_kernel): tile t + 2's loads are issued before tile t's MFMAs
    stg2.load(p, A, Ab, W, m0, n0, 64 * min(1, nk - 1), tid);
        stg.store(smem, tid);
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {
      stg.load(p, A, Ab, W, m0, n0, 64 * min(t + 2, nk - 1), tid);
      compute(smem);
            stg2.store(smem + STAGE, tid);
      __syncthreads();
      if (t + 1 >= nk) break;
      stg2.load(p, A, Ab, W, m0, n0, 64 * min(t + 3, nk - 1), tid);
      compute(smem + STAGE);
            stg.store(smem, tid);
      __syncthreads();
    }
  }
  if constexpr (CBF) {
    // bf16 C through LDS: the 16x16 accumulator layout gives each lane one column of 4 rows, i.e. 2-byte
    // stores in 32-B row pieces (measured 1.85x slower than the fp32 epilogue on 20480 x 3072 x 768).
    // Each wave rounds its WM x WN sub-tile (epilogue applied) into its own LDS region, then stores it as
    // 16-B row chunks: 128-B contiguous row pieces. The stage buffers are free once every wave is past
    // its last MFMA (the barrier).
    static_assert(WAVES_M * WAVES_N * WM * WN * 2 <= (int)sizeof(smem), "bf16 tile must fit the LDS stages");
    __syncthreads();
    unsigned short* T = reinterpret_cast<unsigned short*>(smem) + wave * (WM * WN);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = 16 * j + (lane & 15), col = min(n0 + wn + cl, p.N - 1);
      const float bj = p.bias ? p.bias[col] : 0.f, cs = p.colscale ? p.colscale[col] : 1.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = 16 * i + 4 * (lane >> 4) + r;
          float v = apply_act(p.alpha * acc[i][j][r] + bj, p.act);
          if (p.aux) v *= p.aux[(long)b * p.sAux + (long)min(m0 + wm + rl, p.M - 1) * p.ld_aux + col];
          T[rl * WN + cl] = __builtin_bit_cast(unsigned short, (__bf16)(v * cs));
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed (wave-private region)
    __builtin_amdgcn_wave_barrier();
    constexpr int CPR = WN / 8;           // 16-B chunks per row
    unsigned short* C = reinterpret_cast<unsigned short*>(p.C) + (long)b * p.sC;
#pragma unroll
    for (int it = 0; it < WM * CPR / 64; ++it) {
      const int q = lane + 64 * it, rl = q / CPR, c8 = (q % CPR) * 8;
      const int row = m0 + wm + rl, col = n0 + wn + c8;
      const uint4 u = *reinterpret_cast<const uint4*>(T + rl * WN + c8);
      if (row < p.M && col < p.N) *reinterpret_cast<uint4*>(C + (long)row * p.ldc + col) = u;
    }
  } else {
    store_tile_mf<16, TM, TN, BM, BN>(p, acc, b, 0, m0, n0, wm, wn, lane);
  }
}

// ---- fp32 GEMM emulated on bf16 matrix cores ("bf16x6") ------------------------------------------
// Every fp32 operand x is split exactly into three bf16 planes, x = hi + mid + lo (hi = bf16(x),
// mid = bf16(x - hi), lo = bf16(x - hi - mid): 3 x 8 significand bits cover fp32's 24). A product
// x * y then expands to nine bf16 products, each EXACT in fp32 (8 + 8 bits); the six kept here
// (hh, hm, mh, hl, lh, mm) leave out terms below 2^-25 |x y|, i.e. under fp32's own rounding of the
// product, and v_mfma_f32_16x16x32_bf16 accumulates them in fp32 — so the result carries fp32
// accuracy (tests/test_kernels_gpu.py compares its error against the native fp32 MFMA kernel's, both
// against fp64) at six bf16 MFMAs per tile step = 6/16 of the fp32 MFMA cost.
// hh goes to its own accumulator, the five small terms to a second one, summed in the epilogue.
// W (the nn.Linear weight) arrives pre-split (dasa_f32_split3_bf16, once per weight version); A is
// split on its way into LDS. LDS holds per stage, per plane, the tile quad-major: 16-B unit (q, row)
// at [q][row] (q = 8-bf16 K group of the 32-deep K tile) — the 16x16x32 fragment read (lane l: row
// l & 15, quad l >> 4) and the 8-lane ds_write_b128 groups (8 consecutive rows of one quad) are both
// bank-conflict-free without a swizzle.

// Split-K form (SPL): blockIdx.z = batch * splitk + split; each split runs K range [split * kchunk,
// +kchunk) and stores its tile partial write-through (sc1) into its own slab; the LAST split to arrive
// (agent-scope ticket on the tile's counter, re-armed to 0) sums the slabs in split order
// (deterministic) and runs the epilogue — the few-tile LXRT / vision GEMMs fill the chip without a
// second reduce launch, and no workgroup ever waits on another.
struct X6Split { unsigned* cnt; float* slab; int splitk, kchunk; };

// (at most 2 waves per SIMD fit the LDS of the 128-row forms anyway: telling the register allocator so
// lets it use 256 VGPRs instead of spilling to reach an occupancy the LDS forbids)
// PRIO (A/B forms 10-13): 1 = s_setprio(1) around every MFMA cluster (cdna_hip_programming.md T5),
// 2 = one static s_setprio(1) for the second half of the workgroup's waves (T5 static form).
// PF = -1 (form 20): ONE LDS stage (48 KB at 128 x 128) and one register stage, two barriers per K step,
// at most 128 registers (waves_per_eu 4): two workgroups share a CU and overlap each other's split / LDS
// phase with their MFMAs — form 8's products in form 8's order (bitwise equal), 1.07-1.14x the previous
// plan on the many-tile K = 768, N >= 2048 shapes (profiles/r03/x6_lds1_forms.txt).
template <int BM, int BN, int WAVES_M, int WAVES_N, bool SEP, int PF = 1, bool SPL = false, int PRIO = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
__attribute__((amdgpu_waves_per_eu(PF < 0 ? 4 : 1, PF < 0 ? 4 : 2)))
void gemm_f32x6_nt_kernel(GemmP p, long plane, X6Split xs) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int NA = BM * 4 / NT, NB = BN * 4 / NT;    // 16-B (8 x bf16) K quads per thread per plane
  static_assert((BM * 4) % NT == 0 && (BN * 4) % NT == 0, "tile quads must split evenly");
  constexpr int PA = BM * 4, PB = BN * 4;               // uint4 per plane image
  constexpr int STAGE = 3 * (PA + PB);
  __shared__ uint4 smem[(PF < 0 ? 1 : 2) * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (PRIO == 2 && __builtin_amdgcn_readfirstlane(tid) >= NT / 2) __builtin_amdgcn_s_setprio(1);
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m > 1) {
    const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
    const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
    m0 = (grp * gm + r % rows) * BM;
    n0 = (r / rows) * BN;
  } else if (p.group_m < -1) {   // grouped along N: -group_m column panels of W stay in L2, A streams
    const int gn = -p.group_m, per = gn * gridDim.y, grp = wgid / per;
    const int cols = min(gn, (int)gridDim.x - grp * gn), r = wgid - grp * per;
    n0 = (grp * gn + r % cols) * BN;
    m0 = (r / cols) * BM;
  } else {
    n0 = (wgid % gridDim.x) * BN;
    m0 = (wgid / gridDim.x) * BM;
  }
  const int b = SPL ? blockIdx.z / xs.splitk : blockIdx.z, split = SPL ? blockIdx.z % xs.splitk : 0;
  const int kb = SPL ? split * xs.kchunk : 0;
  const float* A = p.A + (long)b * p.sA + kb;
  const unsigned short* W = reinterpret_cast<const unsigned short*>(p.B) + (long)b * p.sB + kb;

  floatx4 big[TM][TN], small[SEP ? TM : 1][SEP ? TN : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (SEP) {
#pragma unroll
    for (int i = 0; i < (SEP ? TM : 1); ++i)
#pragma unroll
      for (int j = 0; j < (SEP ? TN : 1); ++j) small[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  // unit u -> (row, quad): 8 consecutive lanes take 8 consecutive rows of one quad (coalesced 128-B
  // row segments per 4 x 8 lanes on the global side, conflict-free ds_write_b128 groups on the LDS side)
  struct Stage {
    u32x4 a[NA][2];   // 8 fp32 of A as bit patterns (integer vectors keep the stages out of scratch)
    u32x4 w[3][NB];
    __device__ __forceinline__ static void unit(int u, int& row, int& q) {
      q = (u >> 3) & 3;
      row = (u & 7) + 8 * (u >> 5);
    }
    __device__ __forceinline__ void load(const GemmP& p, const float* A, const unsigned short* W, long plane, int m0,
                                         int n0, int k0, int tid) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        int row, q;
        unit(tid + NT * i, row, q);
        const float* src = A + (long)min(m0 + row, p.M - 1) * p.lda + k0 + 8 * q;
        a[i][0] = *reinterpret_cast<const u32x4*>(src);
        a[i][1] = *reinterpret_cast<const u32x4*>(src + 4);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int row, q;
        unit(tid + NT * i, row, q);
        const unsigned short* src = W + (long)min(n0 + row, p.N - 1) * p.ldb + k0 + 8 * q;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) w[pl][i] = *reinterpret_cast<const u32x4*>(src + pl * plane);
      }
    }
    __device__ __forceinline__ void store(uint4* S, int tid) const {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        int row, q;
        unit(tid + NT * i, row, q);
        uint4 h, m, l;
        split3_quad(__builtin_bit_cast(float4, a[i][0]), __builtin_bit_cast(float4, a[i][1]), h, m, l);
        S[0 * PA + q * BM + row] = h;
        S[1 * PA + q * BM + row] = m;
        S[2 * PA + q * BM + row] = l;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int row, q;
        unit(tid + NT * i, row, q);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) S[3 * PA + pl * PB + q * BN + row] = __builtin_bit_cast(uint4, w[pl][i]);
      }
    }
  } stg, stg2, stg3;

  auto compute = [&](const uint4* S) {
    const int q = lane >> 4;
    if (PRIO == 1) __builtin_amdgcn_s_setprio(1);
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
        floatx4& sm = SEP ? small[SEP ? i : 0][SEP ? j : 0] : big[i][j];
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[1][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[2][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], bf[0][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[1][j], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[0][j], sm, 0, 0, 0);
        big[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[0][j], big[i][j], 0, 0, 0);
      }
    }
    if (PRIO == 1) __builtin_amdgcn_s_setprio(0);
  };

  const int nk = (SPL ? min(xs.kchunk, p.K - kb) : p.K) / 32;
  stg.load(p, A, W, plane, m0, n0, 0, tid);
  if (PF < 0) {
    stg.store(smem, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      stg.load(p, A, W, plane, m0, n0, 32 * min(t + 1, nk - 1), tid);   // unconditional (clamped re-read)
      compute(smem);
      __syncthreads();
      stg.store(smem, tid);
      __syncthreads();
    }
  } else if (PF == 1) {
    stg.store(smem, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      stg.load(p, A, W, plane, m0, n0, 32 * min(t + 1, nk - 1), tid);   // unconditional (clamped re-read)
      compute(smem + (t & 1) * STAGE);
      stg.store(smem + ((t + 1) & 1) * STAGE, tid);
      __syncthreads();
    }
  } else if (PF == 3) {
    // three register stages: tile t + 3's loads issued before tile t's MFMAs
    stg2.load(p, A, W, plane, m0, n0, 32 * min(1, nk - 1), tid);
    stg3.load(p, A, W, plane, m0, n0, 32 * min(2, nk - 1), tid);
    stg.store(smem, tid);
    __syncthreads();
    for (int t = 0; t < nk; t += 3) {
      stg.load(p, A, W, plane, m0, n0, 32 * min(t + 3, nk - 1), tid);
      compute(smem + (t & 1) * STAGE);
      stg2.store(smem + ((t + 1) & 1) * STAGE, tid);
      __syncthreads();
      if (t + 1 >= nk) break;
      stg2.load(p, A, W, plane, m0, n0, 32 * min(t + 4, nk - 1), tid);
      compute(smem + ((t + 1) & 1) * STAGE);
      stg3.store(smem + (t & 1) * STAGE, tid);
      __syncthreads();
      if (t + 2 >= nk) break;
      stg3.load(p, A, W, plane, m0, n0, 32 * min(t + 5, nk - 1), tid);
      compute(smem + (t & 1) * STAGE);
      stg.store(smem + ((t + 1) & 1) * STAGE, tid);
      __syncthreads();
    }
  } else {
    // two register stages: the loads of tile t + 2 are issued before tile t's MFMAs, so each tile's
    // global reads have two K steps of compute to land in (the L2 / MALL latency under full load)
    stg2.load(p, A, W, plane, m0, n0, 32 * min(1, nk - 1), tid);
        stg.store(smem, tid);
    __syncthreads();
    // PRIO == 3 (A/B form 26): the next stage's split + ds_write interleaved between the MFMA groups
    // (sched_group_barrier: loads, fragment reads, then 6 x {8 MFMA, 8 VALU, 1 ds_write})
    auto interleave = [&]() {
      if constexpr (PRIO == 3) {
        __builtin_amdgcn_sched_group_barrier(0x020, 5, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 18, 0);
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
      }
    };
    for (int t = 0; t < nk; t += 2) {
      stg.load(p, A, W, plane, m0, n0, 32 * min(t + 2, nk - 1), tid);
      compute(smem);
            stg2.store(smem + STAGE, tid);
      interleave();
      __syncthreads();
      if (t + 1 >= nk) break;
      stg2.load(p, A, W, plane, m0, n0, 32 * min(t + 3, nk - 1), tid);
      compute(smem + STAGE);
            stg.store(smem, tid);
      interleave();
      __syncthreads();
    }
  }
  if (SEP) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) big[i][j] += small[SEP ? i : 0][SEP ? j : 0];
  }
  if constexpr (SPL) {
    __shared__ int s_last;
    const int tile = (b * (int)gridDim.y + m0 / BM) * (int)gridDim.x + n0 / BN;
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
  store_tile_mf<16, TM, TN, BM, BN>(p, big, b, 0, m0, n0, wm, wn, lane);
}

// Register-A form (forms 21, 22): LDS holds only the pre-split W planes. Each wave reads its own A
// fragments from global memory straight into registers in the 16x16x32 operand layout (lane l: row
// l & 15 of the fragment, the 8 fp32 of K group l >> 4 — 16 rows x 128 contiguous bytes per fragment) and
// splits them into hi / mid / lo in registers. Form 8 per 32-deep K step moves, per CU, 48 KB into LDS
// (A's three planes + W's) and 18 ds_read_b128 per wave out of it: ~1200 LDS cycles against 768 MFMA
// cycles per SIMD — LDS-bound. Here the A planes never touch LDS: 24 KB in and 12 reads per wave out.
// The cost moves to VALU (each of the WAVES_N waves sharing an A row splits it) and to L1/L2 (each
// A row fetched by WAVES_N waves). Same products in the same order with the same two accumulators as
// form 8: bitwise equal to it. Ring: W(t+1) sits in registers while tile t computes and goes to the
// other LDS stage after it; A(t+2) is loaded into the register stage tile t has just consumed.
// MEASURED AND REJECTED (sweeps only, profiles/r05/x6_register_a_forms.log): 0.75-0.85x form 8 / 20 for
// 128 x 128 with 8 waves (form 22), 0.55-0.6x with 4 waves of 64 x 64 (form 21) on the many-tile shapes —
// the LDS budget above is not what bounds form 8; the per-wave fragment loads (one K step of lookahead,
// half-sector 16-B accesses) and the duplicated split cost more than the LDS traffic they remove.
template <int BM, int BN, int WAVES_M, int WAVES_N, int OCC = 2>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) __attribute__((amdgpu_waves_per_eu(1, OCC)))
void gemm_f32x6_ra_kernel(GemmP p, long plane) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int NB = BN * 4 / NT;
  static_assert((BN * 4) % NT == 0 && WM % 16 == 0 && WN % 16 == 0, "tile must split evenly");
  constexpr int PB = BN * 4;                 // uint4 per W plane image
  constexpr int STAGE = 3 * PB;
  __shared__ uint4 smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m > 1) {
    const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
    const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
    m0 = (grp * gm + r % rows) * BM;
    n0 = (r / rows) * BN;
  } else if (p.group_m < -1) {
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

  struct ARegs {
    u32x4 a[TM][2];
    __device__ __forceinline__ void load(const GemmP& p, const float* A, int m0, int wm, int lane, int k0) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = A + (long)min(m0 + wm + 16 * i + (lane & 15), p.M - 1) * p.lda + k0 + 8 * (lane >> 4);
        a[i][0] = *reinterpret_cast<const u32x4*>(src);
        a[i][1] = *reinterpret_cast<const u32x4*>(src + 4);
      }
    }
  } ra0, ra1;
  struct WRegs {
    u32x4 w[3][NB];
    __device__ __forceinline__ void load(const GemmP& p, const unsigned short* W, long plane, int n0, int k0, int tid) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int u = tid + NT * i, q = (u >> 3) & 3, row = (u & 7) + 8 * (u >> 5);
        const unsigned short* src = W + (long)min(n0 + row, p.N - 1) * p.ldb + k0 + 8 * q;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) w[pl][i] = *reinterpret_cast<const u32x4*>(src + pl * plane);
      }
    }
    __device__ __forceinline__ void store(uint4* S, int tid) const {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int u = tid + NT * i, q = (u >> 3) & 3, row = (u & 7) + 8 * (u >> 5);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) S[pl * PB + q * BN + row] = __builtin_bit_cast(uint4, w[pl][i]);
      }
    }
  } rw;

  auto compute = [&](const uint4* S, const ARegs& ar) {
    const int q = lane >> 4;
    bf16x8_t bf[3][TN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[pl][j] = __builtin_bit_cast(bf16x8_t, S[pl * PB + q * BN + wn + 16 * j + (lane & 15)]);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      uint4 h, m, l;
      split3_quad(__builtin_bit_cast(float4, ar.a[i][0]), __builtin_bit_cast(float4, ar.a[i][1]), h, m, l);
      const bf16x8_t af[3] = {__builtin_bit_cast(bf16x8_t, h), __builtin_bit_cast(bf16x8_t, m),
                              __builtin_bit_cast(bf16x8_t, l)};
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

  const int nk = p.K / 32;
  rw.load(p, W, plane, n0, 0, tid);
  ra0.load(p, A, m0, wm, lane, 0);
  rw.store(smem, tid);
  __syncthreads();
  const int k1 = 32 * min(1, nk - 1);
  rw.load(p, W, plane, n0, k1, tid);
  ra1.load(p, A, m0, wm, lane, k1);
  for (int t = 0; t < nk; t += 2) {
    compute(smem, ra0);
    rw.store(smem + STAGE, tid);                       // W(t + 1) -> the stage tile t - 1 used
    int kn = 32 * min(t + 2, nk - 1);                  // clamped re-reads past the end
    rw.load(p, W, plane, n0, kn, tid);
    ra0.load(p, A, m0, wm, lane, kn);
    __syncthreads();
    if (t + 1 >= nk) break;
    compute(smem + STAGE, ra1);
    rw.store(smem, tid);
    kn = 32 * min(t + 3, nk - 1);
    rw.load(p, W, plane, n0, kn, tid);
    ra1.load(p, A, m0, wm, lane, kn);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] += small[i][j];
  store_tile_mf<16, TM, TN, BM, BN>(p, big, b, 0, m0, n0, wm, wn, lane);
}

// All-DMA form (form 16, sweeps only: 0.80-0.90x form 8 on the 12800-row shapes, profiles/r03/
// x6_dma_form.txt): the same tile, products, product order and epilogue as form 8 (bitwise equal),
// but nothing is staged through VGPRs or written by ds_write: A (fp32) and the pre-split W planes go
// HBM/L2 -> LDS by global_load_lds_dwordx4 into a ring of three K stages, two steps ahead, and A is split
// into its bf16 planes at fragment-read time (each A fragment is split by the WAVES_N waves that read it:
// 2x form 8's split VALU, issued between MFMAs instead of in a split + ds_write phase that every wave of
// a SIMD reaches at once after the barrier). Per K step a wave waits for its own stage-t DMAs (counted
// vmcnt: stage t+1's stay in flight), one s_barrier (every wave's stage-t DMAs landed; every wave is
// done reading stage t-1, whose slot stage t+2 now refills), issues stage t+2, and computes stage t.
// LDS images (16-B units, DMA lane-linear: one wave-instruction = 64 consecutive units):
//   A  [q2][row], q2 = the 4-float K group (0..7) -> the 16x16x32 fragment of lane l (row l & 15, K
//      quad q = l >> 4) is units (2q, row), (2q + 1, row): 16 lanes read 16 consecutive units
//   W  [plane][q][row] as form 8
// The DMAs and the waits on them are inline asm, outside hipcc's waitcnt model: its LDS-DMA tracking
// merged the ring's stages at the loop header and drained vmcnt(0) before reading the stage that had
// landed (profiles/r03/x6_dma_form.txt). The asm barrier / waits carry "memory" clobbers, so no LDS
// read of a stage moves across the barrier that frees or publishes it; M0 (the DMA's LDS base) is set
// in the same asm statement and is used by nothing else in this kernel.
__device__ __forceinline__ void lds_dma16(const void* g, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_base)
               : "memory", "m0");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)((const __attribute__((address_space(3))) void*)p);
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) __attribute__((amdgpu_waves_per_eu(1, 2)))
void gemm_f32x6_dma_kernel(GemmP p, long plane) {
  constexpr int NWV = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int UA = BM * 8, PB = BN * 4;                    // 16-B units: A stage, one W plane
  constexpr int IA = UA / 64 / NWV, IW = 3 * PB / 64 / NWV;  // DMA wave-instructions per wave per stage
  static_assert(IA * 64 * NWV == UA && IW * 64 * NWV == 3 * PB, "stage units must split evenly");
  static_assert(IA + IW == 5, "the vmcnt immediates below are written for 5 DMAs per wave per stage");
  __shared__ uint4 sA[3][UA];
  __shared__ uint4 sW[3][3 * PB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m > 1) {
    const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
    const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
    m0 = (grp * gm + r % rows) * BM;
    n0 = (r / rows) * BN;
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
    for (int j = 0; j < TN; ++j) {
      big[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      small[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

  // per-lane DMA sources (rows past M / N re-read the last row; their outputs are dropped) and the
  // wave-uniform LDS bases of its DMA slots in stage 0 (stage s adds s * the stage size)
  const float* asrc[IA];
  unsigned adst[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int u = (wave * IA + j) * 64 + lane, q2 = u / BM, row = u % BM;
    asrc[j] = A + (long)min(m0 + row, p.M - 1) * p.lda + 4 * q2;
    adst[j] = __builtin_amdgcn_readfirstlane(lds_addr(&sA[0][(wave * IA + j) * 64]));
  }
  const unsigned short* wsrc[IW];
  unsigned wdst[IW];
#pragma unroll
  for (int j = 0; j < IW; ++j) {
    const int u = (wave * IW + j) * 64 + lane, pl = u / PB, rem = u % PB, q = rem / BN, row = rem % BN;
    wsrc[j] = W + pl * plane + (long)min(n0 + row, p.N - 1) * p.ldb + 8 * q;
    wdst[j] = __builtin_amdgcn_readfirstlane(lds_addr(&sW[0][(wave * IW + j) * 64]));
  }
  const int nk = p.K / 32;
  auto dma = [&](int stage, int t) {   // stage t's slice of this wave, unconditional (clamped re-read)
    const int k0 = 32 * min(t, nk - 1);
#pragma unroll
    for (int j = 0; j < IA; ++j) lds_dma16(asrc[j] + k0, adst[j] + stage * UA * 16);
#pragma unroll
    for (int j = 0; j < IW; ++j) lds_dma16(wsrc[j] + k0, wdst[j] + stage * 3 * PB * 16);
  };
  const int q = lane >> 4;
  auto compute = [&](int stage) {
    const uint4* SA = sA[stage];
    const uint4* SW = sW[stage];
    bf16x8_t af[TM][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm + 16 * i + (lane & 15);
      uint4 h, m, l;
      split3_quad(__builtin_bit_cast(float4, SA[(2 * q) * BM + row]), __builtin_bit_cast(float4, SA[(2 * q + 1) * BM + row]),
                  h, m, l);
      af[i][0] = __builtin_bit_cast(bf16x8_t, h);
      af[i][1] = __builtin_bit_cast(bf16x8_t, m);
      af[i][2] = __builtin_bit_cast(bf16x8_t, l);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8_t bf[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bf[pl] = __builtin_bit_cast(bf16x8_t, SW[pl * PB + q * BN + wn + 16 * j + (lane & 15)]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        floatx4& sm = small[i][j];
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[1], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[2], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bf[0], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[1], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[0], sm, 0, 0, 0);
        big[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[0], big[i][j], 0, 0, 0);
      }
    }
  };
  dma(0, 0);
  dma(1, 1);
  int stage = 0;
  for (int t = 0; t < nk; ++t) {
    // own stage-t DMAs landed (the 5 of stage t+1 may still fly), then everyone's; stage t-1 is free
    asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
    dma(stage == 0 ? 2 : stage - 1, t + 2);
    compute(stage);
    stage = stage == 2 ? 0 : stage + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA into LDS outlives the workgroup
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] += small[i][j];
  store_tile_mf<16, TM, TN, BM, BN>(p, big, b, 0, m0, n0, wm, wn, lane);
}

// x [rows][ldx] fp32 -> y planes [3][rows][cols] bf16 (plane stride rows * cols), x = hi + mid + lo.
__global__ void split3_bf16_kernel(const float* __restrict__ x, long ldx, uint4* __restrict__ y, int rows, int cols) {
  const int cq = cols / 8;
  const long n = (long)rows * cq, plane = n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cq;
    const int c = (int)(i - r * cq) * 8;
    const float* src = x + r * ldx + c;
    uint4 h, m, l;
    split3_quad(*reinterpret_cast<const float4*>(src), *reinterpret_cast<const float4*>(src + 4), h, m, l);
    y[i] = h;
    y[i + plane] = m;
    y[i + 2 * plane] = l;
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, unsigned* __restrict__ y, long npairs) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < npairs; i += (long)gridDim.x * blockDim.x) {
    const float2 v = reinterpret_cast<const float2*>(x)[i];
    y[i] = pack_bf16x2(v.x, v.y);
  }
}

// ------------------------------------------------------------------------------- skinny GEMMs
// The per-step decoder / critic / attention projections at B <= 32 rows (model.py:263-264, 437,
// 970-982; M = 20 at the headline batch) and their input gradients dX = dY.W are weight streaming:
// every weight element is used M <= 32 times, so the kernel's job is to read W once at HBM rate.
// The f32 MFMA 16x16x4 runs with the WEIGHT on the 16-row side and the activations (M padded to 16 or
// 32) on the 16-column side, so both operands come straight from global memory in float4 per lane
// (K-permuted: in each 32-deep step, lane group g = lane >> 4 supplies k = 8g + e to MFMA e): no LDS
// staging of W, no cross-lane reduction, one HBM pass. A workgroup of 4 waves splits its K range
// between the waves (summed through LDS in fixed order); K ranges beyond one workgroup are split over
// blockIdx.y with the partials handed to the last-arriving workgroup (write-through stores, agent
// ticket, fixed-order sum: deterministic), which runs the fused epilogue.
struct SkinnyP {
  unsigned* cnt;   // per-column-block arrival counters (workspace head; zero on entry, re-armed)
  float* slab;     // split partials: [cols][splits][NACC][64 lanes] float4
  int splits;
};

// Fused epilogue of a lane's E output elements (m[e], n[e]): every optional operand is gathered for
// all E elements inside one uniform branch before it is used (a per-element branch around a load
// makes the compiler wait for each load in turn).
template <int E>
__device__ __forceinline__ void skinny_store(const GemmP& p, const int (&m)[E], const int (&n)[E], float (&v)[E]) {
  int mc[E], nc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    mc[e] = min(m[e], p.M - 1);
    nc[e] = min(n[e], p.N - 1);
    v[e] *= p.alpha;
  }
  if (p.bias) {
    float b[E];
#pragma unroll
    for (int e = 0; e < E; ++e) b[e] = p.bias[nc[e]];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] += b[e];
  }
  if (p.act != DASA_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = apply_act(v[e], p.act);
  }
  if (p.aux) {
    float a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) a[e] = p.aux[(long)mc[e] * p.ld_aux + nc[e]];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] *= a[e];
  }
  if (p.colscale) {
    float c[E];
#pragma unroll
    for (int e = 0; e < E; ++e) c[e] = p.colscale[nc[e]];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] *= c[e];
  }
  if (p.beta != 0.f) {
    float c[E];
#pragma unroll
    for (int e = 0; e < E; ++e) c[e] = p.C[(long)mc[e] * p.ldc + nc[e]];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] += p.beta * c[e];
  }
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (m[e] < p.M && n[e] < p.N) p.C[(long)m[e] * p.ldc + n[e]] = v[e];
}

// Sum the 4 waves' accumulators (fixed order), then either run the epilogue (one split) or hand the
// workgroup partial to the last arriver of its column block. Returns true in the wave that holds the
// final sum (wave 0 of the single / last-arriving workgroup); acc then holds it.
template <int NACC>
__device__ __forceinline__ bool skinny_reduce(floatx4 (&acc)[NACC], const SkinnyP& sp, int col, int split) {
  __shared__ floatx4 red[3][NACC][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w > 0) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) red[w - 1][a][lane] = acc[a];
  }
  __syncthreads();
  if (w > 0) return false;
#pragma unroll
  for (int v = 0; v < 3; ++v)
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] += red[v][a][lane];
  if (sp.splits == 1) return true;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sp.slab, 0, 0x7fffffff, 0x00020000);
  const long base = (long)col * sp.splits;
#pragma unroll
  for (int a = 0; a < NACC; ++a) {
    const int off = (int)((((base + split) * NACC + a) * 64 + lane) * 16);
    const u32x4 u = {__float_as_uint(acc[a][0]), __float_as_uint(acc[a][1]), __float_as_uint(acc[a][2]),
                     __float_as_uint(acc[a][3])};
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);   // sc1: write-through
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(sp.cnt + col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __shfl(t, 0, 64);
  if (t != (unsigned)(sp.splits - 1)) return false;
  if (lane == 0) __hip_atomic_store(sp.cnt + col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: sc1 loads below the ticket
#pragma unroll
  for (int a = 0; a < NACC; ++a) acc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int s2 = 0; s2 < sp.splits; ++s2) {   // fixed order: deterministic whoever arrives last
#pragma unroll
    for (int a = 0; a < NACC; ++a) {
      const int off = (int)((((base + s2) * NACC + a) * 64 + lane) * 16);
      const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);   // sc1
      acc[a][0] += __uint_as_float(u.x);
      acc[a][1] += __uint_as_float(u.y);
      acc[a][2] += __uint_as_float(u.z);
      acc[a][3] += __uint_as_float(u.w);
    }
  }
  return true;
}

__device__ __forceinline__ float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// NT: Y[M,N] = epi(X[M,K] . W[N,K]^T). Workgroup = 16 output features (rows of W) x 4 waves x KS
// 32-deep steps per wave; MFMA rows = features, columns = the M <= 16*MT activation rows.
// Lane (r = lane & 15, g = lane >> 4) loads W[n0 + r][k .. k+7] and X[16t + r][k .. k+7], k = step*32 + 8g.
// XR = 4 (hybrid, 16 < M <= 20, the headline batch): one MFMA column tile for rows 0..15 and the last
// M - 16 rows on the VALU from the W values already in registers (8 fma per row per step, X rows staged
// in LDS once per workgroup, summed over the 4 lane groups at the end) instead of a second 16-column
// MFMA tile that would be 3/4 padding.
template <int MT, int KS, int XR = 0>
__global__ __launch_bounds__(256, 2) void gemm_skinny_nt_kernel(GemmP p, SkinnyP sp) {
  static_assert(XR == 0 || (XR == 4 && MT == 1), "hybrid form: one MFMA tile + 4 VALU rows");
  constexpr int KSPAN = 4 * KS * 32;                  // the workgroup's K range
  constexpr int NXQ = XR * KSPAN / 4;                 // float4 of the staged extra rows
  constexpr int NXI = XR ? (NXQ + 255) / 256 : 1;
  __shared__ float4 xs[XR ? NXQ : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int col = blockIdx.x, split = blockIdx.y, n0 = col * 16;
  const int K = p.K, kq = K - 4;   // last whole quad (K % 4 == 0)
  const float* wrow = p.B + (long)min(n0 + r, p.N - 1) * p.ldb;
  const float* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xrow[t] = p.A + (long)min(16 * t + r, p.M - 1) * p.lda;
  const int kbase = (split * 4 + w) * KS * 32 + 8 * g;
  float4 xe[NXI];
  if constexpr (XR > 0) {   // issued first, so storing them below waits for these loads only
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int idx = min((int)threadIdx.x + 256 * i, NXQ - 1), q = idx / (KSPAN / 4);
      const int k = split * KSPAN + 4 * (idx % (KSPAN / 4));
      xe[i] = ldg4(p.A + (long)min(16 + q, p.M - 1) * p.lda + min(k, kq));
    }
  }
  // every load first (clamped, unconditional: out-of-range quads re-read the last one and are zeroed
  // below), so each wave has KS x 2 KB of W in flight
  float4 wv[KS][2], xv[KS][MT][2];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = kbase + 32 * s;
    wv[s][0] = ldg4(wrow + min(k, kq));
    wv[s][1] = ldg4(wrow + min(k + 4, kq));
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      xv[s][t][0] = ldg4(xrow[t] + min(k, kq));
      xv[s][t][1] = ldg4(xrow[t] + min(k + 4, kq));
    }
  }
  // keep every load above the MFMAs (the scheduler would otherwise sink each load to its use and
  // leave one step in flight); the waitcnt pass then waits step by step
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (XR > 0) {
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int idx = (int)threadIdx.x + 256 * i;
      if (idx < NXQ) {
        const int q = idx / (KSPAN / 4), k = split * KSPAN + 4 * (idx % (KSPAN / 4));
        const float z = (16 + q < p.M && k < K) ? 1.f : 0.f;
        xs[idx] = make_float4(z * xe[i].x, z * xe[i].y, z * xe[i].z, z * xe[i].w);
      }
    }
    __syncthreads();
  }
  constexpr int NA = MT + (XR ? 1 : 0);
  floatx4 acc[NA];
#pragma unroll
  for (int t = 0; t < NA; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = kbase + 32 * s;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool ok = k + 4 * h < K;
      const float4 a = sel4(ok, wv[s][h]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, e), f4get(sel4(ok, xv[s][t][h]), e), acc[t], 0, 0, 0);
      }
      if constexpr (XR > 0) {   // rows 16..19: k .. k+3 of this quad against the staged X rows
        const int kl = (w * KS * 32 + 32 * s + 8 * g) / 4 + h;
#pragma unroll
        for (int q = 0; q < XR; ++q) {
          const float4 x = xs[q * (KSPAN / 4) + kl];
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
  if constexpr (XR > 0) {   // sum the 4 lane groups (k slices) of each feature row
#pragma unroll
    for (int q = 0; q < XR; ++q) {
      float v = acc[MT][q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[MT][q] = v;
    }
  }
  if (!skinny_reduce<NA>(acc, sp, col, split)) return;
  // C[feature = 4g + j][act row = r]  ->  Y[16t + r][n0 + 4g + j]; hybrid rows: lane group 0 of
  // feature row r holds Y[16 + q][n0 + r]
  int mm[4 * NA], nn[4 * NA];
  float v[4 * NA];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mm[4 * t + j] = 16 * t + r;
      nn[4 * t + j] = n0 + 4 * g + j;
      v[4 * t + j] = acc[t][j];
    }
  if constexpr (XR > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      mm[4 * MT + q] = g == 0 ? 16 + q : p.M;   // p.M: not stored
      nn[4 * MT + q] = n0 + r;
      v[4 * MT + q] = acc[MT][q];
    }
  }
  skinny_store<4 * NA>(p, mm, nn, v);
}

// NN: Y[M,N] = epi(X[M,K] . B[K,N]) with B row-major (ldb) - the input gradient dX = dY . W of an
// nn.Linear (W [out, in] read along its rows). Workgroup = 64 output columns x 4 waves x KS steps.
// Lane (r, g) loads B[k + e][n0 + 4r .. +3] for e = 0..7 (k = step*32 + 8g: four 256-B row pieces per
// instruction) and X[16t + r][k .. k+7]; MFMA (e, c) takes component c of the B quad as the 16-row
// operand, so accumulator c holds output columns n0 + 4*row + c.
template <int MT, int KS>
__global__ __launch_bounds__(256, 2) void gemm_skinny_nn_kernel(GemmP p, SkinnyP sp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int col = blockIdx.x, split = blockIdx.y, n0 = col * 64;
  const int K = p.K, kq = K - 4;
  const float* bcol = p.B + min(n0 + 4 * r, p.N - 4);
  const float* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xrow[t] = p.A + (long)min(16 * t + r, p.M - 1) * p.lda;
  const int kbase = (split * 4 + w) * KS * 32 + 8 * g;
  float4 bv[KS][8], xv[KS][MT][2];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = kbase + 32 * s;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[s][e] = ldg4(bcol + (long)min(k + e, K - 1) * p.ldb);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      xv[s][t][0] = ldg4(xrow[t] + min(k, kq));
      xv[s][t][1] = ldg4(xrow[t] + min(k + 4, kq));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  floatx4 acc[4 * MT];
#pragma unroll
  for (int a = 0; a < 4 * MT; ++a) acc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = kbase + 32 * s;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = k + e < K;
      const float4 b = sel4(ok, bv[s][e]);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const float xs = ok ? f4get(xv[s][t][e >> 2], e & 3) : 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[4 * t + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(b, c), xs, acc[4 * t + c], 0, 0, 0);
      }
    }
  }
  if (!skinny_reduce<4 * MT>(acc, sp, col, split)) return;
  // accumulator (t, c): C[row = 4g + j][act row = r]  ->  Y[16t + r][n0 + 16g + 4j + c]
  int mm[16 * MT], nn[16 * MT];
  float v[16 * MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int e = 16 * t + 4 * j + c;
        mm[e] = 16 * t + r;
        nn[e] = n0 + 16 * g + 4 * j + c;
        v[e] = acc[4 * t + c][j];
      }
  skinny_store<16 * MT>(p, mm, nn, v);
}


// ---- bf16 NT GEMM with both operands by LDS-DMA (configs[4]'s bf16 mode, A already bf16) -------------
// gemm_bf16_nt_kernel stages A and W through VGPRs (global load -> ds_write, a __syncthreads per K tile):
// 0.55-0.70x hipBLASLt on the configs[4] shapes (profiles/r06/bf16_vs_hipblaslt.log). With A already bf16
// (a producer rounded it: the LayerNorm twin, the GELU / attention outputs) both operands can go HBM / L2 ->
// LDS by global_load_lds_dwordx4 with no VGPR staging: a ring of NSTAGE = 3 LDS stages of 64-deep K tiles,
// DMAs two tiles ahead, ONE s_barrier per K tile after a counted vmcnt that leaves the next tile's DMAs in
// flight (MI355X guide §5 "glds with >1 tile in flight across the barrier"; the DMAs are inline asm, so
// hipcc's own waits never drain them early). LDS image per stage and operand: gemm_bf16_nt_kernel's
// swizzled rows (128-B row r holds K group q at 16-B slot q ^ bswz(r)); a DMA wave-instruction fills 8
// whole rows (full 128-B lines; the swizzle is applied to the per-lane SOURCE address), the 16x16x32
// fragment reads of a 16-lane group hit 16 distinct slots. (A [q][row] image, 64 rows of one K group per
// instruction, reads 16 B of 64 different lines per DMA: 0.55-0.65x the register-staged kernel.) Wave tiles
// 64 x 64 (256 x 128 tiles) or 32 x 64 (128 x 128). fp32 or bf16 C through gemm_bf16_nt_kernel's epilogues.
__device__ __forceinline__ void dma16(const void* g, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_base)
               : "memory", "m0");
}
__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(size_t)((const __attribute__((address_space(3))) void*)p);
}

template <int BM, int BN, int WAVES_M, int WAVES_N, bool CBF>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) __attribute__((amdgpu_waves_per_eu(1, 2)))
void gemm_bf16_dma_kernel(GemmP p) {
  constexpr int NWV = WAVES_M * WAVES_N, NSTAGE = 3;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int PA = BM * 8, PB = BN * 8, STAGE = PA + PB;   // 16-B units per operand image / stage
  constexpr int IA = PA / 64 / NWV, IW = PB / 64 / NWV;        // DMA wave-instructions per wave per stage
  static_assert(IA * 64 * NWV == PA && IW * 64 * NWV == PB && BM % 64 == 0 && BN % 64 == 0,
                "stage units must split evenly over the waves, 64 rows per instruction");
  static_assert(IA + IW == 6 || IA + IW == 4, "the vmcnt immediates below count 4 or 6 DMAs per stage");
  __shared__ uint4 smem[NSTAGE * STAGE];   // ONE shared array (a second one can de-pipeline the DMA waits)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int wgid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  int m0, n0;
  if (p.group_m > 1) {
    const int gm = p.group_m, per = gm * gridDim.x, grp = wgid / per;
    const int rows = min(gm, (int)gridDim.y - grp * gm), r = wgid - grp * per;
    m0 = (grp * gm + r % rows) * BM;
    n0 = (r / rows) * BN;
  } else {
    n0 = (wgid % gridDim.x) * BN;
    m0 = (wgid / gridDim.x) * BM;
  }
  const unsigned short* A = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* W = reinterpret_cast<const unsigned short*>(p.B);
  // per-lane DMA sources (rows past M / N re-read the last row; their outputs are never stored) and the
  // wave-uniform LDS bases of its DMA slots in stage 0
  const unsigned short* asrc[IA];
  unsigned adst[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = 8 * (wave * IA + j) + (lane >> 3), q = (lane & 7) ^ bswz(row);
    asrc[j] = A + (long)min(m0 + row, p.M - 1) * p.lda + 8 * q;
    adst[j] = __builtin_amdgcn_readfirstlane(lds_u32(&smem[(wave * IA + j) * 64]));
  }
  const unsigned short* wsrc[IW];
  unsigned wdst[IW];
#pragma unroll
  for (int j = 0; j < IW; ++j) {
    const int row = 8 * (wave * IW + j) + (lane >> 3), q = (lane & 7) ^ bswz(row);
    wsrc[j] = W + (long)min(n0 + row, p.N - 1) * p.ldb + 8 * q;
    wdst[j] = __builtin_amdgcn_readfirstlane(lds_u32(&smem[PA + (wave * IW + j) * 64]));
  }
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = p.K / 64;
  auto dma = [&](int stage, int t) {   // tile t's slice of this wave, unconditional (clamped re-read)
    const int k0 = 64 * min(t, nk - 1);
#pragma unroll
    for (int j = 0; j < IA; ++j) dma16(asrc[j] + k0, adst[j] + stage * STAGE * 16);
#pragma unroll
    for (int j = 0; j < IW; ++j) dma16(wsrc[j] + k0, wdst[j] + stage * STAGE * 16);
  };
  auto compute = [&](const uint4* S) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = 4 * s + (lane >> 4);
      bf16x8_t bf[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + 16 * j + (lane & 15);
        bf[j] = __builtin_bit_cast(bf16x8_t, S[PA + row * 8 + (q ^ bswz(row))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm + 16 * i + (lane & 15);
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, S[row * 8 + (q ^ bswz(row))]);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  dma(0, 0);
  dma(1, 1);
  int stage = 0;
  for (int t = 0; t < nk; ++t) {
    // own tile-t DMAs landed (tile t+1's may still fly), then everyone's; stage t-1 is free again
    if constexpr (IA + IW == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    dma(stage == 0 ? 2 : stage - 1, t + 2);
    compute(smem + stage * STAGE);
    stage = stage == 2 ? 0 : stage + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA into LDS outlives the loop
  if constexpr (CBF) {
    // bf16 C through LDS (gemm_bf16_nt_kernel's CBF epilogue): each wave rounds its WM x WN sub-tile into its
    // own LDS region, then stores 16-B row chunks
    static_assert(NWV * WM * WN * 2 <= (int)sizeof(smem), "bf16 tile must fit the LDS stages");
    __syncthreads();
    unsigned short* T = reinterpret_cast<unsigned short*>(smem) + wave * (WM * WN);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = 16 * j + (lane & 15), col = min(n0 + wn + cl, p.N - 1);
      const float bj = p.bias ? p.bias[col] : 0.f, cs = p.colscale ? p.colscale[col] : 1.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = 16 * i + 4 * (lane >> 4) + r;
          float v = apply_act(p.alpha * acc[i][j][r] + bj, p.act);
          if (p.aux) v *= p.aux[(long)min(m0 + wm + rl, p.M - 1) * p.ld_aux + col];
          T[rl * WN + cl] = __builtin_bit_cast(unsigned short, (__bf16)(v * cs));
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed (wave-private region)
    __builtin_amdgcn_wave_barrier();
    constexpr int CPR = WN / 8;           // 16-B chunks per row
    unsigned short* C = reinterpret_cast<unsigned short*>(p.C);
#pragma unroll
    for (int it = 0; it < WM * CPR / 64; ++it) {
      const int q = lane + 64 * it, rl = q / CPR, c8 = (q % CPR) * 8;
      const int row = m0 + wm + rl, col = n0 + wn + c8;
      const uint4 u = *reinterpret_cast<const uint4*>(T + rl * WN + c8);
      if (row < p.M && col < p.N) *reinterpret_cast<uint4*>(C + (long)row * p.ldc + col) = u;
    }
  } else {
    store_tile_mf<16, TM, TN, BM, BN>(p, acc, 0, 0, m0, n0, wm, wn, lane);
  }
}

}  // namespace

struct Plan { int cfg, splitk, kchunk; int64_t ws; int sk_grid, sk_dp, sk_tiles, sk_ipt; int group_m; };

// Leading words of every GEMM workspace: stream-K arrival counters (zero on allocation, re-armed
// to zero by each call). Split-K partials and stream-K slabs follow.
constexpr int64_t kCntWords = 16384;
constexpr int64_t kCntBytes = kCntWords * 4;

static int num_cus() {
  static int n[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}

// non-stream-K twin of a stream-K configuration (same tile and kernel body)
static int sk_twin(int cfg) {
  switch (cfg) {
    case 31: return 21;
    case 32: return 24;
    case 33: return 25;
    case 34: return 26;
    default: return 27;
  }
}

static int g_force_cfg = -2;   // DASA_GEMM_CFG=<index> pins a tile config (tuning sweeps)
static int g_force_group = -2; // DASA_GEMM_GROUP=<n> pins the L2 group height (tuning sweeps)

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
  // NT operands with K % 64 == 0 (the nn.Linear forward) take the 64-deep K kernels where they win
  // (profiles/r01c/gemm_k64_sk.txt): 128x128 / 64x128 tiles on large problems, and stream-K 64x64
  // tiles at four workgroups per CU on mid-size long-K problems (no quantisation tail).
  const bool nt64 = d->opA == 0 && d->opB == 1 && K % 64 == 0 && M > 32;
  int sk_occ = 1;
  // Short GEMMs (33..192 rows, < 160 64x64 tiles: the B = 2 finetune's language / LXRT projections) are
  // bound by one CU's fp32 MFMA rate on too few tiles: 32x64 tiles, K split to ~240 (K <= 1024) or ~480
  // workgroups (profiles/r03/gemm_split_probe.txt: 160x768x768 18.8 -> 9.8 us, 160x768x3072 28 -> 18 us).
  const bool short_m = M > 32 && M <= 192 && batch == 1 && t64 < 160;
  if (short_m) pl.cfg = 5;
  else if (nt64 && t64 >= 2048) pl.cfg = N >= 2048 ? 27 : 25;
  else if (nt64 && K >= 1536 && t64 >= 128) { pl.cfg = 34; sk_occ = 4; }
  else if (M <= 32) pl.cfg = 5;
  else if (d->opA == 1 && K >= 8192 && t64 >= 256) pl.cfg = 8;   // weight grads over many rows
  else if (t64 >= 2048) pl.cfg = 6;                              // profiles/r01/gemm_grid_v4.txt
  else if (t64 >= 800) pl.cfg = 4;
  else if (t64 >= 400) pl.cfg = (t64 >= 500 && K < 1536) ? 5 : 4;
  else if (t64 >= 250 && (K < 1536 || t64 >= 320)) pl.cfg = 5;
  else pl.cfg = 4;
  // forced value = cfg + 64 * split + 4096 * group (tuning sweeps)
  const int fval = g_force_cfg < (1 << 20) ? g_force_cfg : -1;   // >= 1 << 20: a bf16 configuration
  const int fcfg = fval >= 0 ? fval % 64 : -1, fsplit = fval >= 0 ? (fval / 64) % 64 : 0;
  const int fgroup = fval >= 0 ? fval / 4096 : 0;
  if (fcfg >= 0 && fcfg < kNumCfgs) pl.cfg = fcfg;
  const int bm = kCfgs[pl.cfg].bm, bn = kCfgs[pl.cfg].bn;
  const long blocks = tiles(bm, bn);
  int splitk = 1;
  if (short_m) {
    if (blocks < 128) {
      splitk = (int)cdiv(K <= 1024 ? 240 : 480, blocks);
      const int maxs = std::min(8, K / 128);
      splitk = std::max(1, std::min(splitk, maxs));
    }
  } else if (M <= 32) {
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
  // split partials: [split][b][M][N] for splitk_reduce_kernel, or one BM x BN slab per (tile, split) for the
  // in-kernel reduction of gemm_f32_kernel (padded tiles): room for either
  pl.ws = splitk > 1 ? (int64_t)splitk * batch * (cdiv(M, bm) * bm) * (cdiv(N, bn) * bn) * (int64_t)sizeof(float) : 0;
  pl.sk_grid = pl.sk_dp = pl.sk_tiles = pl.sk_ipt = 0;
  // 64-deep K tiles over many row panels walk 4-panel groups (profiles/r01e/gemm_k32_group.txt: +1-5%
  // on the 12800-row language GEMMs, never slower)
  pl.group_m = fgroup > 0 ? fgroup : ((pl.cfg == 25 || pl.cfg == 27) && cdiv(M, bm) >= 8 ? 4 : 1);
  if (kCfgs[pl.cfg].sk) {
    const int ipt = K / 64;
    const long nt = blocks;
    int G = num_cus() * (fsplit > 0 ? fsplit : sk_occ);
    long dp = nt >= 2L * G ? (nt / G - 1) * G : 0;
    const long I = (nt - dp) * ipt;
    if (G > I) G = (int)I;
    if (K % 64 != 0 || ipt == 0 || nt - dp > kCntWords || G <= 0) {
      pl.cfg = sk_twin(pl.cfg);    // not stream-K-able: the same tile, one workgroup per tile
    } else {
      pl.splitk = 1;
      pl.kchunk = K;
      pl.sk_grid = G;
      pl.sk_dp = (int)dp;
      pl.sk_tiles = (int)nt;
      pl.sk_ipt = ipt;
      pl.ws = 2LL * G * bm * bn * (int64_t)sizeof(float);
    }
  }
  pl.ws += kCntBytes;
  return pl;
}

// Skinny plan (gemm_skinny_*_kernel): M <= 32, one batch, X K-contiguous, W either [N][K] (NT, the
// nn.Linear forward) or [K][N] (NN, dX = dY . W), 16-B aligned float4-able rows. KS (32-deep steps per
// wave) is the largest that still gives >= `target` waves (default 1024 = 4 per CU: enough W requests
// in flight to stream HBM), the K range left over is split across workgroups.
struct SkinnyPlan { bool ok, nn; int mt, xr, ks, cols, splits; int64_t ws; };
static int g_skinny_waves = -2;   // DASA_SKINNY_WAVES=<n>: target wave count; 0 disables the skinny kernels
static int g_skinny_ks = -2;      // DASA_SKINNY_KS=<1|2|4|8>: pin KS (sweeps)
static int g_skinny_hybrid = -2;  // DASA_SKINNY_HYBRID=0: 17..20-row NT GEMMs on two MFMA tiles instead

static SkinnyPlan skinny_plan(const dasa_gemm_desc* d) {
  if (g_skinny_waves == -2) {
    const char* e = getenv("DASA_SKINNY_WAVES");
    g_skinny_waves = e ? atoi(e) : -1;
    const char* e2 = getenv("DASA_SKINNY_KS");
    g_skinny_ks = e2 ? atoi(e2) : -1;
  }
  SkinnyPlan sp{};
  const int M = d->M, N = d->N, K = d->K;
  if (g_skinny_waves == 0 || d->batch > 1 || M < 1 || M > 32 || N < 1 || d->opA != 0 || K < 4 || (K & 3)) return sp;
  const bool nn = d->opB == 0;
  const uintptr_t am = (uintptr_t)d->A | (uintptr_t)d->B;
  if ((am & 15) || (d->lda & 3) || (d->ldb & 3) || (nn && (N & 3))) return sp;
  sp.nn = nn;
  if (g_skinny_hybrid == -2) {
    const char* e = getenv("DASA_SKINNY_HYBRID");
    g_skinny_hybrid = e ? atoi(e) : 1;
  }
  sp.mt = M <= 16 ? 1 : 2;
  sp.xr = 0;
  if (!nn && M > 16 && M <= 20 && g_skinny_hybrid) {
    sp.mt = 1;
    sp.xr = 4;
  }
  const long ksteps = cdiv(K, 32);
  sp.cols = (int)(nn ? cdiv(N, 64) : cdiv(N, 16));
  // target: 1024 waves for the NT form at M > 16 (two tiles or the hybrid), 512 otherwise
  // (tools/skinny_probe.py sweeps, profiles/r02/skinny_probe*.txt); the first KS from the top that reaches it while padding the K range
  // by <= 10 % (K steps beyond K still issue their MFMAs on zeros)
  const long target = g_skinny_waves > 0 ? g_skinny_waves : (!nn && (sp.mt == 2 || sp.xr) ? 1024 : 512);
  const int kmax = nn ? (sp.mt == 2 ? 2 : 4) : 8;
  int ks = kmax;
  for (; ks > 1; ks >>= 1) {
    const long spl = cdiv(ksteps, 4 * ks);
    if ((long)sp.cols * spl * 4 >= target && (spl * 4 * ks - ksteps) * 10 <= ksteps) break;
  }
  if (g_skinny_ks > 0) {
    ks = 1;
    while (ks * 2 <= g_skinny_ks && ks * 2 <= kmax) ks *= 2;
  }
  sp.ks = ks;
  const long splits = cdiv(ksteps, 4 * ks);
  const int nacc = nn ? 4 * sp.mt : sp.mt + (sp.xr ? 1 : 0);
  const int64_t slab = (int64_t)sp.cols * splits * nacc * 64 * 16;
  if (splits > 65535 || (splits > 1 && (sp.cols > kCntWords || slab >= (1LL << 31)))) return sp;
  sp.splits = (int)splits;
  sp.ws = splits > 1 ? kCntBytes + slab : 0;
  sp.ok = true;
  return sp;
}

template <int MT, int KS>
static void skinny_launch(bool nn, dim3 grid, hipStream_t st, const GemmP& p, const SkinnyP& s, int xr = 0) {
  if constexpr (MT == 1) {
    if (xr) {
      hipLaunchKernelGGL((gemm_skinny_nt_kernel<1, KS, 4>), grid, dim3(256), 0, st, p, s);
      return;
    }
  }
  if constexpr (KS <= 4) {
    if (nn) {
      hipLaunchKernelGGL((gemm_skinny_nn_kernel<MT, KS>), grid, dim3(256), 0, st, p, s);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_skinny_nt_kernel<MT, KS>), grid, dim3(256), 0, st, p, s);
}

static int launch_skinny(const SkinnyPlan& pl, const GemmP& p, void* ws, hipStream_t st) {
  SkinnyP s{};
  s.splits = pl.splits;
  if (pl.splits > 1) {
    s.cnt = (unsigned*)ws;
    s.slab = (float*)((char*)ws + kCntBytes);
  }
  const dim3 grid(pl.cols, pl.splits);
  if (pl.mt == 1) {
    switch (pl.ks) {
      case 1: skinny_launch<1, 1>(pl.nn, grid, st, p, s, pl.xr); break;
      case 2: skinny_launch<1, 2>(pl.nn, grid, st, p, s, pl.xr); break;
      case 4: skinny_launch<1, 4>(pl.nn, grid, st, p, s, pl.xr); break;
      default: skinny_launch<1, 8>(pl.nn, grid, st, p, s, pl.xr); break;
    }
  } else {
    switch (pl.ks) {
      case 1: skinny_launch<2, 1>(pl.nn, grid, st, p, s); break;
      case 2: skinny_launch<2, 2>(pl.nn, grid, st, p, s); break;
      case 4: skinny_launch<2, 4>(pl.nn, grid, st, p, s); break;
      default: skinny_launch<2, 8>(pl.nn, grid, st, p, s); break;
    }
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_gemm_skinny_tune(int target_waves, int ks) {
  // ks >= 16: the 17..20-row hybrid form off (KS pinned to ks - 16, or the plan's at 16) - sweeps
  // compare it with two MFMA tiles
  g_skinny_hybrid = ks >= 16 ? 0 : 1;
  g_skinny_waves = target_waves;
  g_skinny_ks = ks >= 16 ? (ks > 16 ? ks - 16 : -1) : ks;
  return 0;
}

// DASA_X6_FORM=<form>: A/B override of the default non-split bf16x6 form (the split-K plan keeps form 8)
static int g_x6_form = -1;
static int x6_form_override() {
  if (g_x6_form < 0) {
    const char* e = getenv("DASA_X6_FORM");
    g_x6_form = e ? atoi(e) : 0;
  }
  return g_x6_form;
}

// DASA_X6_GROUP=<g>: A/B of the bf16x6 tile order (g > 1: g row panels per L2 group, walked column by
// column — the default 4; g < -1: -g column panels per group, walked row by row; 1: plain row-major)
static int g_x6_group = 0x7fffffff;
static int x6_group_override() {
  if (g_x6_group == 0x7fffffff) {
    const char* e = getenv("DASA_X6_GROUP");
    g_x6_group = e ? atoi(e) : 0;
  }
  return g_x6_group;
}

// DASA_X6_BALANCE: 0 = no split-K on many-tile problems (default), 1 = 2- or 3-way, 2 = 2-way only. Off:
// measured slower in isolation on every shape but 12800 x 768 x 3072 (+4 %; 1600 x 4096 x 768 -23 %,
// 720 x 3072 x 768 -20 %) and within run-to-run noise in the training iteration (3359-3604 on vs
// 3550-3558 off, profiles/r03/x6_balance_ab.txt): the split slabs cost more than the idle tail saves.
static int g_x6_balance = -1;
static int x6_balance() {
  if (g_x6_balance < 0) {
    const char* e = getenv("DASA_X6_BALANCE");
    g_x6_balance = (e && (e[0] == '1' || e[0] == '2')) ? e[0] - '0' : 0;
  }
  return g_x6_balance;
}

extern "C" int dasa_gemm_x6_set_balance(int32_t mode) {
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  g_x6_balance = mode;
  return 0;
}

extern "C" int dasa_gemm_force_config(int cfg) {
  g_force_cfg = cfg;
  if (cfg < 0) g_force_group = -1;
  return kNumCfgs;
}

extern "C" int64_t dasa_gemm_f32_workspace(const dasa_gemm_desc* d) {
  if (!d || d->M < 0 || d->N < 0 || d->K < 0) return 0;
  const SkinnyPlan sk = skinny_plan(d);
  if (sk.ok && g_force_cfg < 0) return sk.ws;
  return make_plan(d).ws;
}

extern "C" int dasa_gemm_f32(const dasa_gemm_desc* d, void* ws, int64_t ws_bytes, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  Plan pl = make_plan(d);
  if (ws == nullptr || ws_bytes < pl.ws) {  // no (or too small a) workspace: single pass, no stream-K
    pl.splitk = 1;
    pl.kchunk = K > 0 ? (int)(cdiv(K, 64) * 64) : 64;
    if (kCfgs[pl.cfg].sk) pl.cfg = sk_twin(pl.cfg);
    pl.sk_grid = 0;
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
  p.ws = ws ? (float*)((char*)ws + kCntBytes) : nullptr;
  if (g_force_group == -2) {
    const char* e = getenv("DASA_GEMM_GROUP");
    g_force_group = e ? atoi(e) : -1;
  }
  p.group_m = g_force_group > 0 ? g_force_group : pl.group_m;
  if (g_force_cfg < 0) {
    const SkinnyPlan skp = skinny_plan(d);
    if (skp.ok && (skp.splits == 1 || (ws != nullptr && ws_bytes >= skp.ws)))
      return launch_skinny(skp, p, ws, (hipStream_t)stream);
  }
  SkP sk{};
  if (pl.sk_grid > 0) {
    sk.grid = pl.sk_grid;
    sk.dp = pl.sk_dp;
    sk.tiles = pl.sk_tiles;
    sk.ipt = pl.sk_ipt;
    sk.tiles_n = (int)cdiv(N, kCfgs[pl.cfg].bn);
    sk.tiles_mn = (int)(cdiv(M, kCfgs[pl.cfg].bm) * sk.tiles_n);
    sk.cnt = (unsigned*)ws;
    sk.slab = p.ws;
  }
  hipStream_t st = (hipStream_t)stream;
  int rc;
  const int kalign = pl.cfg >= 21 ? 63 : 31;
  const bool glds_ok = vec && d->opA == 0 && d->opB == 1 && (K & kalign) == 0 && (pl.kchunk & kalign) == 0;
  // gemm_f32_kernel forms (tile configs 0..14, and every config without float4 operands) reduce their
  // K splits in-kernel when the workspace holds one tile slab per (tile, split)
  p.cnt = nullptr;
  const int ecfg = (kCfgs[pl.cfg].glds && !glds_ok) ? glds_fallback(pl.cfg) : pl.cfg;   // launch_cfg's choice
  const bool tile_kernel = !vec || !kCfgs[ecfg].glds;
  if (pl.splitk > 1 && tile_kernel && ws != nullptr) {
    const int bm = vec ? kCfgs[ecfg].bm : (kCfgs[ecfg].bm == 32 ? 32 : 64);
    const int bn = vec ? kCfgs[ecfg].bn : (kCfgs[ecfg].bm == 32 ? 128 : 64);
    const long ntile = cdiv(M, bm) * cdiv(N, bn) * batch;
    const int64_t slabs = ntile * pl.splitk * (int64_t)bm * bn * 4;
    if (ntile <= kCntWords && slabs < 0x7fffffffLL && kCntBytes + slabs <= ws_bytes) p.cnt = (unsigned*)ws;
  }
  rc = launch_cfg(pl.cfg, vec, glds_ok, p, pl.sk_grid > 0 ? &sk : nullptr, d->opA, d->opB, st);
  if (rc) return rc;
  if (pl.splitk > 1 && p.cnt == nullptr) {
    const long total = (long)batch * M * N;
    int grid = (int)cdiv(total, 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, p);
    DASA_CHECK_LAUNCH();
  }
  return 0;
}

// bf16 plan: 128x128 tiles of 8 waves (4x2 of 32x64; 64 KB LDS, two workgroups per CU), or 256x256 tiles
// of 16 waves on large problems (profiles/r01e/gemm_bf16.txt, profiles/r02/gemm_bf16_sweep.txt); the
// other tile/wave/prefetch forms stay for sweeps: dasa_gemm_force_config(kBf16Force + cfg), cfg 0..10.
constexpr int kBf16Force = 1 << 20;
constexpr int kX6Force = 1 << 21;   // dasa_gemm_force_config(kX6Force + cfg): bf16x6 tile forms 0..5

extern "C" int dasa_gemm_bf16(const dasa_gemm_desc* d, void* stream) { return dasa_gemm_bf16_ex(d, 0, stream); }

static int g_bf16_dma = -1;   // the LDS-DMA bf16 probe form: -1 = not read from DASA_BF16_DMA yet
extern "C" int dasa_gemm_bf16_dma(int32_t on) {
  if (g_bf16_dma < 0) {
    const char* e = getenv("DASA_BF16_DMA");
    g_bf16_dma = (e && e[0] == '1') ? 1 : 0;
  }
  const int prev = g_bf16_dma;
  if (on >= 0) g_bf16_dma = on ? 1 : 0;
  return prev;
}

extern "C" int dasa_gemm_bf16_ex(const dasa_gemm_desc* d, int32_t flags, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  const bool abf = flags & DASA_BF16_A, cbf = flags & DASA_BF16_C;
  if (M < 0 || N < 0 || K < 0 || d->opA != 0 || d->opB != 1) return (int)hipErrorInvalidValue;
  if (flags & ~(DASA_BF16_A | DASA_BF16_C)) return (int)hipErrorInvalidValue;
  if (K % 64 != 0 || (d->lda & (abf ? 7 : 3)) || (d->ldb & 7) || d->lda < K || d->ldb < K || d->ldc < N)
    return (int)hipErrorInvalidValue;
  if (cbf && (d->beta != 0.f || ((uintptr_t)d->C & 15) || (N & 7) || (d->ldc & 7) || (batch > 1 && (d->strideC & 7))))
    return (int)hipErrorInvalidValue;
  if (abf && batch > 1 && (d->strideA & 7)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15) || (batch > 1 && ((d->strideA & 3) || (d->strideB & 7))))
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
  p.ws = nullptr;
  // 256x256 tiles of 16 waves (128 KB LDS, one workgroup per CU) once there are >= 200 of them:
  // +8-25% over 128x128 on the configs[4] shapes (profiles/r02/gemm_bf16_sweep.txt)
  int cfg = cdiv(M, 256) * cdiv(N, 256) * batch >= 200 ? 9 : 2;
  if (g_force_cfg >= kBf16Force && g_force_cfg < kX6Force) {
    cfg = (g_force_cfg - kBf16Force) % 16;
    if (cfg > 10) return (int)hipErrorInvalidValue;   // forms 0..10 only (the switch below)
  }
  // tile rows / columns of each form, as the kernel instantiations below
  const int bm = (cfg == 1 || cfg == 5 || cfg == 7 || cfg == 9) ? 256 : 128,
            bn = cfg == 3 ? 64 : (cfg == 6 || cfg == 9 || cfg == 10) ? 256 : 128;
  p.group_m = cdiv(M, bm) >= 8 ? 4 : 1;
  dim3 grid((unsigned)cdiv(N, bn), (unsigned)cdiv(M, bm), batch);
  hipStream_t st = (hipStream_t)stream;
  // DASA_BF16_DMA=1 (probe, off by default): A already bf16, one batch -> both operands by LDS-DMA
  // (gemm_bf16_dma_kernel), 256 x 128 tiles when there are >= 240 of them, else 128 x 128. Bitwise equal to
  // the register-staged forms below but 0.8-1.2x them on the configs[4] shapes (profiles/r06/bf16_dma/)
  if (abf && batch == 1 && dasa_gemm_bf16_dma(-1) && !(g_force_cfg >= kBf16Force && g_force_cfg < kX6Force) && (d->ldb & 7) == 0) {
    const bool wide = cdiv(M, 256) * cdiv(N, 128) >= 240;
    p.group_m = cdiv(M, wide ? 256 : 128) >= 8 ? 4 : 1;
    const dim3 gw((unsigned)cdiv(N, 128), (unsigned)cdiv(M, 256)), gs((unsigned)cdiv(N, 128), (unsigned)cdiv(M, 128));
    hipStream_t s2 = (hipStream_t)stream;
    if (wide) {
      if (cbf) hipLaunchKernelGGL((gemm_bf16_dma_kernel<256, 128, 4, 2, true>), gw, dim3(512), 0, s2, p);
      else hipLaunchKernelGGL((gemm_bf16_dma_kernel<256, 128, 4, 2, false>), gw, dim3(512), 0, s2, p);
    } else {
      if (cbf) hipLaunchKernelGGL((gemm_bf16_dma_kernel<128, 128, 4, 2, true>), gs, dim3(512), 0, s2, p);
      else hipLaunchKernelGGL((gemm_bf16_dma_kernel<128, 128, 4, 2, false>), gs, dim3(512), 0, s2, p);
    }
    DASA_CHECK_LAUNCH();
    return 0;
  }
  if (abf || cbf) {   // the bf16-activation forms: the two tile shapes of the default plan
    const dim3 g9((unsigned)cdiv(N, 256), (unsigned)cdiv(M, 256), batch), g2((unsigned)cdiv(N, 128), (unsigned)cdiv(M, 128), batch);
    const bool big = cfg == 9;
    p.group_m = cdiv(M, big ? 256 : 128) >= 8 ? 4 : 1;
#define DASA_BF16_FORM(AB, CB)                                                                              \
    if (big) hipLaunchKernelGGL((gemm_bf16_nt_kernel<256, 256, 4, 4, 1, AB, CB>), g9, dim3(1024), 0, st, p); \
    else hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 4, 2, 1, AB, CB>), g2, dim3(512), 0, st, p);
    if (abf && cbf) { DASA_BF16_FORM(true, true) }
    else if (abf) { DASA_BF16_FORM(true, false) }
    else { DASA_BF16_FORM(false, true) }
#undef DASA_BF16_FORM
    DASA_CHECK_LAUNCH();
    return 0;
  }
  switch (cfg) {
    case 1: hipLaunchKernelGGL((gemm_bf16_nt_kernel<256, 128, 4, 2>), grid, dim3(512), 0, st, p); break;
    case 2: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 4, 2>), grid, dim3(512), 0, st, p); break;
    case 3: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 64, 2, 2>), grid, dim3(256), 0, st, p); break;
    case 4: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 4, 4>), grid, dim3(1024), 0, st, p); break;
    case 5: hipLaunchKernelGGL((gemm_bf16_nt_kernel<256, 128, 8, 2>), grid, dim3(1024), 0, st, p); break;
    case 6: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 256, 2, 4>), grid, dim3(512), 0, st, p); break;
    case 7: hipLaunchKernelGGL((gemm_bf16_nt_kernel<256, 128, 4, 2, 2>), grid, dim3(512), 0, st, p); break;
    case 8: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 4, 2, 2>), grid, dim3(512), 0, st, p); break;
    case 9: hipLaunchKernelGGL((gemm_bf16_nt_kernel<256, 256, 4, 4>), grid, dim3(1024), 0, st, p); break;
    case 10: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 256, 2, 4, 2>), grid, dim3(512), 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 2, 2>), grid, dim3(256), 0, st, p); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

// bf16x6 plan: forms 0..9 = tile / accumulator / prefetch variants, 15 = 128x128 one accumulator, 16 =
// all-DMA 128x128 (3 x 40 KB ring; 256x128 would need 168 KB), 20 = form 8 with one LDS stage in <= 128
// registers (two workgroups per CU) (sweeps: dasa_gemm_force_config(kX6Force + cfg + 32 * splitk)). r03
// also measured and removed a ping-pong form (wave groups offset by half a K step), inline-asm stage
// loads (0.90-0.98x form 8, profiles/r03/x6_forms_pp_asm.txt) and small-tile high-occupancy forms
// (x6_occupancy_forms_rejected.txt). Default: 128x128 tiles, separate small-term accumulator, two
// register stages of prefetch (form 8) on every shape with >= 128 output tiles (profiles/r02/
// gemm_x6_sweep_b.txt: 136-178 fp32-equivalent TFLOP/s on the 1600- to 20480-row language / LXRT / LSTM
// shapes), 256x128 (form 7) on the wide >= 4096-row ones, form 20 on short-K wide ones with >= 256
// tiles (below). Fewer tiles (the 720- / 1600-row LXRT and vision GEMMs: 36-108
// tiles) split K over the tiles' workgroups until ~256 workgroups fill the chip, reduced in-kernel by
// the last split to arrive (X6Split); needs the workspace.
struct X6Plan { int cfg, bm, bn, splitk, kchunk; int64_t ws; };


static bool x6_lds1() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("DASA_X6_LDS1");
    on = !(e && e[0] == '0');
  }
  return on != 0;
}

// tile rows / columns of each bf16x6 form (the kernel instantiations of dasa_gemm_f32x6_ws)
static int x6_form_bm(int cfg) {
  return (cfg == 1 || cfg == 3 || cfg == 6 || cfg == 7 || cfg == 12 || cfg == 13) ? 256
         : (cfg == 4 || cfg == 5 || cfg == 28) ? 64 : 128;
}
static int x6_form_bn(int cfg) { return (cfg == 5 || cfg == 27) ? 64 : 128; }

static X6Plan x6_plan(const dasa_gemm_desc* d) {
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  X6Plan pl{8, 128, 128, 1, K, 0};
  int fsplit = 0;
  // 256x128 tiles (form 7: the same products and order as form 8, bitwise equal) on the wide
  // 12800-row language GEMMs: +4-8 % on 12800 x 2304 / 3072 x 768, slower on N = 768 and on fewer rows
  // (profiles/r02/x6_forms.txt)
  if (M >= 4096 && N >= 2048) pl.cfg = 7;
  // form 20 (one LDS stage, two workgroups per CU) on short-K wide problems with >= 256 tiles: 12800 x
  // {3072, 2304} x 768 1.07-1.08x form 7, 1600 x {3072, 4096} x 768 1.11-1.14x form 8; slower at K = 3072,
  // N = 768 and below ~2 tiles per CU (profiles/r03/x6_lds1_forms.txt). DASA_X6_LDS1=0 turns it off (A/B).
  if (K <= 1024 && N >= 2048 && (long)cdiv(M, 128) * cdiv(N, 128) * batch >= 256 && x6_lds1()) pl.cfg = 20;
  if (g_force_cfg >= kX6Force) {
    pl.cfg = (g_force_cfg - kX6Force) % 32;
    fsplit = ((g_force_cfg - kX6Force) / 32) % 64;
  }
  pl.bm = x6_form_bm(pl.cfg);
  pl.bn = x6_form_bn(pl.cfg);
  const long tiles = (long)cdiv(M, pl.bm) * cdiv(N, pl.bn) * batch;
  // split count (profiles/r02/gemm_x6_splitk.txt): the most splits that keep tiles x splits <= 256
  // (one wave of workgroups) with >= 8 32-deep K steps per split; forced splits may go to 4 steps
  int splitk = 1;
  if (fsplit > 0) splitk = fsplit < K / 128 ? fsplit : K / 128;
  else if (tiles < 128) splitk = (int)(256 / tiles) < K / 256 ? (int)(256 / tiles) : K / 256;
  else if (pl.cfg == 8 && x6_balance() > 0) {
    // (opt-in, see x6_balance) many tiles, one workgroup per CU: the last round of tiles can leave most
    // of the chip idle (12800 x 768: 600 tiles = 2.34 rounds -> 78 % of the CU-time busy). Split K 2- or
    // 3-way when that fills the rounds at least 8 points better (2 splits: 4.69 rounds -> 94 %) and every
    // split keeps >= 8 K steps; the split partials are reduced in-kernel by the last arriver.
    const double cus = (double)num_cus();
    auto fill = [&](int s) { const double u = (double)tiles * s / cus; return u / ceil(u); };
    double best = fill(1);
    for (int s = 2; s <= (x6_balance() == 2 ? 2 : 3); ++s)
      if (K / s >= 256 && fill(s) > best + 0.08) { best = fill(s); splitk = s; }
  }
  const bool spl_form = pl.cfg == 8 || pl.cfg == 4 || pl.cfg == 5;
  if (!spl_form || splitk < 1 || tiles * splitk > 32767 || tiles > kCntWords) splitk = 1;
  if (splitk > 1) {
    pl.kchunk = (int)(cdiv(cdiv(K, splitk), 32) * 32);
    pl.splitk = (int)cdiv(K, pl.kchunk);
  }
  if (pl.splitk > 1) pl.ws = kCntBytes + tiles * pl.splitk * (int64_t)pl.bm * pl.bn * (int64_t)sizeof(float);
  else if (g_force_cfg < kX6Force && x6_form_override() > 0) {   // A/B: DASA_X6_FORM replaces forms 7 / 8
    pl.cfg = x6_form_override();
    pl.bm = x6_form_bm(pl.cfg);
    pl.bn = x6_form_bn(pl.cfg);
  }
  return pl;
}


// fp32-accurate GEMM on bf16 MFMA (bf16x6 split; see gemm_f32x6_nt_kernel). d->B = the hi plane of
// the pre-split weight, planes `plane` bf16 elements apart. ws (zero-initialised once, counters
// re-armed by every call; dasa_gemm_f32x6_workspace bytes) enables the split-K form; without it every
// problem runs one workgroup per tile.
// Whole rounds + split-K tail (r05): a many-tile problem whose last round of workgroups would leave most
// CUs idle (12800 x 768: 600 tiles of 128 x 128 = 2.34 rounds of 256 CUs -> 78 % of the CU-time busy;
// 11200 x 768: 2.06 rounds -> 69 %) runs as TWO launches over row bands: the first M1 rows as whole rounds
// of the planned form, then the remaining rows as 128 x 128 tiles with K split so that they fill one round
// (the X6Split form: partials reduced in-kernel by the last split, in split order — deterministic). Taken
// when the cost model (rounds x tile work) promises >= 10 % less; DASA_X6_TAIL=0 turns it off (A/B).
struct X6Tail { int M1; X6Plan dp, rem; };

static int g_x6_tail = -1;
static bool x6_tail_on() {
  if (g_x6_tail < 0) {
    const char* e = getenv("DASA_X6_TAIL");
    g_x6_tail = !(e && e[0] == '0');
  }
  return g_x6_tail != 0;
}

// tests / A/B: 1 = whole rounds + split-K tail where the cost model takes it (the default), 0 = one launch
extern "C" int dasa_gemm_x6_set_tail(int32_t on) {
  if (on < 0 || on > 1) return (int)hipErrorInvalidValue;
  g_x6_tail = on;
  return 0;
}

static bool x6_tail_plan(const dasa_gemm_desc* d, const X6Plan& pl, X6Tail& tp) {
  const int M = d->M, N = d->N, K = d->K;
  if (g_force_cfg >= kX6Force || !x6_tail_on() || d->batch > 1 || pl.splitk > 1) return false;
  if (!(pl.cfg == 7 || pl.cfg == 8 || pl.cfg == 20)) return false;
  const long cus = num_cus(), S = cus * (pl.cfg == 20 ? 2 : 1);
  const long tn = cdiv(N, pl.bn), tm = cdiv(M, pl.bm), T = tn * tm;
  const long full = T / S;
  if (full < 1) return false;
  const long panels1 = full * S / tn;   // row panels that make whole rounds
  if (panels1 < 1 || panels1 >= tm) return false;
  const int M1 = (int)panels1 * pl.bm, M2 = M - M1;
  const long t2 = cdiv(M2, 128) * cdiv(N, 128);
  int sk = (int)(cus / t2);
  if (sk > K / 256) sk = K / 256;
  if (sk < 2 || t2 > kCntWords) return false;
  // cost in units of one 128 x 128 tile over the full K on one CU (form 20's two workgroups per CU each
  // take twice as long); the split tail adds ~5 % of a tile for its slab round trip
  const double u = (double)pl.bm * pl.bn / (128.0 * 128.0) * (pl.cfg == 20 ? 2.0 : 1.0);
  const double plain = ceil((double)T / S) * u;
  const double dpsk = (double)full * u + ceil((double)t2 * sk / cus) / sk + 0.05;
  if (dpsk > 0.9 * plain) return false;
  tp.M1 = M1;
  tp.dp = pl;
  tp.rem = X6Plan{8, 128, 128, sk, (int)(cdiv(cdiv(K, sk), 32) * 32), 0};
  tp.rem.splitk = (int)cdiv(K, tp.rem.kchunk);
  tp.rem.ws = kCntBytes + t2 * tp.rem.splitk * (int64_t)128 * 128 * (int64_t)sizeof(float);
  (void)M2;
  return true;
}

static int x6_run(const dasa_gemm_desc* d, X6Plan pl, int64_t plane, void* ws, int64_t ws_bytes, hipStream_t st);

extern "C" int dasa_gemm_f32x6_kernels(const dasa_gemm_desc* d, int64_t ws_bytes) {
  if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0) return 0;
  X6Tail tp;
  return (x6_tail_plan(d, x6_plan(d), tp) && ws_bytes >= tp.rem.ws) ? 2 : 1;
}

extern "C" int64_t dasa_gemm_f32x6_workspace(const dasa_gemm_desc* d) {
  if (!d || d->M < 0 || d->N < 0 || d->K < 0) return 0;
  const X6Plan pl = x6_plan(d);
  X6Tail tp;
  if (x6_tail_plan(d, pl, tp)) return tp.rem.ws > pl.ws ? tp.rem.ws : pl.ws;
  return pl.ws;
}

extern "C" int dasa_gemm_f32x6_ws(const dasa_gemm_desc* d, int64_t plane, void* ws, int64_t ws_bytes, void* stream) {
  if (!d) return (int)hipErrorInvalidValue;
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  if (M < 0 || N < 0 || K < 0 || d->opA != 0 || d->opB != 1) return (int)hipErrorInvalidValue;
  if (K % 32 != 0 || (d->lda & 3) || (d->ldb & 7) || (plane & 7) || d->lda < K || d->ldb < K || d->ldc < N)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15) || (batch > 1 && ((d->strideA & 3) || (d->strideB & 7))))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  const X6Plan pl = x6_plan(d);
  X6Tail tp;
  if (x6_tail_plan(d, pl, tp) && ws != nullptr && ws_bytes >= tp.rem.ws) {
    dasa_gemm_desc d1 = *d, d2 = *d;
    d1.M = tp.M1;
    d2.M = M - tp.M1;
    d2.A = d->A + (long)tp.M1 * d->lda;
    d2.C = d->C + (long)tp.M1 * d->ldc;
    if (d->aux) d2.aux = d->aux + (long)tp.M1 * d->ld_aux;
    const int rc = x6_run(&d1, tp.dp, plane, nullptr, 0, (hipStream_t)stream);
    if (rc) return rc;
    return x6_run(&d2, tp.rem, plane, ws, ws_bytes, (hipStream_t)stream);
  }
  return x6_run(d, pl, plane, ws, ws_bytes, (hipStream_t)stream);
}

static int x6_run(const dasa_gemm_desc* d, X6Plan pl, int64_t plane, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int M = d->M, N = d->N, K = d->K, batch = d->batch < 1 ? 1 : d->batch;
  GemmP p{};
  p.M = M; p.N = N; p.K = K; p.batch = batch; p.splitk = 1; p.kchunk = K;
  p.A = d->A; p.lda = d->lda; p.sA = d->strideA;
  p.B = d->B; p.ldb = d->ldb; p.sB = d->strideB;
  p.C = d->C; p.ldc = d->ldc; p.sC = d->strideC;
  p.bias = d->bias; p.act = d->act;
  p.aux = d->aux; p.ld_aux = d->ld_aux; p.sAux = d->strideAux;
  p.colscale = d->colscale; p.alpha = d->alpha; p.beta = d->beta;
  p.ws = nullptr;
  if (pl.splitk > 1 && (ws == nullptr || ws_bytes < pl.ws)) { pl.splitk = 1; pl.kchunk = K; }
  const int cfg = pl.cfg, bm = pl.bm, bn = pl.bn;
  // tile order: groups of 8 W column panels, A streaming under them (r04 sweep, profiles/r04/x6_group_sweep.txt:
  // 12800 x {3072, 2304} x 768 fetch 460 -> 332 MB / 367 -> 274 MB per launch, time within +-1 %)
  p.group_m = cdiv(M, bm) >= 8 ? -8 : 1;
  if (x6_group_override() != 0) p.group_m = x6_group_override();   // A/B: DASA_X6_GROUP (< -1: along N)
  X6Split xs{};
  if (pl.splitk > 1) {
    xs.cnt = (unsigned*)ws;
    xs.slab = (float*)((char*)ws + kCntBytes);
    xs.splitk = pl.splitk;
    xs.kchunk = pl.kchunk;
    p.group_m = 1;
    dim3 grid((unsigned)cdiv(N, bn), (unsigned)cdiv(M, bm), batch * pl.splitk);
    switch (cfg) {
      case 4: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<64, 128, 2, 2, true, 2, true>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
      case 5: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<64, 64, 2, 2, true, 2, true>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
      default: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2, true>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    }
    DASA_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((unsigned)cdiv(N, bn), (unsigned)cdiv(M, bm), batch);
  switch (cfg) {
    case 1: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, false>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 2: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, false>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 3: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, true>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 4: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<64, 128, 2, 2, true>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
    case 5: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<64, 64, 2, 2, true>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
    case 6: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, false, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 7: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, true, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 8: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 10: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2, false, 1>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 11: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2, false, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 12: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, true, 2, false, 1>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 13: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<256, 128, 4, 2, true, 2, false, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 9: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 3>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 15: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, false, 2>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 16: hipLaunchKernelGGL((gemm_f32x6_dma_kernel<128, 128, 4, 2>), grid, dim3(512), 0, st, p, (long)plane); break;
    case 20: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, -1>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    // forms 27 / 28 (r06 probe, sweep-only): form 20's one LDS stage at half the tile (36 KB, 4 waves) so FOUR
    // workgroups share a CU and three keep their MFMAs going while one splits / stores (form 20: one of two).
    // Bitwise form 8; measured 0.80-0.90x form 20 on the many-tile shapes (profiles/r06/k64/probe_quarter.log):
    // twice the tiles re-read A / W through L2 and the 128-VGPR budget spills 3-9 registers
    case 27: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 64, 2, 2, true, -1>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
    case 28: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<64, 128, 2, 2, true, -1>), grid, dim3(256), 0, st, p, (long)plane, xs); break;
    case 26: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2, false, 3>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
    case 21: hipLaunchKernelGGL((gemm_f32x6_ra_kernel<128, 128, 2, 2>), grid, dim3(256), 0, st, p, (long)plane); break;
    case 22: hipLaunchKernelGGL((gemm_f32x6_ra_kernel<128, 128, 4, 2>), grid, dim3(512), 0, st, p, (long)plane); break;
    default: hipLaunchKernelGGL((gemm_f32x6_nt_kernel<128, 128, 4, 2, true>), grid, dim3(512), 0, st, p, (long)plane, xs); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_gemm_f32x6(const dasa_gemm_desc* d, int64_t plane, void* stream) {
  return dasa_gemm_f32x6_ws(d, plane, nullptr, 0, stream);
}

extern "C" int dasa_f32_split3_bf16(const float* x, int64_t ldx, uint16_t* y, int32_t rows, int32_t cols,
                                    void* stream) {
  if (rows < 0 || cols < 0 || (cols & 7) || (ldx & 3) || ldx < cols || ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return (int)hipErrorInvalidValue;
  const long n = (long)rows * (cols / 8);
  if (n == 0) return 0;
  const int grid = (int)std::min<long>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(split3_bf16_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, (long)ldx,
                     reinterpret_cast<uint4*>(y), rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_f32_to_bf16(const float* x, uint16_t* y, int64_t n, void* stream) {
  if (n < 0 || (n & 1) || ((uintptr_t)x & 7) || ((uintptr_t)y & 3)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const long np = n / 2;
  const int grid = (int)std::min<long>(cdiv(np, 256), 4096);
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x,
                     reinterpret_cast<unsigned*>(y), np);
  DASA_CHECK_LAUNCH();
  return 0;
}
