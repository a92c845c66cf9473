// Persistent (one launch per sequence) bi-LSTM recurrence for the DicEncoder top LSTM
// (r2rmodel.py:2239-2243, 2339-2354), forward and BPTT.
//
// Why: the per-timestep kernels in lstm.hip re-read W_hh (2 x 16 MB fp32) from MALL every step, so a
// step costs ~15 us (fwd) / ~21 us (BPTT) at B = 20. Here each of the 256 workgroups (one per CU, 128
// per direction) keeps its 8-unit slice of W_hh (128 KB) in VGPRs for the whole sequence; a step is
// one MFMA pass over the recurrent state + the cell update, and the directions' workgroups exchange
// the new state through a per-direction counter barrier inside the launch.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md "Valid forms", row 1):
// every handed-off word is stored sc1 (write-through), every storing wave drains vmcnt, the workgroup
// barriers, ONE lane adds to the direction's arrival counter (agent-scope atomic), then polls it with
// sc1 loads (bounded by a wall-clock limit that sets a timeout word instead of hanging); the other
// waves join at a workgroup barrier and read the state with sc1 loads only. (A per-workgroup flag array
// polled by one wave measured slower: profiles/r02/lstm_stamps.txt.)
// Residency: one 1024-thread workgroup per CU, 2*H/8 <= 256 workgroups; the grid is checked against
// the occupancy query once (the caller uses the step kernels if it would not be co-resident). The
// callers run nothing concurrently with it (the encoder's side stream is joined before the LSTM).
// A barrier that times out (a workgroup was not co-resident, e.g. another process or stream held
// CUs) never returns silently: every workgroup that sees the timeout word fills its outputs with NaN
// and ORs a bit into the library's error word (dasa_set_error_word), which the host reads at its next
// sync point and raises on (dasa_amd.ops.check_device_errors).
#include "common.h"
#include "lstm_internal.h"
#include <cstdlib>

namespace {

constexpr int PU = 8;                       // hidden units per workgroup
constexpr int PW = 16;                      // waves per workgroup
constexpr long long kSpinTicks = 20000000;  // 200 ms of the 100 MHz wall clock per barrier wait

__device__ __forceinline__ float4 selz(bool c, float4 v) {
  return make_float4(c ? v.x : 0.f, c ? v.y : 0.f, c ? v.z : 0.f, c ? v.w : 0.f);
}
__device__ __forceinline__ float f4e(const float4& v, int e) {
  return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}
__device__ __forceinline__ float4 ld_sc1(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16 /* sc1 */));
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_store_dword ... sc1
}

// Arrive + wait on the direction's monotonic counter, kept as 8 shards (the arriving workgroup adds to shard
// blockIdx % 8, i.e. its XCD under round-robin placement; the waiter sums all 8): 128 arrivals on ONE word
// serialise at ≈12 ns each (MI355X_MICROARCH.md "fanin": shard the counter per XCD above a few dozen
// arrivers), 16 per shard do not. Shard k of direction d at sync[32 + 16 (8 d + k)] (64 B apart); the
// caller zeroes sync[0 .. 512). Returns false (after setting *tmo) if the other workgroups did not arrive
// within kSpinTicks; every thread of the workgroup gets the answer. `force` (test hook
// dasa_persist_force_timeout) takes the timeout path without waiting.
__device__ bool dir_barrier(unsigned* sync, int dir, unsigned target, unsigned* tmo, float* flag_lds, int force) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x < 64) {                              // wave 0 arrives and polls (uniform loop)
    const int lane = threadIdx.x;
    unsigned* shards = sync + 32 + dir * 8 * 16;
    if (lane == 0) __hip_atomic_fetch_add(shards + (blockIdx.x & 7) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = wall_clock64();
    bool ok = true;
    if (force) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = false;
    }
    // the 8 shards through a buffer resource (lanes >= 8 read past num_records: 0) with sc1, one offset VGPR
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)shards, (short)0, 8 * 16 * 4, 0x00020000);
    while (ok) {
      unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 64, 0, 16 /* sc1 */);
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (__shfl(v, 0, 64) >= target) break;
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > kSpinTicks) {
        if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
      }
    }
    if (lane == 0) *flag_lds = ok ? 1.f : 0.f;
  }
  __syncthreads();
  return *flag_lds != 0.f;
}

// After the recurrence: did any workgroup of this launch time out? (every thread gets the answer)
__device__ bool launch_failed(unsigned* tmo, unsigned* err, unsigned bit, float* flag_lds) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t && err) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_lds = t ? 1.f : 0.f;
  }
  __syncthreads();
  return *flag_lds != 0.f;
}

// ------------------------------------------------------------------------------------- forward
struct PFwd {
  const float* xproj;     // [B][L][2][4H]
  const float* whh0;      // [4H][H]
  const float* whh1;
  const int* len;         // [B]
  float* out;             // [B][L][2H]
  float* save_act;        // [L][2][B][4H] or NULL
  float* save_c;          // [L][2][B][H] or NULL
  float* h_n;             // [2][B][H] or NULL
  float* c_n;
  float* hbuf;            // [2 parity][2 dir][B][H] hand-off
  unsigned* sync;         // [0], [1] arrivals per direction; [2] timeout word (zeroed by the caller)
  unsigned* err;          // library error word (dasa_set_error_word) or NULL
  int force_tmo;          // test hook: every barrier times out
  int B, L, H;
  unsigned long long* stamps;   // diagnostic (dasa_persist_stamps): workgroup 0's per-step phase clocks
};

__device__ __forceinline__ void stamp(unsigned long long* buf, int i) {
  if (buf && blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf[i] = t;
  }
}

// bf16x6 recurrent product (X6): h and the W_hh slice split exactly into three bf16 planes each
// (x = hi + mid + lo), the six kept products (hh, hm, mh, hl, lh, mm) on v_mfma_f32_16x16x32_bf16 —
// fp32-accurate, as gemm.hip's gemm_f32x6_nt_kernel — at 6/16 of the 32x32x2 f32 MFMA cycles per FLOP.
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const f32x2_t w = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(w, bf16x2_t));
}
__device__ __forceinline__ void split3_pair(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  h = pk_bf16(a, b);
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(ra, rb);
  l = pk_bf16(ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u));
}
// 8 consecutive fp32 (x then y) -> the three bf16x8 planes
__device__ __forceinline__ void split3_8(const float4& x, const float4& y, bf16x8_t (&o)[3]) {
  unsigned h0, h1, h2, h3, m0, m1, m2, m3, l0, l1, l2, l3;
  split3_pair(x.x, x.y, h0, m0, l0);
  split3_pair(x.z, x.w, h1, m1, l1);
  split3_pair(y.x, y.y, h2, m2, l2);
  split3_pair(y.z, y.w, h3, m3, l3);
  o[0] = __builtin_bit_cast(bf16x8_t, u32x4{h0, h1, h2, h3});
  o[1] = __builtin_bit_cast(bf16x8_t, u32x4{m0, m1, m2, m3});
  o[2] = __builtin_bit_cast(bf16x8_t, u32x4{l0, l1, l2, l3});
}
// b: the hi and mid planes (VGPRs), blo: the lo plane (read back from LDS)
__device__ __forceinline__ void mfma_x6(const bf16x8_t (&a)[3], const bf16x8_t (&b)[2], const bf16x8_t& blo,
                                        floatx4& big, floatx4& sm) {
  sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], sm, 0, 0, 0);
  sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], blo, sm, 0, 0, 0);
  sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], sm, 0, 0, 0);
  sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], sm, 0, 0, 0);
  sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], sm, 0, 0, 0);
  big = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], big, 0, 0, 0);
}

// NG = H / 128: K-groups of 8 per wave (the wave's K slice is H / 16). NBT = 32-row batch tiles
// (B <= 32 * NBT): every timestep runs the MFMA pass, the 16-wave reduction and the cell update once
// per tile, then ONE direction barrier. Thread i < 256 owns (row i / 8 of every tile, unit i % 8); the
// c / h state of tiles past the first lives in LDS (registers are capped at 128 per lane here).
// X6: the recurrent product on bf16 MFMA (above); the wave's K slice is KS = NG / 4 steps of 32, its
// 32 x 32 output four 16 x 16 tiles; the W_hh slice is split into three bf16 planes once: hi and mid
// live in VGPRs (32), lo in LDS (64 KB per workgroup, lane-linear, read back per product).
template <int NG, int NBT, bool X6 = false>
__global__ __launch_bounds__(1024) void bilstm_persist_fwd_kernel(PFwd a) {
  __shared__ __attribute__((aligned(16))) float smem[PW * 1024 + 4];
  __shared__ float cst[NBT > 1 ? NBT * 256 : 1], hst[NBT > 1 ? NBT * 256 : 1];
  __shared__ uint4 wlo_s[X6 ? PW * 2 * (NG / 4) * 64 : 1];   // X6: [wave][j][K step][lane]
  const int H = a.H, B = a.B, L = a.L, G = H / PU;
  const int dir = blockIdx.x / G, u0 = (blockIdx.x % G) * PU;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 31, hh = lane >> 5;
  const int k0 = w * (8 * NG);
  // This workgroup's 32 W_hh rows (gate q = n / 8 of unit u0 + n % 8), this wave's K slice, in the
  // 32x32x2 B-operand layout with the K-permuted float4 per lane (k = 8g + 4hh + e feeds MFMA e).
  constexpr int KS = X6 ? NG / 4 : 1;
  static_assert(!X6 || (NG % 4 == 0), "X6: the wave's K slice is whole 32-deep steps");
  float4 wf[X6 ? 1 : NG];
  bf16x8_t wx[X6 ? 2 : 1][KS][2];   // X6: [16-column tile j][K step][hi, mid]; lane: col l & 15, k 8(l >> 4)..+7
  if constexpr (!X6) {
    const float* wp = (dir ? a.whh1 : a.whh0) + ((long)(n / PU) * H + u0 + (n % PU)) * H + k0 + 4 * hh;
#pragma unroll
    for (int g = 0; g < NG; ++g) wf[g] = *reinterpret_cast<const float4*>(wp + 8 * g);
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nn = 16 * j + (lane & 15);
      const float* wp = (dir ? a.whh1 : a.whh0) + ((long)(nn / PU) * H + u0 + (nn % PU)) * H + k0 + 8 * (lane >> 4);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8_t t[3];
        split3_8(*reinterpret_cast<const float4*>(wp + 32 * ks), *reinterpret_cast<const float4*>(wp + 32 * ks + 4), t);
        wx[j][ks][0] = t[0];
        wx[j][ks][1] = t[1];
        wlo_s[((w * 2 + j) * KS + ks) * 64 + lane] = __builtin_bit_cast(uint4, t[2]);   // own slot: no barrier
      }
    }
  }

  const bool own = threadIdx.x < 32 * PU;
  const int oi = threadIdx.x / PU, ou = threadIdx.x % PU, uj = u0 + ou;   // row in tile, unit
  float c1 = 0.f, h1 = 0.f;   // NBT == 1: the state stays in registers
  if (NBT > 1 && own) {
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      cst[bt * 256 + threadIdx.x] = 0.f;
      hst[bt * 256 + threadIdx.x] = 0.f;
    }
  }
  const int b = lane & 31;
  // One batch tile (B <= 32: the sampled rollout's per-step launches): the owners' input-projection gates of
  // the NEXT timestep are fetched into LDS by buffer_load ... lds before this step's barrier (they do not
  // depend on the recurrence; no registers held), the lengths once — the cell update then waits on no
  // global load (phase clocks: cell+store 2860 -> 1930 cycles per step at B = 20, r05). The owners are
  // waves 0-3: wave w's 64 lanes fill 64 consecutive words of each gate row. (Multi-tile launches keep the
  // direct loads: their unrolled tile loop spills with the prefetch.)
  constexpr int XQ = NBT == 1 ? 1 : 0;
  __shared__ float xq_s[XQ ? 4 * 256 : 1];
  __shared__ int len_s[XQ ? 256 : 1];
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xproj, (short)0, (int)((long)B * L * 8 * H * 4), 0x00020000);
  const int xvoff = (min(oi, B - 1) * L * 8 * H + uj) * 4;
  auto load_xq = [&](int s_) {
    if (!own) return;   // wave-uniform
    const int t_ = dir == 0 ? s_ : L - 1 - s_;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(xq_s + q * 256 + 64 * w), 4,
                                               xvoff, (t_ * 8 * H + dir * 4 * H + q * H) * 4, 0, 0);
  };
  if constexpr (XQ) {
    if (own) len_s[threadIdx.x] = a.len[min(oi, B - 1)];
    load_xq(0);
  }
  for (int s = 0; s < L; ++s) {
    stamp(a.stamps, 8 * s);
    const int t = dir == 0 ? s : L - 1 - s;
    if constexpr (XQ) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's gate fetch has landed
    const float* hin = a.hbuf + (long)((s & 1) * 2 + dir) * B * H;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)hin, (short)0, B * H * 4, 0x00020000);
#pragma unroll(X6 ? 1 : NBT)   // X6 unrolled over tiles spills (the compiler hoists the next tile's loads)
    for (int bt = 0; bt < NBT; ++bt) {
      if (bt * 32 >= B) break;   // uniform
      if constexpr (!X6) {
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        if (s > 0) {   // h_0 = 0: the first step has no recurrent term
          const int row = bt * 32 + b, bc = min(row, B - 1);
          const bool bval = row < B;
          float4 hf[NG];
#pragma unroll
          for (int g = 0; g < NG; ++g) hf[g] = selz(bval, ld_sc1(rs, (bc * H + k0 + 8 * g + 4 * hh) * 4));
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4e(hf[g], e), f4e(wf[g], e), acc, 0, 0, 0);
        }
        // C[b][n] partial over this wave's K slice: lane -> col n, reg r -> row (r&3) + 8(r>>2) + 4hh
        if (bt == 0) {
          asm volatile("" :: "v"(acc[0]));
          stamp(a.stamps, 8 * s + 1);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[w * 1024 + r * 64 + lane] = acc[r];
      } else {
        floatx4 big[2][2], sml[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) big[i][j] = sml[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (s > 0) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            float4 hx[2][2];   // [16-row tile i][half]: row l & 15 of tile i, k 8(l >> 4)..+7 of step ks
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int row = bt * 32 + 16 * i + (lane & 15), bc = min(row, B - 1);
              const int off = (bc * H + k0 + 32 * ks + 8 * (lane >> 4)) * 4;
              hx[i][0] = selz(row < B, ld_sc1(rs, off));
              hx[i][1] = selz(row < B, ld_sc1(rs, off + 16));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              bf16x8_t ha[3];
              split3_8(hx[i][0], hx[i][1], ha);
#pragma unroll
              for (int j = 0; j < 2; ++j)
                mfma_x6(ha, wx[j][ks], __builtin_bit_cast(bf16x8_t, wlo_s[((w * 2 + j) * KS + ks) * 64 + lane]),
                        big[i][j], sml[i][j]);
            }
          }
        }
        if (bt == 0) {
          asm volatile("" :: "v"(big[0][0][0]));
          stamp(a.stamps, 8 * s + 1);
        }
        // C[b][n] partial, natural [b][n] layout: tile (i, j), lane -> col 16j + (l & 15), reg r -> row
        // 16i + 4(l >> 4) + r
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              smem[w * 1024 + (16 * i + 4 * (lane >> 4) + r) * 32 + 16 * j + (lane & 15)] = big[i][j][r] + sml[i][j][r];
      }
      __syncthreads();
      if (bt == 0) stamp(a.stamps, 8 * s + 2);
      {   // sum the 16 wave partials: thread i owns element i of the 32x32 tile
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < PW; ++ww) sum += smem[ww * 1024 + threadIdx.x];
        smem[threadIdx.x] = sum;   // only this thread reads or writes index threadIdx.x of slot 0
      }
      __syncthreads();
      const int ob = bt * 32 + oi;
      if (own && ob < B) {
        const int rr = (oi & 3) + 4 * (oi >> 3), lh = ((oi >> 2) & 1) * 32;   // (32x32x2 C layout)
        const float* xp = a.xproj + (((long)ob * L + t) * 2 + dir) * 4 * H;
        float gq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          gq[q] = (XQ ? xq_s[q * 256 + threadIdx.x] : xp[q * H + uj]) + smem[X6 ? oi * 32 + q * PU + ou : rr * 64 + lh + q * PU + ou];
        float* outp = a.out + ((long)ob * L + t) * 2 * H + dir * H + uj;
        float* sa = a.save_act ? a.save_act + (((long)t * 2 + dir) * B + ob) * 4 * H : nullptr;
        float c = NBT > 1 ? cst[bt * 256 + threadIdx.x] : c1;
        float hp = NBT > 1 ? hst[bt * 256 + threadIdx.x] : h1;
        if (t < (XQ ? len_s[threadIdx.x] : a.len[ob])) {
          const float i = sigmoidf_(gq[0]), f = sigmoidf_(gq[1]), gg = tanhf(gq[2]), o = sigmoidf_(gq[3]);
          c = f * c + i * gg;
          hp = o * tanhf(c);
          *outp = hp;
          if (sa) { sa[uj] = i; sa[H + uj] = f; sa[2 * H + uj] = gg; sa[3 * H + uj] = o; }
        } else {   // packed sequence: state frozen (fwd) / still zero (bwd), output zero
          *outp = 0.f;
          if (sa) { sa[uj] = 0.f; sa[H + uj] = 0.f; sa[2 * H + uj] = 0.f; sa[3 * H + uj] = 0.f; }
        }
        if (a.save_c) a.save_c[(((long)t * 2 + dir) * B + ob) * H + uj] = c;
        if (s + 1 < L) st_sc1(a.hbuf + (long)(((s + 1) & 1) * 2 + dir) * B * H + (long)ob * H + uj, hp);
        if (NBT > 1) {
          cst[bt * 256 + threadIdx.x] = c;
          hst[bt * 256 + threadIdx.x] = hp;
        } else {
          c1 = c;
          h1 = hp;
        }
      }
      // the owners read slot 0 before the next tile's partials overwrite it
      if (bt + 1 < NBT && (bt + 1) * 32 < B) __syncthreads();
    }
    stamp(a.stamps, 8 * s + 3);
    if (XQ && s + 1 < L) load_xq(s + 1);   // in flight across the barrier
    if (s + 1 < L && !dir_barrier(a.sync, dir, (unsigned)(s + 1) * G, &a.sync[2], &smem[PW * 1024], a.force_tmo))
      break;
    stamp(a.stamps, 8 * s + 4);
  }
  const bool failed = launch_failed(&a.sync[2], a.err, 1u, &smem[PW * 1024]);
  const float qnan = __builtin_nanf("");
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int ob = bt * 32 + oi;
    if (own && ob < B) {
      const long si = ((long)dir * B + ob) * H + uj;
      if (failed) {   // poison everything this workgroup owns: no partial result passes for a good one
        for (int t = 0; t < L; ++t) a.out[((long)ob * L + t) * 2 * H + dir * H + uj] = qnan;
        if (a.h_n) a.h_n[si] = qnan;
        if (a.c_n) a.c_n[si] = qnan;
        continue;
      }
      if (a.h_n) a.h_n[si] = NBT > 1 ? hst[bt * 256 + threadIdx.x] : h1;
      if (a.c_n) a.c_n[si] = NBT > 1 ? cst[bt * 256 + threadIdx.x] : c1;
    }
  }
}

// ------------------------------------------------------------------------------------- BPTT
struct PBwd {
  const float* whh0;      // [4H][H]
  const float* whh1;
  const int* len;
  const float* save_act;  // [L][2][B][4H]
  const float* save_c;    // [L][2][B][H]
  const float* dout;      // [B][L][2H]
  const float* dh_n;      // [2][B][H] or NULL
  const float* dc_n;
  float* dgates;          // [B][L][2][4H]: output and the step-to-step hand-off (stored sc1)
  unsigned* sync;
  unsigned* err;
  int force_tmo;
  int B, L, H;
};

// rec[b][j] = sum_n dgates_prev[b][n] W_hh[n][j] with v_mfma_f32_16x16x4_f32: rows b (two 16-row
// tiles), cols j (the workgroup's 8 units, padded to 16), K = 4H split over the 16 waves (4H/16 each,
// NGB = 4H/256 K-groups of 16). W_hh[:, j-slice] lives in VGPRs in the K-permuted B-operand layout.
// T2 = false (B <= 16, the finetune rollout's B = 2): one row tile — half the hand-off loads and MFMAs, and
// the loads of eight K-groups (not four) in flight per round trip, so a step waits on half as many.
template <int NGB, bool T2 = true>
__global__ __launch_bounds__(1024) void bilstm_persist_bwd_kernel(PBwd a) {
  __shared__ __attribute__((aligned(16))) float smem[PW * 512 + 4];
  const int H = a.H, B = a.B, L = a.L, G = H / PU, G4 = 4 * H;
  const int dir = blockIdx.x / G, j0 = (blockIdx.x % G) * PU;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c16 = lane & 15, kq = lane >> 4;
  const int k0 = w * (16 * NGB);
  float4 wf[NGB];
  {
    const float* W = dir ? a.whh1 : a.whh0;
    const bool cv = c16 < PU;
    const int jj = j0 + (cv ? c16 : 0);
#pragma unroll
    for (int g = 0; g < NGB; ++g) {
      const int nb = k0 + 16 * g + 4 * kq;
      const float4 v = make_float4(W[(long)(nb + 0) * H + jj], W[(long)(nb + 1) * H + jj],
                                   W[(long)(nb + 2) * H + jj], W[(long)(nb + 3) * H + jj]);
      wf[g] = selz(cv, v);
    }
  }
  const bool owner = threadIdx.x < B * PU;
  const int ob = threadIdx.x / PU, oj = threadIdx.x % PU, j = j0 + oj;
  const int lenb = owner ? a.len[ob] : 0;
  float dh = 0.f, dc = 0.f;
  if (owner) {
    const long si = ((long)dir * B + ob) * H + j;
    if (a.dh_n) dh = a.dh_n[si];
    if (a.dc_n) dc = a.dc_n[si];
  }
  const int r16 = lane & 15;
  const int b0 = min(r16, B - 1), b1 = min(16 + r16, B - 1);
  const bool v0 = r16 < B, v1 = 16 + r16 < B;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dgates, (short)0, B * L * 2 * G4 * 4, 0x00020000);
  // the owner's saved activations / cell states / output gradient of the NEXT step are loaded before this
  // step's barrier (they do not depend on the recurrence): the cell phase then waits on no global load
  float pf_do = 0.f, pf_i = 0.f, pf_f = 0.f, pf_g = 0.f, pf_o = 0.f, pf_c = 0.f, pf_cp = 0.f;
  auto prefetch = [&](int s_) {
    if (!owner) return;
    const int t_ = dir == 0 ? (L - 1 - s_) : s_;
    if (t_ >= lenb) return;
    pf_do = a.dout[((long)ob * L + t_) * 2 * H + dir * H + j];
    const float* sa = a.save_act + (((long)t_ * 2 + dir) * B + ob) * G4;
    pf_i = sa[j];
    pf_f = sa[H + j];
    pf_g = sa[2 * H + j];
    pf_o = sa[3 * H + j];
    pf_c = a.save_c[(((long)t_ * 2 + dir) * B + ob) * H + j];
    const int tq = dir == 0 ? t_ - 1 : t_ + 1;   // previous step in forward order
    pf_cp = (tq >= 0 && tq < L) ? a.save_c[(((long)tq * 2 + dir) * B + ob) * H + j] : 0.f;
  };
  prefetch(0);
  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? (L - 1 - s) : s;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      const int tp = dir == 0 ? t + 1 : t - 1;   // the step processed just before (BPTT order)
      const int base0 = (((b0 * L + tp) * 2 + dir) * G4 + k0 + 4 * kq) * 4;
      const int base1 = (((b1 * L + tp) * 2 + dir) * G4 + k0 + 4 * kq) * 4;
      if constexpr (!T2) {
        constexpr int CH = NGB % 8 == 0 ? 8 : 4;
#pragma unroll
        for (int g0 = 0; g0 < NGB; g0 += CH) {
          float4 x0[CH];
#pragma unroll
          for (int g = 0; g < CH; ++g) x0[g] = selz(v0, ld_sc1(rs, base0 + 64 * (g0 + g)));
#pragma unroll
          for (int g = 0; g < CH; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4e(x0[g], e), f4e(wf[g0 + g], e), acc0, 0, 0, 0);
        }
      } else {
#pragma unroll
      for (int g0 = 0; g0 < NGB; g0 += 4) {
        float4 x0[4], x1[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          x0[g] = selz(v0, ld_sc1(rs, base0 + 64 * (g0 + g)));
          x1[g] = selz(v1, ld_sc1(rs, base1 + 64 * (g0 + g)));
        }
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4e(x0[g], e), f4e(wf[g0 + g], e), acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4e(x1[g], e), f4e(wf[g0 + g], e), acc1, 0, 0, 0);
          }
      }
      }
    }
    // 16x16 C map: col = lane & 15 (unit), row = 4 * (lane >> 4) + reg (batch within the tile)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      smem[w * 512 + r * 64 + lane] = acc0[r];
      smem[w * 512 + 256 + r * 64 + lane] = acc1[r];
    }
    __syncthreads();
    if (threadIdx.x < 512) {
      float sum = 0.f;
#pragma unroll
      for (int ww = 0; ww < PW; ++ww) sum += smem[ww * 512 + threadIdx.x];
      smem[PW * 512 - 512 + threadIdx.x] = sum;   // the last wave's slot: read by nobody else now
    }
    __syncthreads();
    if (owner) {
      const int tile = ob >> 4, br = ob & 15;
      const float rec = smem[PW * 512 - 512 + tile * 256 + (br & 3) * 64 + (br >> 2) * 16 + oj];
      float* dg = a.dgates + (((long)ob * L + t) * 2 + dir) * G4;
      if (t < lenb) {
        const float G = rec + pf_do + dh;
        const float i_ = pf_i, f_ = pf_f, g_ = pf_g, o_ = pf_o;
        const float ct = pf_c, cp = pf_cp;
        const float tc = tanhf(ct);
        const float dcv = dc + G * o_ * (1.f - tc * tc);
        st_sc1(dg + j, dcv * g_ * i_ * (1.f - i_));
        st_sc1(dg + H + j, dcv * cp * f_ * (1.f - f_));
        st_sc1(dg + 2 * H + j, dcv * i_ * (1.f - g_ * g_));
        st_sc1(dg + 3 * H + j, G * tc * o_ * (1.f - o_));
        dc = dcv * f_;
        dh = 0.f;
      } else {
        st_sc1(dg + j, 0.f);
        st_sc1(dg + H + j, 0.f);
        st_sc1(dg + 2 * H + j, 0.f);
        st_sc1(dg + 3 * H + j, 0.f);
        dh = rec + dh;
      }
    }
    if (s + 1 < L) prefetch(s + 1);   // in flight across the barrier
    if (s + 1 < L && !dir_barrier(a.sync, dir, (unsigned)(s + 1) * G, &a.sync[2], &smem[PW * 512], a.force_tmo))
      break;
  }
  if (launch_failed(&a.sync[2], a.err, 2u, &smem[PW * 512]) && owner) {
    const float qnan = __builtin_nanf("");
    for (int t = 0; t < L; ++t) {
      float* dg = a.dgates + (((long)ob * L + t) * 2 + dir) * G4;
#pragma unroll
      for (int q = 0; q < 4; ++q) dg[q * H + j] = qnan;
    }
  }
}

}  // namespace

// Library error word (device pointer, dasa_set_error_word) and the forced-timeout test hook.
static unsigned* g_err_word = nullptr;
static int g_force_tmo = 0;
static unsigned long long* g_stamps = nullptr;
#ifdef DASA_DEBUG
// debug build: every translation unit registers the setter of its DASA_DCHECK error-word pointer
static void (*(&dbg_setters())[16])(unsigned*) {
  static void (*s[16])(unsigned*) = {};
  return s;
}
void dasa_dbg_register(void (*setter)(unsigned*)) {
  for (auto& f : dbg_setters())
    if (!f || f == setter) { f = setter; return; }
}
#endif
extern "C" int dasa_set_error_word(uint32_t* dev_word) {
  g_err_word = reinterpret_cast<unsigned*>(dev_word);
#ifdef DASA_DEBUG
  for (auto f : dbg_setters())
    if (f) f(g_err_word);
#endif
  return 0;
}
// Diagnostic hook: when buf != NULL, workgroup 0 of every persistent forward launch writes s_memtime
// clocks per timestep s into buf[8s + i]: i = 0 step start, 1 after the h loads + recurrent MFMAs, 2 after
// the wave-partial exchange, 3 after the cell update / state stores, 4 after the direction barrier.
extern "C" int dasa_persist_stamps(uint64_t* buf) {
  g_stamps = reinterpret_cast<unsigned long long*>(buf);
  return 0;
}

extern "C" int dasa_persist_force_timeout(int32_t on) {
  g_force_tmo = on ? 1 : 0;
  return 0;
}
// shared with the other kernels that wait on a bounded inter-workgroup barrier (attn.hip)
unsigned* dasa_err_word_host() { return g_err_word; }
int dasa_force_timeout_host() { return g_force_tmo; }

// Residency check done once per kernel: the grid (one 1024-thread workgroup per CU) must fit the
// device in one wave of workgroups. Launched as plain kernels: a cooperative launch adds only this
// same check (plus ~15 us of host time per launch) and its teardown crashes rocprofv3 on exit.
template <typename K>
bool resident(K kernel, int grid) {
  static int cached = -1;   // per kernel instantiation
  if (cached < 0) {
    int dev = 0, cus = 0, per_cu = 0;
    cached = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 1024, 0) == hipSuccess)
      cached = (per_cu >= 1 && (long)per_cu * cus >= grid) ? 1 : 0;
    (void)hipGetLastError();
  }
  return cached == 1;
}

template <typename K, typename A>
int launch_persistent(K kernel, int grid, const A& a, hipStream_t st) {
  if (!resident(kernel, grid)) return (int)hipErrorCooperativeLaunchTooLarge;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(1024), 0, st, a);
  return (int)hipGetLastError();
}

bool bilstm_persist_ok(int B, int H) {
  return B >= 1 && B <= 32 && H % 256 == 0 && H >= 256 && H <= 1024;
}

// Forward: up to 6 batch tiles of 32 rows at the DicEncoder's H = 1024 (the teacher rollout encodes 4-8
// steps x B = 20 sequences per launch; more tiles would spill); other H keep one tile.
bool bilstm_persist_fwd_ok(int B, int H) {
  return bilstm_persist_ok(B, H) || (H == 1024 && B >= 1 && B <= 192);
}

// X6 recurrence switch (dasa_bilstm_fwd_x6; env DASA_LSTM_X6=0 or DASA_GEMM_EMU=0 start it off)
static int g_fwd_x6 = -1;
static bool fwd_x6() {
  if (g_fwd_x6 < 0) {
    const char* e = getenv("DASA_LSTM_X6");
    const char* g = getenv("DASA_GEMM_EMU");
    g_fwd_x6 = !(e && e[0] == '0') && !(g && g[0] == '0');
  }
  return g_fwd_x6 != 0;
}
bool bilstm_fwd_x6_on() { return fwd_x6(); }
extern "C" int dasa_bilstm_fwd_x6(int32_t on) {
  const int prev = fwd_x6() ? 1 : 0;
  if (on >= 0) g_fwd_x6 = on ? 1 : 0;
  return prev;
}

int bilstm_persist_fwd(const float* xproj, const float* whh_fwd, const float* whh_bwd, const int32_t* lengths,
                       float* out, float* h_n, float* c_n, float* save_act, float* save_c, int B, int L, int H,
                       float* hbuf, unsigned* sync, hipStream_t st) {
  PFwd a{xproj, whh_fwd, whh_bwd, lengths, out, save_act, save_c, h_n, c_n, hbuf, sync, g_err_word, g_force_tmo,
         B, L, H, g_stamps};
  const int grid = 2 * H / PU;
  // the single-tile gate prefetch addresses xproj with 32-bit buffer offsets (the caller takes the step kernels)
  if ((long)B * L * 8 * H * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;
  // X6 at one or two 32-row tiles only (profiles/r03/lstm_x6_probe.txt, L = 80: B = 20 0.69-0.74 vs 0.76
  // ms, B = 40 1.03-1.05 vs 1.16-1.20; B = 96 / 160 3-5 % slower, the tile loop then spills): the step
  // is bound by the h-state hand-off latency and the direction barrier more than by the MFMA cycles
  if (H == 1024 && B <= 64 && fwd_x6()) {
    if (B > 32) return launch_persistent(bilstm_persist_fwd_kernel<8, 2, true>, grid, a, st);
    return launch_persistent(bilstm_persist_fwd_kernel<8, 1, true>, grid, a, st);
  }
  if (B > 32) {
    if (H != 1024 || B > 192) return (int)hipErrorInvalidValue;
    switch ((B + 31) / 32) {
      case 2: return launch_persistent(bilstm_persist_fwd_kernel<8, 2>, grid, a, st);
      case 3: return launch_persistent(bilstm_persist_fwd_kernel<8, 3>, grid, a, st);
      case 4: return launch_persistent(bilstm_persist_fwd_kernel<8, 4>, grid, a, st);
      case 5: return launch_persistent(bilstm_persist_fwd_kernel<8, 5>, grid, a, st);
      default: return launch_persistent(bilstm_persist_fwd_kernel<8, 6>, grid, a, st);
    }
  }
  switch (H / 128) {
    case 2: return launch_persistent(bilstm_persist_fwd_kernel<2, 1>, grid, a, st);
    case 4: return launch_persistent(bilstm_persist_fwd_kernel<4, 1>, grid, a, st);
    case 6: return launch_persistent(bilstm_persist_fwd_kernel<6, 1>, grid, a, st);
    case 8: return launch_persistent(bilstm_persist_fwd_kernel<8, 1>, grid, a, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// the persistent BPTT's one-row-tile form at B <= 16 (dasa_bilstm_bptt_one_tile; env DASA_BPTT_ONE_TILE=0
// starts at 0: the two-tile form at every B)
static int g_bwd_one_tile = -1;
static bool bwd_one_tile() {
  if (g_bwd_one_tile < 0) {
    const char* e = getenv("DASA_BPTT_ONE_TILE");
    g_bwd_one_tile = !(e && e[0] == '0');
  }
  return g_bwd_one_tile != 0;
}
extern "C" int dasa_bilstm_bptt_one_tile(int32_t on) {
  const int prev = bwd_one_tile() ? 1 : 0;
  if (on >= 0) g_bwd_one_tile = on ? 1 : 0;
  return prev;
}

int bilstm_persist_bwd(const float* whh_fwd, const float* whh_bwd, const int32_t* lengths, const float* save_act,
                       const float* save_c, const float* dout, const float* dh_n, const float* dc_n, float* dgates,
                       int B, int L, int H, unsigned* sync, hipStream_t st) {
  PBwd a{whh_fwd, whh_bwd, lengths, save_act, save_c, dout, dh_n, dc_n, dgates, sync, g_err_word, g_force_tmo,
         B, L, H};
  const int grid = 2 * H / PU;
  if (B <= 16 && H == 1024 && bwd_one_tile()) return launch_persistent(bilstm_persist_bwd_kernel<16, false>, grid, a, st);
  switch (H / 64) {   // NGB = 4H / 256
    case 4: return launch_persistent(bilstm_persist_bwd_kernel<4>, grid, a, st);
    case 8: return launch_persistent(bilstm_persist_bwd_kernel<8>, grid, a, st);
    case 12: return launch_persistent(bilstm_persist_bwd_kernel<12>, grid, a, st);
    case 16: return launch_persistent(bilstm_persist_bwd_kernel<16>, grid, a, st);
    default: return (int)hipErrorInvalidValue;
  }
}
