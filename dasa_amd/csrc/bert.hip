// BERT / LXRT building blocks for gfx950 (vilmodel.py:147-325, 443-506, 1014-1095):
// residual+dropout+LayerNorm, embeddings gather+LN, masked multi-head attention core, plus the
// token reversal of DicEncoder (r2rmodel.py:2326-2330), the mu/sigma AdaIN (model.py:1822-1840)
// and a counter-RNG dropout.
//
// LayerNorm: one wave per row, the row held in registers (VPL float4 per lane), two-pass mean/var
// with wave-shuffle reductions — HBM-bound, one read of x/res, one write of y.
// MHA: one workgroup per (batch, head); K and V of that head are staged in LDS (Lk <= 128, dh = 64,
// padded rows so the per-lane key-row reads are conflict-free); each wave owns query rows: lane j
// scores key j (and j+64), wave-shuffle softmax, then lane d accumulates sum_j p_j V[j][d].
#include "common.h"
#include "../../include/dasa_hip.h"

__attribute__((visibility("hidden"))) bool dasa_dropout_vec(const float* x, long ldx, float* y, long ldy, int rows, int cols, float p, uint64_t seed,
                      hipStream_t st);   // elem.hip

namespace {

inline int cdivi(long a, long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------ LayerNorm
template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, float* __restrict__ xsum,
                                                     int M, int N, float eps, float p, uint64_t seed,
                                                     const uint64_t* seed_src, unsigned short* __restrict__ ybf) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  if (p > 0.f) seed = eff_seed(seed, seed_src);
  const int N4 = N >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x + (long)row * N);
  const float4* r4 = res ? reinterpret_cast<const float4*>(res + (long)row * N) : nullptr;
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
  // every load of the row first (clamped quads, unconditional; gamma / beta too), so one memory
  // round trip per wave instead of one per operand
  float4 v[VPL], rv[VPL], gv[VPL], bv[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = min(lane + 64 * i, N4 - 1);
    v[i] = x4[c];
    gv[i] = g4[c];
    bv[i] = b4[c];
  }
  if (r4) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) rv[i] = r4[min(lane + 64 * i, N4 - 1)];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < N4) {
      float4 a = v[i];
      if (p > 0.f) {
        const uint64_t base = (uint64_t)row * N + 4 * c;
        a.x *= dasa_dropout_scale(p, seed, base + 0);
        a.y *= dasa_dropout_scale(p, seed, base + 1);
        a.z *= dasa_dropout_scale(p, seed, base + 2);
        a.w *= dasa_dropout_scale(p, seed, base + 3);
      }
      if (r4) {
        a.x += rv[i].x; a.y += rv[i].y; a.z += rv[i].z; a.w += rv[i].w;
      }
      v[i] = a;
      s += (a.x + a.y) + (a.z + a.w);
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < N4) {
      const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
      q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  }
  const float var = wave_sum(q) / N;
  const float rstd = rsqrtf(var + eps);
  float4* y4 = reinterpret_cast<float4*>(y + (long)row * N);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < N4) {
      if (xsum) reinterpret_cast<float4*>(xsum + (long)row * N)[c] = v[i];
      const float4 g = gv[i], bb = bv[i];
      float4 o;
      o.x = (v[i].x - mean) * rstd * g.x + bb.x;
      o.y = (v[i].y - mean) * rstd * g.y + bb.y;
      o.z = (v[i].z - mean) * rstd * g.z + bb.z;
      o.w = (v[i].w - mean) * rstd * g.w + bb.w;
      y4[c] = o;
      if (ybf) {   // the bf16 twin (RNE), bitwise what a bf16 GEMM rounding y on load would use
        const uint2 u = {(unsigned)__builtin_bit_cast(unsigned short, (__bf16)o.x) |
                             ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)o.y) << 16),
                         (unsigned)__builtin_bit_cast(unsigned short, (__bf16)o.z) |
                             ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)o.w) << 16)};
        reinterpret_cast<uint2*>(ybf + (long)row * N)[c] = u;
      }
    }
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)); dgamma += sum_rows dy*xhat; dbeta += sum_rows dy.
// One launch, two kinds of 1024-thread block: the first ceil(M/16) blocks take one row per wave (dx); the last
// ceil(N/256) take 64 float4 columns each and reduce dgamma / dbeta over ALL rows (16 waves stride the rows, then a
// fixed-order LDS reduction), so the parameter gradients are deterministic and need no atomics (the previous
// per-element global atomics serialised on the same N addresses from every row block: 45 us per launch at the
// finetune shapes).
constexpr int kLnBwdWaves = 16;
template <int VPL>
__global__ __launch_bounds__(1024) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ xsum,
                                                      const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta, int M,
                                                      int N) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rowBlocks = (M + kLnBwdWaves - 1) / kLnBwdWaves;
  const int N4 = N >> 2;
  if ((int)blockIdx.x >= rowBlocks) {
    __shared__ float4 red[2][kLnBwdWaves][64];
    const int c = ((int)blockIdx.x - rowBlocks) * 64 + lane;
    const bool cok = c < N4;
    const int cc = cok ? c : 0;
    float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sb = sg;
    for (int r0 = wave; r0 < M; r0 += 4 * kLnBwdWaves) {
      float4 xs[4], d[4];
      float mu[4], rs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {        // all loads first (clamped rows), then the arithmetic
        const int r = r0 + u * kLnBwdWaves, rr = r < M ? r : M - 1;
        xs[u] = reinterpret_cast<const float4*>(xsum + (long)rr * N)[cc];
        d[u] = reinterpret_cast<const float4*>(dy + (long)rr * N)[cc];
        mu[u] = mean_in[rr];
        rs[u] = r < M ? rstd_in[rr] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (r0 + u * kLnBwdWaves >= M) break;
        sg.x = fmaf(d[u].x, (xs[u].x - mu[u]) * rs[u], sg.x);
        sg.y = fmaf(d[u].y, (xs[u].y - mu[u]) * rs[u], sg.y);
        sg.z = fmaf(d[u].z, (xs[u].z - mu[u]) * rs[u], sg.z);
        sg.w = fmaf(d[u].w, (xs[u].w - mu[u]) * rs[u], sg.w);
        sb.x += d[u].x; sb.y += d[u].y; sb.z += d[u].z; sb.w += d[u].w;
      }
    }
    red[0][wave][lane] = sg;
    red[1][wave][lane] = sb;
    __syncthreads();
    if (wave < 2 && cok) {
      float* dst = wave == 0 ? dgamma : dbeta;
      if (dst) {
        float4 acc = red[wave][0][lane];
        for (int w = 1; w < kLnBwdWaves; ++w) {
          const float4 v = red[wave][w][lane];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        float4* o = reinterpret_cast<float4*>(dst) + c;
        const float4 prev = *o;
        *o = make_float4(prev.x + acc.x, prev.y + acc.y, prev.z + acc.z, prev.w + acc.w);
      }
    }
    return;
  }
  const int row = blockIdx.x * kLnBwdWaves + wave;
  if (row >= M) return;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float4 xh[VPL], gd[VPL];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < N4) {
      const float4 xs = reinterpret_cast<const float4*>(xsum + (long)row * N)[c];
      const float4 d = reinterpret_cast<const float4*>(dy + (long)row * N)[c];
      const float4 g = reinterpret_cast<const float4*>(gamma)[c];
      xh[i] = make_float4((xs.x - mean) * rstd, (xs.y - mean) * rstd, (xs.z - mean) * rstd, (xs.w - mean) * rstd);
      gd[i] = make_float4(d.x * g.x, d.y * g.y, d.z * g.z, d.w * g.w);
      s1 += gd[i].x + gd[i].y + gd[i].z + gd[i].w;
      s2 += gd[i].x * xh[i].x + gd[i].y * xh[i].y + gd[i].z * xh[i].z + gd[i].w * xh[i].w;
    }
  }
  const float m1 = wave_sum(s1) / N, m2 = wave_sum(s2) / N;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < N4) {
      float4 o;
      o.x = rstd * (gd[i].x - m1 - xh[i].x * m2);
      o.y = rstd * (gd[i].y - m1 - xh[i].y * m2);
      o.z = rstd * (gd[i].z - m1 - xh[i].z * m2);
      o.w = rstd * (gd[i].w - m1 - xh[i].w * m2);
      reinterpret_cast<float4*>(dx + (long)row * N)[c] = o;
    }
  }
}

// ------------------------------------------------------------------ embeddings
template <int VPL>
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, const float* __restrict__ word,
                                                    const float* __restrict__ pos, const float* __restrict__ type0,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float* __restrict__ out, int B, int L, int H, float eps, float p,
                                                    uint64_t seed, const uint64_t* seed_src) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * L) return;
  if (p > 0.f) seed = eff_seed(seed, seed_src);
  const int t = row % L;
  const long id = ids[row];
  const int H4 = H >> 2;
  const float4* w4 = reinterpret_cast<const float4*>(word + id * H);
  const float4* p4 = reinterpret_cast<const float4*>(pos + (long)t * H);
  const float4* t4 = reinterpret_cast<const float4*>(type0);
  float4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < H4) {
      const float4 a = w4[c], b = p4[c], d = t4[c];
      // (word + pos) + type, the reference's summation order (vilmodel.py:173)
      v[i] = make_float4((a.x + b.x) + d.x, (a.y + b.y) + d.y, (a.z + b.z) + d.z, (a.w + b.w) + d.w);
      s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float mean = wave_sum(s) / H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < H4) {
      const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
      q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / H + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < H4) {
      const float4 g = reinterpret_cast<const float4*>(gamma)[c], bb = reinterpret_cast<const float4*>(beta)[c];
      float4 o;
      o.x = (v[i].x - mean) * rstd * g.x + bb.x;
      o.y = (v[i].y - mean) * rstd * g.y + bb.y;
      o.z = (v[i].z - mean) * rstd * g.z + bb.z;
      o.w = (v[i].w - mean) * rstd * g.w + bb.w;
      if (p > 0.f) {
        const uint64_t base = (uint64_t)row * H + 4 * c;
        o.x *= dasa_dropout_scale(p, seed, base + 0);
        o.y *= dasa_dropout_scale(p, seed, base + 1);
        o.z *= dasa_dropout_scale(p, seed, base + 2);
        o.w *= dasa_dropout_scale(p, seed, base + 3);
      }
      reinterpret_cast<float4*>(out + (long)row * H)[c] = o;
    }
  }
}

// ------------------------------------------------------------------ multi-head attention
constexpr int kDh = 64;
constexpr int kMaxLk = 128;

struct MhaArgs {
  const float* Q; long ldq; const float* K; long ldk; const float* V; long ldv;
  const float* mask; float* out; long ldo; float* probs;
  int B, heads, Lq, Lk; float scale; float p; uint64_t seed;
  const uint64_t* seed_src;   // device seed source of a graph-captured launch (eff_seed), or null: the
                              // backward of a captured training step re-keys with the same source
};

// Forward on matrix cores (v_mfma_f32_32x32x2_f32): one workgroup per (batch, head), one wave per
// 32-query tile. The head's K and V rows ([Lk][64] each, <= 48 KB) are staged in LDS once by the whole
// workgroup with float4 loads (rows padded to 68 floats: conflict-free ds_read_b128 fragments) and
// shared by the query-tile waves; the per-MFMA operand reads of K (S^T) and V (P V) are then LDS reads
// instead of dependent global loads. Each wave computes S^T = K Q^T (keys on the accumulator rows,
// queries on the lanes), so the softmax over keys is an in-lane reduction plus one cross-half
// shuffle, and the probability tile as it sits in the accumulator is directly the A operand of
// O = P V (register r of lane half hh holds key (r&3) + 8(r>>2) + 4hh; the V operand is read for
// exactly that key). NKT = ceil(Lk / 32) key tiles (Lk <= 128).
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

constexpr int kKvLd = kDh + 4;   // LDS row stride of the staged K / V (floats)

template <int NKT>
__global__ __launch_bounds__(256) void mha_fwd_kernel(MhaArgs a, int nqt) {
  __shared__ __attribute__((aligned(16))) float kv[2 * NKT * 32 * kKvLd + NKT * 32];
  float* Ks = kv;
  float* Vs = kv + NKT * 32 * kKvLd;
  float* Ms = kv + 2 * NKT * 32 * kKvLd;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.x;
  const int h = bh % a.heads, b = bh / a.heads;
  const int Lq = a.Lq, Lk = a.Lk;
  const uint64_t seed = a.p > 0.f ? eff_seed(a.seed, a.seed_src) : 0;
  const int qt = w, q0 = qt * 32;
  const int j = lane & 31, hh = lane >> 5;
  // Every global load of the workgroup is issued before the first is waited for (one HBM round trip
  // per workgroup instead of one per staging pass): this wave's Q fragment, the K / V rows (clamped,
  // zeroed past Lk when written to LDS) and the key mask.
  // B operand of S^T: Q^T, lane (query j, half hh) holds Q[q0 + j][8g + 4hh .. +3] (K-permuted)
  const float* qp = a.Q + ((long)b * Lq + min(q0 + j, Lq - 1)) * a.ldq + h * kDh + 4 * hh;
  float4 qf[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) qf[g] = *reinterpret_cast<const float4*>(qp + 8 * g);
  constexpr int NF = NKT * 32 * (kDh / 4) / 256;   // float4 of K (and of V) per thread (blockDim = 256)
  float4 kx[NF], vx[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int idx = threadIdx.x + 256 * i, row = min(idx / (kDh / 4), Lk - 1), c4 = idx % (kDh / 4);
    kx[i] = reinterpret_cast<const float4*>(a.K + ((long)b * Lk + row) * a.ldk + h * kDh)[c4];
    vx[i] = reinterpret_cast<const float4*>(a.V + ((long)b * Lk + row) * a.ldv + h * kDh)[c4];
  }
  const int mk = min((int)threadIdx.x, Lk - 1);
  const float mv = a.mask ? a.mask[(long)b * Lk + mk] : 0.f;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx / (kDh / 4), c4 = idx % (kDh / 4);
    const float k = row < Lk ? 1.f : 0.f;   // component-wise (a whole-float4 select goes through scratch)
    *reinterpret_cast<float4*>(Ks + row * kKvLd + 4 * c4) =
        make_float4(k * kx[i].x, k * kx[i].y, k * kx[i].z, k * kx[i].w);
    *reinterpret_cast<float4*>(Vs + row * kKvLd + 4 * c4) =
        make_float4(k * vx[i].x, k * vx[i].y, k * vx[i].z, k * vx[i].w);
  }
  if (threadIdx.x < NKT * 32) Ms[threadIdx.x] = (int)threadIdx.x < Lk ? mv : -INFINITY;
  __syncthreads();
  if (qt >= nqt) return;   // (no barrier below)
  floatx16 st[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const float* kp = Ks + (kt * 32 + j) * kKvLd + 4 * hh;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 kf = *reinterpret_cast<const float4*>(kp + 8 * g);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.x, qf[g].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.y, qf[g].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.z, qf[g].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.w, qf[g].w, acc, 0, 0, 0);
    }
    st[kt] = acc;
  }
  // scale + additive key mask; keys past Lk -> -inf
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = st[kt][r] * a.scale + Ms[kt * 32 + acc_row(r, hh)];
      st[kt][r] = v;
      m = fmaxf(m, v);
    }
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __expf(st[kt][r] - m);
      st[kt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
  const int q = q0 + j;
  const long prow = ((long)bh * Lq + q) * (long)Lk;   // probs / dropout index base of this query row
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + acc_row(r, hh);
      float p = st[kt][r] * inv;
      if (a.probs && q < Lq && key < Lk) a.probs[prow + key] = p;
      if (a.p > 0.f) p *= dasa_dropout_scale(a.p, seed, (uint64_t)(prow + key));
      st[kt][r] = p;
    }
  // O = P V: A operand = the probability accumulator (rows = keys), B operand = V[key][d0 + lane]
  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* vr = Vs + (kt * 32 + acc_row(r, hh)) * kKvLd + j;
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(st[kt][r], vr[0], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(st[kt][r], vr[32], o1, 0, 0, 0);
    }
  // O tile: col = d (lane), row = query q0 + acc_row(r, hh)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qq = q0 + acc_row(r, hh);
    if (qq < Lq) {
      float* op = a.out + ((long)b * Lq + qq) * a.ldo + h * kDh + j;
      op[0] = o0[r];
      op[32] = o1[r];
    }
  }
}

// Backward (no attention dropout): one workgroup per (b, h); dQ, dK, dV written (not accumulated).
__global__ __launch_bounds__(256) void mha_bwd_kernel(MhaArgs a, const float* dO, long lddo, float* dQ, float* dK,
                                                      float* dV) {
  __shared__ float Ks[kMaxLk][kDh + 1];
  __shared__ float Vs[kMaxLk][kDh + 1];
  __shared__ float dKs[kMaxLk][kDh + 1];
  __shared__ float dVs[kMaxLk][kDh + 1];
  __shared__ float qs[4][kDh];
  __shared__ float dos[4][kDh];
  __shared__ float dss[4][kMaxLk];
  const int bh = blockIdx.x, b = bh / a.heads, h = bh % a.heads;
  const int Lk = a.Lk;
  for (int idx = threadIdx.x; idx < Lk * kDh; idx += 256) {
    const int j = idx / kDh, d = idx % kDh;
    Ks[j][d] = a.K[((long)b * Lk + j) * a.ldk + h * kDh + d];
    Vs[j][d] = a.V[((long)b * Lk + j) * a.ldv + h * kDh + d];
    dKs[j][d] = 0.f;
    dVs[j][d] = 0.f;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // waves take query rows round-robin; dK/dV accumulated per wave into LDS with atomics
  for (int i = w; i < a.Lq; i += 4) {
    qs[w][lane] = a.Q[((long)b * a.Lq + i) * a.ldq + h * kDh + lane];
    dos[w][lane] = dO[((long)b * a.Lq + i) * lddo + h * kDh + lane];
    __builtin_amdgcn_wave_barrier();
    const long prow = (((long)b * a.heads + h) * a.Lq + i) * Lk;
    float p0 = lane < Lk ? a.probs[prow + lane] : 0.f;
    float p1 = lane + 64 < Lk ? a.probs[prow + lane + 64] : 0.f;
    // attention-probs dropout (train mode): the same counter-RNG mask as the forward
    const uint64_t sd = a.p > 0.f ? eff_seed(a.seed, a.seed_src) : 0;
    const float k0 = a.p > 0.f ? dasa_dropout_scale(a.p, sd, (uint64_t)prow + lane) : 1.f;
    const float k1 = a.p > 0.f ? dasa_dropout_scale(a.p, sd, (uint64_t)prow + lane + 64) : 1.f;
    float dp0 = 0.f, dp1 = 0.f;
    if (lane < Lk)
      for (int d = 0; d < kDh; ++d) dp0 = fmaf(dos[w][d], Vs[lane][d], dp0);
    if (lane + 64 < Lk)
      for (int d = 0; d < kDh; ++d) dp1 = fmaf(dos[w][d], Vs[lane + 64][d], dp1);
    dp0 *= k0;
    dp1 *= k1;
    const float dot = wave_sum(p0 * dp0 + p1 * dp1);
    const float ds0 = p0 * (dp0 - dot) * a.scale, ds1 = p1 * (dp1 - dot) * a.scale;
    dss[w][lane] = ds0;
    dss[w][lane + 64] = ds1;
    __builtin_amdgcn_wave_barrier();
    float dq = 0.f;
    for (int j = 0; j < Lk; ++j) dq = fmaf(dss[w][j], Ks[j][lane], dq);
    dQ[((long)b * a.Lq + i) * a.ldq + h * kDh + lane] = dq;
    // dK[j][d] += ds_j * q[d]; dV[j][d] += p_j * dO[d]  (lane = d)
    const float pd0 = p0 * k0, pd1 = p1 * k1;   // dropped probs feed dV
    for (int j = 0; j < Lk; ++j) {
      const float pj = j < 64 ? __shfl(pd0, j, 64) : __shfl(pd1, j - 64, 64);
      atomicAdd(&dKs[j][lane], dss[w][j] * qs[w][lane]);
      atomicAdd(&dVs[j][lane], pj * dos[w][lane]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < Lk * kDh; idx += 256) {
    const int j = idx / kDh, d = idx % kDh;
    dK[((long)b * Lk + j) * a.ldk + h * kDh + d] = dKs[j][d];
    dV[((long)b * Lk + j) * a.ldv + h * kDh + d] = dVs[j][d];
  }
}

// Backward for Lq, Lk <= 80 (the language / LXRT shapes): one workgroup per (b, h), every operand staged
// in LDS once (K-major copies where a product needs them: dO^T, V^T, dS^T), and the four products
//   dP = dO V^T (x the dropout scale),  dV = P_dropped^T dO,  dQ = dS K,  dK = dS^T Q,
//   dS = P (dP - rowsum(P dP)) * scale
// as register-blocked 4x4 outer products over LDS rows (two float4 reads per 16 FMAs). No atomics: the
// previous form accumulated dK / dV with per-element LDS atomics row by row (0.64 ms per launch at the
// finetune shapes, B = 2; bench.py cfg4 leg).
// `parts` workgroups per (b, h) (r05; B x heads far below the CU count, e.g. 24 at the finetune's B = 2):
// every part computes the whole dS (dP, its row sums, dS — the row sums need whole rows), then only its
// share of the 4-row blocks of dV / dK (key rows) and dQ (query rows). Each output element is still
// computed by one workgroup with the same loop order: bitwise equal to parts = 1.
constexpr int kBwdMaxL = 80;
constexpr int kBwdLd = kBwdMaxL + 4;   // row stride of [.][Lq] / [.][Lk] tiles
constexpr int kBwdLdD = kDh + 4;       // row stride of [.][64] tiles
constexpr int kBwdBufA = (kDh * kBwdLd > kBwdMaxL * kBwdLdD) ? kDh * kBwdLd : kBwdMaxL * kBwdLdD;
constexpr int kBwdBufL = kBwdMaxL * kBwdLd;
// 8 waves: the LDS footprint (~146 KB) allows one workgroup per CU, so the MFMA tiles and elementwise phases
// are spread over 8 waves rather than 4 (r06)
constexpr int kBwdThreads = 512, kBwdWaves = kBwdThreads / 64;

// C[m][n] = sum_k A[k][m] B[k][n] over 4x4 register blocks (A, B row-major in LDS, m / n multiples of 4),
// m-blocks mb0 .. mb0 + MB - 1.
template <typename Epi>
__device__ __forceinline__ void lds_tn_blocks(const float* A, int lda, const float* B, int ldb, int K, int mb0, int MB,
                                              int NB, Epi epi) {
  for (int blk = threadIdx.x; blk < MB * NB; blk += blockDim.x) {
    const int m0 = (mb0 + blk / NB) * 4, n0 = (blk % NB) * 4;
    float acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float4 av = *reinterpret_cast<const float4*>(A + k * lda + m0);
      const float4 bv = *reinterpret_cast<const float4*>(B + k * ldb + n0);
      const float am[4] = {av.x, av.y, av.z, av.w}, bn[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(am[r], bn[c], acc[r][c]);
    }
    epi(m0, n0, acc);
  }
}

// Diagnosis (dasa_mha_bwd_stamps): workgroup 0's clock (s_memtime, shader cycles) at
// each phase boundary; one record of kBwdStamps per launch, overwritten by the next.
constexpr int kBwdStamps = 9;

// C[m][n] = sum_{k < K} A[k][m] B[k][n] (A, B row-major in LDS) on v_mfma_f32_32x32x2_f32, for rows m in
// [mlo, mhi) and the 64 columns n: 32 x 32 tiles dealt round-robin to the workgroup's waves; lane (col jl,
// half hh) supplies k = kk + 4 hh + e to MFMA e of each 8-deep k step (A column / B column reads per k row),
// k >= K masked to zero. epi(m, n, v) per output of the tile (m may exceed mhi: the caller checks).
template <typename Epi>
__device__ __forceinline__ void lds_tn_mfma(const float* A, int lda, const float* B, int ldb, int K, int mlo, int mhi,
                                            Epi epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, jl = lane & 31, hh = lane >> 5;
  const int ntm = (mhi - mlo + 31) / 32, ntiles = ntm * (kDh / 32);
  for (int tile = w; tile < ntiles; tile += kBwdWaves) {
    const int m0 = mlo + (tile >> 1) * 32, n0 = (tile & 1) * 32;
    const float* ap = A + min(m0 + jl, lda - 1);
    const float* bp = B + n0 + jl;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int kk = 0; kk < K; kk += 8) {
      float av[4], bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = kk + 4 * hh + e, kc = min(k, K - 1);
        const float z = k < K ? 1.f : 0.f;
        av[e] = z * ap[kc * lda];
        bv[e] = bp[kc * ldb];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bv[e], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) epi(m0 + acc_row(r, hh), n0 + jl, acc[r]);
  }
}


template <bool STAMP>
__device__ __forceinline__ void bwd_stamp(unsigned long long* buf, int i) {
  if (!STAMP) return;   // the product instantiation carries no stamp code (no scheduling barriers)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf[i] = t;
  }
}

template <bool STAMP>
__global__ __launch_bounds__(kBwdThreads) void mha_bwd_lds_kernel(MhaArgs a, const float* dO, long lddo, float* dQ, float* dK,
                                                          float* dV, int parts, unsigned long long* stamps) {
  bwd_stamp<STAMP>(stamps, 0);
  __shared__ float bufA[kBwdBufA];   // Q [Lq][64] (after dS)
  __shared__ float bufB[kBwdBufA];   // V [Lk][64]; then K [Lk][64]
  __shared__ float sP[kBwdBufL];     // P [Lq][Lk]; then P_dropped
  __shared__ float sdO[kBwdMaxL * kBwdLdD];   // dO [Lq][64]
  __shared__ float sdS[kBwdBufL];    // dP, then dS [Lq][Lk]
  __shared__ float sdST[kBwdBufL];   // dS^T [Lk][Lq]
  __shared__ float rowdot[kBwdMaxL];
  const uint64_t sdk = a.p > 0.f ? eff_seed(a.seed, a.seed_src) : 0;   // dropout seed of this launch
  const int bh = blockIdx.x / parts, part = blockIdx.x % parts, b = bh / a.heads, h = bh % a.heads, t = threadIdx.x;
  const int Lq = a.Lq, Lk = a.Lk, Lq4 = (Lq + 3) & ~3, Lk4 = (Lk + 3) & ~3;
  const int kper = (Lk4 / 4 + parts - 1) / parts, kb0 = part * kper, kbn = max(0, min(kper, Lk4 / 4 - kb0));
  const int qper = (Lq4 / 4 + parts - 1) / parts, qb0 = part * qper, qbn = max(0, min(qper, Lq4 / 4 - qb0));
  const long pbase = ((long)b * a.heads + h) * Lq * Lk;
  const bool drop = a.p > 0.f;
  // staging: every global load of dO, V and P issued before the first LDS store (fixed trip counts, fully
  // unrolled: 33 loads in flight per thread, one memory round trip instead of one per loop iteration)
  constexpr int NR = kBwdMaxL * kDh / kBwdThreads, NP = (kBwdMaxL * kBwdMaxL + kBwdThreads - 1) / kBwdThreads;
  static_assert(NR * kBwdThreads == kBwdMaxL * kDh, "staging trip counts");
  {
    float vo[NR], vv[NR], vp[NP];
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / kDh, d = idx % kDh;
      vo[it] = i < Lq ? dO[((long)b * Lq + i) * lddo + h * kDh + d] : 0.f;
      vv[it] = i < Lk ? a.V[((long)b * Lk + i) * a.ldv + h * kDh + d] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / Lk4, j = idx % Lk4;
      vp[it] = (i < Lq && j < Lk) ? a.probs[pbase + (long)i * Lk + j] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / kDh, d = idx % kDh;
      if (i < Lq4) sdO[i * kBwdLdD + d] = vo[it];
      if (i < Lk4) bufB[i * kBwdLdD + d] = vv[it];   // V row-major: the dP MFMA's B fragments
    }
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / Lk4, j = idx % Lk4;
      if (idx < Lq4 * Lk4) sP[i * kBwdLd + j] = vp[it];
    }
  }
  __syncthreads();
  bwd_stamp<STAMP>(stamps, 1);
  // dP = dO V^T (masked by the forward's dropout scale) into sdS, on v_mfma_f32_32x32x2_f32 (r06: on the VALU
  // 4x4 blocks it was the kernel's longest phase, 14-29 k cycles, tools/mha_bwd_stamps.py): 32x32 tiles of
  // (query i, key j) dealt round-robin to the waves; A = dO rows, B = V rows, lane (j, half hh) feeding
  // dims 8g + 4hh + e to MFMA e (the forward's K-permutation); rows past the staged ones clamp to row 79
  // (their outputs are never stored)
  {
    const int lane = t & 63, w = t >> 6, jl = lane & 31, hh = lane >> 5;
    const int ntj = (Lk4 + 31) / 32, ntiles = ((Lq4 + 31) / 32) * ntj;
    for (int tile = w; tile < ntiles; tile += kBwdWaves) {
      const int i0 = (tile / ntj) * 32, j0 = (tile % ntj) * 32;
      const float* ap = sdO + min(i0 + jl, kBwdMaxL - 1) * kBwdLdD + 4 * hh;
      const float* bp = bufB + min(j0 + jl, kBwdMaxL - 1) * kBwdLdD + 4 * hh;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const float4 af = *reinterpret_cast<const float4*>(ap + 8 * g);
        const float4 bf = *reinterpret_cast<const float4*>(bp + 8 * g);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.x, bf.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.y, bf.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.z, bf.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.w, bf.w, acc, 0, 0, 0);
      }
      const int j = j0 + jl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + acc_row(r, hh);
        if (i < Lq4 && j < Lk4) {
          float v = 0.f;
          if (i < Lq && j < Lk)
            v = drop ? acc[r] * dasa_dropout_scale(a.p, sdk, (uint64_t)(pbase + (long)i * Lk + j)) : acc[r];
          sdS[i * kBwdLd + j] = v;
        }
      }
    }
  }
  __syncthreads();
  bwd_stamp<STAMP>(stamps, 2);
  for (int i = t; i < Lq; i += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < Lk; ++j) s = fmaf(sP[i * kBwdLd + j], sdS[i * kBwdLd + j], s);
    rowdot[i] = s;
  }
  __syncthreads();
  bwd_stamp<STAMP>(stamps, 3);
  for (int idx = t; idx < Lq4 * Lk4; idx += blockDim.x) {
    const int i = idx / Lk4, j = idx % Lk4;
    float g = 0.f;
    if (i < Lq && j < Lk) g = sP[i * kBwdLd + j] * (sdS[i * kBwdLd + j] - rowdot[i]) * a.scale;
    sdS[i * kBwdLd + j] = g;
    sdST[j * kBwdLd + i] = g;
  }
  __syncthreads();
  bwd_stamp<STAMP>(stamps, 4);
  // the dropped probabilities feed dV; Q and K replace dO^T / V^T
  if (drop)
    for (int idx = t; idx < Lq * Lk; idx += blockDim.x) {
      const int i = idx / Lk, j = idx % Lk;
      sP[i * kBwdLd + j] *= dasa_dropout_scale(a.p, sdk, (uint64_t)(pbase + idx));
    }
  {
    float vq[NR], vk[NR];
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / kDh, d = idx % kDh;
      vq[it] = i < Lq ? a.Q[((long)b * Lq + i) * a.ldq + h * kDh + d] : 0.f;
      vk[it] = i < Lk ? a.K[((long)b * Lk + i) * a.ldk + h * kDh + d] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int idx = t + kBwdThreads * it, i = idx / kDh, d = idx % kDh;
      if (i < Lq4) bufA[i * kBwdLdD + d] = vq[it];
      if (i < Lk4) bufB[i * kBwdLdD + d] = vk[it];
    }
  }
  __syncthreads();
  bwd_stamp<STAMP>(stamps, 5);
  // dV / dQ / dK on v_mfma_f32_32x32x2_f32 (lds_tn_mfma; r06: each was ~9 % of the kernel on the VALU blocks).
  // dV[j][d] = sum_i Pd[i][j] dO[i][d], rows j of this part
  const int jlo = 4 * kb0, jhi = 4 * (kb0 + kbn), ilo = 4 * qb0, ihi = 4 * (qb0 + qbn);
  lds_tn_mfma(sP, kBwdLd, sdO, kBwdLdD, Lq, jlo, jhi, [&](int j, int d, float v) {
    if (j < jhi && j < Lk) dV[((long)b * Lk + j) * a.ldv + h * kDh + d] = v;
  });
  bwd_stamp<STAMP>(stamps, 6);
  // dQ[i][d] = sum_j dS[i][j] K[j][d], rows i of this part
  lds_tn_mfma(sdST, kBwdLd, bufB, kBwdLdD, Lk, ilo, ihi, [&](int i, int d, float v) {
    if (i < ihi && i < Lq) dQ[((long)b * Lq + i) * a.ldq + h * kDh + d] = v;
  });
  bwd_stamp<STAMP>(stamps, 7);
  // dK[j][d] = sum_i dS[i][j] Q[i][d], rows j of this part
  lds_tn_mfma(sdS, kBwdLd, bufA, kBwdLdD, Lq, jlo, jhi, [&](int j, int d, float v) {
    if (j < jhi && j < Lk) dK[((long)b * Lk + j) * a.ldk + h * kDh + d] = v;
  });
  if (STAMP) {   // (stamp 8: this thread's stores drained)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bwd_stamp<STAMP>(stamps, 8);
  }
}

// ------------------------------------------------------------------ misc
__global__ void reverse_valid_kernel(const float* __restrict__ x, const int* __restrict__ len, float* __restrict__ out,
                                     int B, int L, int H) {
  const long total = (long)B * L * (H / 4);
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % (H / 4));
    const long rt = idx / (H / 4);
    const int t = (int)(rt % L), b = (int)(rt / L);
    const int n = len[b];
    DASA_DCHECK(n >= 0 && n <= L, 64);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < n) v = reinterpret_cast<const float4*>(x + ((long)b * L + (n - 1 - t)) * H)[c];
    reinterpret_cast<float4*>(out + ((long)b * L + t) * H)[c] = v;
  }
}

__global__ void dropout_kernel(const float* __restrict__ x, long ldx, float* __restrict__ y, long ldy, int rows,
                               int cols, float p, uint64_t seed, const uint64_t* seed_src) {
  seed = eff_seed(seed, seed_src);
  const long total = (long)rows * cols;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int r = (int)(idx / cols), c = (int)(idx % cols);
    y[(long)r * ldy + c] = x[(long)r * ldx + c] * dasa_dropout_scale(p, seed, (uint64_t)idx);
  }
}

// AdaIN mu/sigma: two rows (content, style) per wave; unbiased variance + eps, sqrt (model.py:1822-1830).
__global__ __launch_bounds__(256) void adain_musigma_kernel(const float* __restrict__ cnt, long ldc,
                                                            const float* __restrict__ sty, long lds,
                                                            float* __restrict__ out, long ldo, float* __restrict__ stats,
                                                            int M, int N, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* c = cnt + (long)row * ldc;
  const float* s = sty + (long)row * lds;
  float sc = 0.f, ss = 0.f;
  for (int i = lane; i < N; i += 64) { sc += c[i]; ss += s[i]; }
  const float mc = wave_sum(sc) / N, ms = wave_sum(ss) / N;
  float vc = 0.f, vs = 0.f;
  for (int i = lane; i < N; i += 64) {
    const float a = c[i] - mc, b = s[i] - ms;
    vc += a * a;
    vs += b * b;
  }
  const float sdc = sqrtf(wave_sum(vc) / (N - 1) + eps), sds = sqrtf(wave_sum(vs) / (N - 1) + eps);
  float* o = out + (long)row * ldo;
  for (int i = lane; i < N; i += 64) o[i] = (c[i] - mc) / sdc * sds + ms;
  if (stats && lane == 0) {
    stats[4 * row + 0] = mc; stats[4 * row + 1] = sdc; stats[4 * row + 2] = ms; stats[4 * row + 3] = sds;
  }
}

// Register-resident variant for N = 256 * NV (2048 -> NV = 8): each lane holds its NV float4 of
// both rows, so content and style are read from HBM exactly once (one round trip per wave).
template <int NV>
__global__ __launch_bounds__(256) void adain_musigma_reg_kernel(const float* __restrict__ cnt, long ldc,
                                                                const float* __restrict__ sty, long lds,
                                                                float* __restrict__ out, long ldo,
                                                                float* __restrict__ stats, int M, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  constexpr int N = 256 * NV;
  const float4* c4 = reinterpret_cast<const float4*>(cnt + (long)row * ldc);
  const float4* s4 = reinterpret_cast<const float4*>(sty + (long)row * lds);
  float4 c[NV], t[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    c[k] = c4[lane + 64 * k];
    t[k] = s4[lane + 64 * k];
  }
  float sc = 0.f, ss = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    sc += (c[k].x + c[k].y) + (c[k].z + c[k].w);
    ss += (t[k].x + t[k].y) + (t[k].z + t[k].w);
  }
  const float mc = wave_sum(sc) / N, ms = wave_sum(ss) / N;
  float vc = 0.f, vs = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float4 a = make_float4(c[k].x - mc, c[k].y - mc, c[k].z - mc, c[k].w - mc);
    const float4 b = make_float4(t[k].x - ms, t[k].y - ms, t[k].z - ms, t[k].w - ms);
    vc += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
    vs += (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
  }
  const float sdc = sqrtf(wave_sum(vc) / (N - 1) + eps), sds = sqrtf(wave_sum(vs) / (N - 1) + eps);
  float4* o4 = reinterpret_cast<float4*>(out + (long)row * ldo);
#pragma unroll
  for (int k = 0; k < NV; ++k)
    o4[lane + 64 * k] = make_float4((c[k].x - mc) / sdc * sds + ms, (c[k].y - mc) / sdc * sds + ms,
                                    (c[k].z - mc) / sdc * sds + ms, (c[k].w - mc) / sdc * sds + ms);
  if (stats && lane == 0) {
    stats[4 * row + 0] = mc; stats[4 * row + 1] = sdc; stats[4 * row + 2] = ms; stats[4 * row + 3] = sds;
  }
}

// AdaIN mu/sigma backward (autograd of model.py:1822-1840), one wave per row, statistics recomputed.
// With xh = (c - mc)/sc, g = dout:  dc = (ss/sc) * (g - mean(g) - xh * sum(g xh)/(N-1));
// ds = sum(g)/N + sum(g xh) * (s - ms) / ((N-1) ss). dc / ds may be NULL.
__global__ __launch_bounds__(256) void adain_musigma_bwd_kernel(const float* __restrict__ cnt, long ldc,
                                                                const float* __restrict__ sty, long lds,
                                                                const float* __restrict__ dout, long ldg,
                                                                float* __restrict__ dc, long lddc,
                                                                float* __restrict__ ds, long ldds, int M, int N,
                                                                float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* c = cnt + (long)row * ldc;
  const float* s = sty + (long)row * lds;
  const float* g = dout + (long)row * ldg;
  float sc = 0.f, ss = 0.f;
  for (int i = lane; i < N; i += 64) { sc += c[i]; ss += s[i]; }
  const float mc = wave_sum(sc) / N, ms = wave_sum(ss) / N;
  float vc = 0.f, vs = 0.f;
  for (int i = lane; i < N; i += 64) {
    const float a = c[i] - mc, b = s[i] - ms;
    vc += a * a;
    vs += b * b;
  }
  const float sdc = sqrtf(wave_sum(vc) / (N - 1) + eps), sds = sqrtf(wave_sum(vs) / (N - 1) + eps);
  const float rc = 1.f / sdc;
  float sg = 0.f, sgx = 0.f;
  for (int i = lane; i < N; i += 64) {
    const float gi = g[i];
    sg += gi;
    sgx += gi * (c[i] - mc) * rc;
  }
  sg = wave_sum(sg);
  sgx = wave_sum(sgx);
  const float mg = sg / N, kx = sgx / (N - 1);
  if (dc) {
    float* o = dc + (long)row * lddc;
    const float f = sds * rc;
    for (int i = lane; i < N; i += 64) o[i] = f * (g[i] - mg - (c[i] - mc) * rc * kx);
  }
  if (ds) {
    float* o = ds + (long)row * ldds;
    const float ks = sgx / ((N - 1) * sds);
    for (int i = lane; i < N; i += 64) o[i] = mg + (s[i] - ms) * ks;
  }
}

// ---- bf16 attention core (BASELINE configs[4]'s bf16 mode: bf16 activations, fp32 accumulation) ------
// mha_fwd_kernel's structure on v_mfma_f32_32x32x16_bf16: Q / K / V arrive as bf16 (the fused QKV GEMM's
// bf16 output), S^T = K Q^T and O = P V accumulate in fp32, the scale / mask / softmax run in fp32 on the
// accumulator and P is rounded to bf16 (RNE) as the P V operand. One workgroup per (batch, head), one wave
// per 32-query tile. K is staged in LDS row-major ([key][64] bf16, 144-B rows: conflict-free 16-B fragment
// reads); V is staged TRANSPOSED ([dim][key], 272-B rows), because the P V B-operand of lane (dim d, half
// hh) is 8 keys of one dim: with the probability accumulator as the A operand, k-slot i of half hh is key
// 16u + (i & 3) + 8 (i >> 2) + 4 hh of the 32-key tile (u = 0, 1: the tile's two 16-key MFMAs) — the
// accumulator rows acc_row(8u + i, hh) — i.e. two runs of 4 consecutive keys: two ds_read_b64 per MFMA.
// The output is fp32, or bf16 (RNE) for a bf16 consumer (the attention output projection).
typedef short mha_bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kKLdH = kDh + 8;     // K rows in LDS (bf16 elements)
constexpr int kVtLdH = kMaxLk + 8;  // V^T rows in LDS (bf16 elements)

struct MhaBfArgs {
  const unsigned short* Q; long ldq; const unsigned short* K; long ldk; const unsigned short* V; long ldv;
  const float* mask; void* out; long ldo;
  int B, heads, Lq, Lk; float scale; float p; uint64_t seed; const uint64_t* seed_src;
};

__device__ __forceinline__ unsigned short bf16_rne(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }

template <int NKT, bool OBF>
__global__ __launch_bounds__(256) void mha_fwd_bf16_kernel(MhaBfArgs a, int nqt) {
  __shared__ __attribute__((aligned(16))) unsigned short ks[NKT * 32 * kKLdH];
  __shared__ __attribute__((aligned(16))) unsigned short vt[kDh * kVtLdH];
  __shared__ float ms[NKT * 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.x, h = bh % a.heads, b = bh / a.heads;
  const int Lq = a.Lq, Lk = a.Lk;
  const uint64_t seed = a.p > 0.f ? eff_seed(a.seed, a.seed_src) : 0;
  const int q0 = w * 32, j = lane & 31, hh = lane >> 5;
  // every global load first: this wave's Q fragments (B operand of S^T: lane (query j, half hh) holds
  // Q[q0 + j][16 s + 8 hh .. +7]), the K / V rows of the head (16-B pieces, rows clamped) and the mask
  const unsigned short* qp = a.Q + ((long)b * Lq + min(q0 + j, Lq - 1)) * a.ldq + h * kDh + 8 * hh;
  mha_bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const mha_bf16x8*>(qp + 16 * s);
  uint4 kx[NKT], vx[NKT];   // NKT * 32 rows x 8 pieces over 256 threads
#pragma unroll
  for (int i = 0; i < NKT; ++i) {
    const int idx = threadIdx.x + 256 * i, row = min(idx >> 3, Lk - 1), c = idx & 7;
    kx[i] = *reinterpret_cast<const uint4*>(a.K + ((long)b * Lk + row) * a.ldk + h * kDh + 8 * c);
    vx[i] = *reinterpret_cast<const uint4*>(a.V + ((long)b * Lk + row) * a.ldv + h * kDh + 8 * c);
  }
  const int mk = min((int)threadIdx.x, Lk - 1);
  const float mv = a.mask ? a.mask[(long)b * Lk + mk] : 0.f;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NKT; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx >> 3, c = idx & 7;
    const unsigned z = row < Lk ? 0xffffffffu : 0u;
    *reinterpret_cast<uint4*>(ks + row * kKLdH + 8 * c) = uint4{kx[i].x & z, kx[i].y & z, kx[i].z & z, kx[i].w & z};
    const unsigned vv[4] = {vx[i].x & z, vx[i].y & z, vx[i].z & z, vx[i].w & z};
#pragma unroll
    for (int e = 0; e < 8; ++e)
      vt[(8 * c + e) * kVtLdH + row] = (unsigned short)(vv[e >> 1] >> (16 * (e & 1)));
  }
  if (threadIdx.x < NKT * 32) ms[threadIdx.x] = (int)threadIdx.x < Lk ? mv : -INFINITY;
  __syncthreads();
  if (w >= nqt) return;   // (no barrier below)
  floatx16 st[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const unsigned short* kp = ks + (kt * 32 + j) * kKLdH + 8 * hh;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const mha_bf16x8*>(kp + 16 * s), qf[s], acc, 0,
                                                   0, 0);
    st[kt] = acc;
  }
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = st[kt][r] * a.scale + ms[kt * 32 + acc_row(r, hh)];
      st[kt][r] = v;
      m = fmaxf(m, v);
    }
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __expf(st[kt][r] - m);
      st[kt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
  const long prow = ((long)bh * Lq + q0 + j) * (long)Lk;   // dropout index base of this query row
  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      mha_bf16x8 pa;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float pv = st[kt][8 * u + i] * inv;
        if (a.p > 0.f) pv *= dasa_dropout_scale(a.p, seed, (uint64_t)(prow + kt * 32 + acc_row(8 * u + i, hh)));
        pa[i] = (short)bf16_rne(pv);
      }
      const unsigned short* v0 = vt + j * kVtLdH + kt * 32 + 16 * u + 4 * hh;
      const unsigned short* v1 = v0 + 32 * kVtLdH;
      const uint2 a0 = *reinterpret_cast<const uint2*>(v0), b0 = *reinterpret_cast<const uint2*>(v0 + 8);
      const uint2 a1 = *reinterpret_cast<const uint2*>(v1), b1 = *reinterpret_cast<const uint2*>(v1 + 8);
      o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(mha_bf16x8, uint4{a0.x, a0.y, b0.x, b0.y}),
                                                  o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(mha_bf16x8, uint4{a1.x, a1.y, b1.x, b1.y}),
                                                  o1, 0, 0, 0);
    }
  // O tile: column = dim j (+32), row = query q0 + acc_row(r, hh)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qq = q0 + acc_row(r, hh);
    if (qq < Lq) {
      const long o = ((long)b * Lq + qq) * a.ldo + h * kDh + j;
      if (OBF) {
        unsigned short* op = reinterpret_cast<unsigned short*>(a.out) + o;
        op[0] = bf16_rne(o0[r]);
        op[32] = bf16_rne(o1[r]);
      } else {
        float* op = reinterpret_cast<float*>(a.out) + o;
        op[0] = o0[r];
        op[32] = o1[r];
      }
    }
  }
}

}  // namespace

extern "C" int dasa_version(void) { return 2; }
extern "C" const char* dasa_build_info(void) { return "libdasa_hip gfx950 (CDNA4) fp32-MFMA v1"; }

#define DASA_VPL_DISPATCH_B(N, KERNEL, GRID, BLOCK, ...)                                    \
  do {                                                                                     \
    const int vpl = ((N) / 4 + 63) / 64;                                                   \
    switch (vpl) {                                                                         \
      case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(BLOCK), 0, st, __VA_ARGS__); break; \
      case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(BLOCK), 0, st, __VA_ARGS__); break; \
      case 3: hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(BLOCK), 0, st, __VA_ARGS__); break; \
      case 4: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(BLOCK), 0, st, __VA_ARGS__); break; \
      case 8: case 5: case 6: case 7:                                                      \
        hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(BLOCK), 0, st, __VA_ARGS__); break;       \
      default: return (int)hipErrorInvalidValue;                                           \
    }                                                                                      \
  } while (0)
#define DASA_VPL_DISPATCH(N, KERNEL, GRID, ...) DASA_VPL_DISPATCH_B(N, KERNEL, GRID, 256, __VA_ARGS__)

extern "C" int dasa_layernorm_fwd_bf16(const float* x, const float* res, const float* gamma, const float* beta,
                                       float* y, uint16_t* ybf, float* mean, float* rstd, float* xsum, int32_t M,
                                       int32_t N, float eps, float drop_p, uint64_t seed, void* stream) {
  if (M <= 0) return 0;
  if ((N & 3) || N > 8192 || ((uintptr_t)ybf & 7)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DASA_VPL_DISPATCH(N, ln_fwd_kernel, dim3(cdivi(M, 4)), x, res, gamma, beta, y, mean, rstd, xsum, M, N, eps, drop_p,
                    seed, drop_p > 0.f ? dasa_seed_src_host() : nullptr, reinterpret_cast<unsigned short*>(ybf));
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_layernorm_fwd(const float* x, const float* res, const float* gamma, const float* beta, float* y,
                                  float* mean, float* rstd, float* xsum, int32_t M, int32_t N, float eps,
                                  float drop_p, uint64_t seed, void* stream) {
  return dasa_layernorm_fwd_bf16(x, res, gamma, beta, y, nullptr, mean, rstd, xsum, M, N, eps, drop_p, seed, stream);
}

extern "C" int dasa_layernorm_bwd(const float* dy, const float* xsum, const float* gamma, const float* mean,
                                  const float* rstd, float* dx, float* dgamma, float* dbeta, int32_t M, int32_t N,
                                  void* stream) {
  if (M <= 0) return 0;
  if ((N & 3) || N > 8192) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int colBlocks = (dgamma || dbeta) ? cdivi(N >> 2, 64) : 0;
  DASA_VPL_DISPATCH_B(N, ln_bwd_kernel, dim3(cdivi(M, kLnBwdWaves) + colBlocks), 64 * kLnBwdWaves, dy, xsum, gamma,
                      mean, rstd, dx, dgamma, dbeta, M, N);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_bert_embed_fwd(const int64_t* ids, const float* word, const float* pos, const float* type0,
                                   const float* gamma, const float* beta, float* out, int32_t B, int32_t L, int32_t H,
                                   float eps, float drop_p, uint64_t seed, void* stream) {
  if (B <= 0 || L <= 0) return 0;
  if ((H & 3) || H > 8192) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DASA_VPL_DISPATCH(H, embed_kernel, dim3(cdivi((long)B * L, 4)), ids, word, pos, type0, gamma, beta, out, B, L, H,
                    eps, drop_p, seed, drop_p > 0.f ? dasa_seed_src_host() : nullptr);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_mha_fwd(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                            const float* addmask, float* out, int64_t ldo, float* probs, int32_t B, int32_t heads,
                            int32_t Lq, int32_t Lk, int32_t dh, float scale, float drop_p, uint64_t seed,
                            void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (dh != kDh || Lk <= 0 || Lk > kMaxLk || ((ldq | ldk | ldv) & 3) ||
      (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V) & 15))
    return (int)hipErrorInvalidValue;
  MhaArgs a{Q, ldq, K, ldk, V, ldv, addmask, out, ldo, probs, B, heads, Lq, Lk, scale, drop_p, seed,
            drop_p > 0.f ? dasa_seed_src_host() : nullptr};
  const int nqt = cdivi(Lq, 32);
  if (nqt > 4) return (int)hipErrorInvalidValue;   // one wave per 32-query tile, Lq <= 128
  // 4 waves always: all of them stage K / V, waves past the query tiles then leave
  const dim3 grid(B * heads), block(256);
  hipStream_t st = (hipStream_t)stream;
  switch (cdivi(Lk, 32)) {
    case 1: hipLaunchKernelGGL(mha_fwd_kernel<1>, grid, block, 0, st, a, nqt); break;
    case 2: hipLaunchKernelGGL(mha_fwd_kernel<2>, grid, block, 0, st, a, nqt); break;
    case 3: hipLaunchKernelGGL(mha_fwd_kernel<3>, grid, block, 0, st, a, nqt); break;
    default: hipLaunchKernelGGL(mha_fwd_kernel<4>, grid, block, 0, st, a, nqt); break;
  }
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_mha_fwd_bf16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv,
                                 const float* addmask, void* out, int64_t ldo, int32_t out_bf16, int32_t B,
                                 int32_t heads, int32_t Lq, int32_t Lk, int32_t dh, float scale, float drop_p,
                                 uint64_t seed, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (dh != kDh || Lk <= 0 || Lk > kMaxLk || ((ldq | ldk | ldv) & 7) ||
      (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V) & 15) || !out)
    return (int)hipErrorInvalidValue;
  const int nqt = cdivi(Lq, 32);
  if (nqt > 4) return (int)hipErrorInvalidValue;   // one wave per 32-query tile, Lq <= 128
  MhaBfArgs a{(const unsigned short*)Q, ldq, (const unsigned short*)K, ldk, (const unsigned short*)V, ldv, addmask,
              out, ldo, B, heads, Lq, Lk, scale, drop_p, seed, drop_p > 0.f ? dasa_seed_src_host() : nullptr};
  const dim3 grid(B * heads), block(256);
  hipStream_t st = (hipStream_t)stream;
  const int nkt = cdivi(Lk, 32);
#define DASA_MHA_BF(NKT)                                                                      \
  if (out_bf16) hipLaunchKernelGGL((mha_fwd_bf16_kernel<NKT, true>), grid, block, 0, st, a, nqt); \
  else hipLaunchKernelGGL((mha_fwd_bf16_kernel<NKT, false>), grid, block, 0, st, a, nqt);
  switch (nkt) {
    case 1: DASA_MHA_BF(1) break;
    case 2: DASA_MHA_BF(2) break;
    case 3: DASA_MHA_BF(3) break;
    default: DASA_MHA_BF(4) break;
  }
#undef DASA_MHA_BF
  DASA_CHECK_LAUNCH();
  return 0;
}

// workgroups per (batch, head) of the Lq, Lk <= 80 attention backward: 0 = automatic, n >= 1 forced
static int g_mha_bwd_parts = 0;
static unsigned long long* g_mha_stamps = nullptr;   // dasa_mha_bwd_stamps (diagnosis)
extern "C" int dasa_mha_bwd_stamps(void* buf) {
  g_mha_stamps = (unsigned long long*)buf;
  return kBwdStamps;
}
extern "C" int dasa_mha_bwd_split(int32_t parts) {
  const int prev = g_mha_bwd_parts;
  if (parts >= 0) g_mha_bwd_parts = parts > 16 ? 16 : parts;
  return prev;
}

extern "C" int dasa_mha_bwd(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                            const float* probs, const float* dout, int64_t lddo, float* dQ, float* dK, float* dV,
                            int32_t B, int32_t heads, int32_t Lq, int32_t Lk, int32_t dh, float scale, float drop_p,
                            uint64_t seed, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (dh != kDh || Lk <= 0 || Lk > kMaxLk || !probs) return (int)hipErrorInvalidValue;
  MhaArgs a{Q, ldq, K, ldk, V, ldv, nullptr, nullptr, 0, const_cast<float*>(probs), B, heads, Lq, Lk, scale, drop_p,
            seed, drop_p > 0.f ? dasa_seed_src_host() : nullptr};
  const bool vec = ((ldq | ldk | ldv) & 3) == 0 && (((uintptr_t)dQ | (uintptr_t)dK | (uintptr_t)dV) & 15) == 0;
  if (Lq <= kBwdMaxL && Lk <= kBwdMaxL && vec) {
    int parts = g_mha_bwd_parts;
    if (parts <= 0) {   // auto: up to 4 parts while B x heads x parts stays within one round of 256 CUs
      parts = 256 / (B * heads);
      parts = parts < 1 ? 1 : parts > 4 ? 4 : parts;
    }
    if (g_mha_stamps)
      hipLaunchKernelGGL(mha_bwd_lds_kernel<true>, dim3(B * heads * parts), dim3(kBwdThreads), 0, (hipStream_t)stream, a, dout,
                         (long)lddo, dQ, dK, dV, parts, g_mha_stamps);
    else
      hipLaunchKernelGGL(mha_bwd_lds_kernel<false>, dim3(B * heads * parts), dim3(kBwdThreads), 0, (hipStream_t)stream, a,
                         dout, (long)lddo, dQ, dK, dV, parts, nullptr);
  } else
    hipLaunchKernelGGL(mha_bwd_kernel, dim3(B * heads), dim3(256), 0, (hipStream_t)stream, a, dout, (long)lddo, dQ, dK,
                       dV);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_reverse_valid(const float* x, const int32_t* lengths, float* out, int32_t B, int32_t L, int32_t H,
                                  void* stream) {
  if (B <= 0 || L <= 0) return 0;
  if (H & 3) return (int)hipErrorInvalidValue;
  const long total = (long)B * L * (H / 4);
  int grid = cdivi(total, 256);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(reverse_valid_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, lengths, out, B, L, H);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_dropout_fwd(const float* x, int64_t ldx, float* y, int64_t ldy, int32_t rows, int32_t cols,
                                float p, uint64_t seed, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (dasa_dropout_vec(x, (long)ldx, y, (long)ldy, rows, cols, p, seed, (hipStream_t)stream)) {
    DASA_CHECK_LAUNCH();
    return 0;
  }
  const long total = (long)rows * cols;
  int grid = cdivi(total, 256);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, (long)ldx, y, (long)ldy, rows,
                     cols, p, seed, dasa_seed_src_host());
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_adain_musigma_fwd(const float* content, int64_t ldc_, const float* style, int64_t lds, float* out,
                                      int64_t ldo, float* stats, int32_t M, int32_t N, float eps, void* stream) {
  if (M <= 0) return 0;
  if (N < 2) return (int)hipErrorInvalidValue;
  const bool al = !(((uintptr_t)content | (uintptr_t)style | (uintptr_t)out) & 15) && !((ldc_ | lds | ldo) & 3);
  if (al && N == 2048) {
    hipLaunchKernelGGL(adain_musigma_reg_kernel<8>, dim3(cdivi(M, 4)), dim3(256), 0, (hipStream_t)stream, content,
                       (long)ldc_, style, (long)lds, out, (long)ldo, stats, M, eps);
    DASA_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(adain_musigma_kernel, dim3(cdivi(M, 4)), dim3(256), 0, (hipStream_t)stream, content,
                     (long)ldc_, style, (long)lds, out, (long)ldo, stats, M, N, eps);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_adain_musigma_bwd(const float* content, int64_t ldc_, const float* style, int64_t lds,
                                      const float* dout, int64_t ldg, float* dcontent, int64_t lddc, float* dstyle,
                                      int64_t ldds, int32_t M, int32_t N, float eps, void* stream) {
  if (M <= 0 || (!dcontent && !dstyle)) return 0;
  if (N < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adain_musigma_bwd_kernel, dim3(cdivi(M, 4)), dim3(256), 0, (hipStream_t)stream, content,
                     (long)ldc_, style, (long)lds, dout, (long)ldg, dcontent, (long)lddc, dstyle, (long)ldds, M, N,
                     eps);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" const char* dasa_error_string(int e) { return hipGetErrorString((hipError_t)e); }
