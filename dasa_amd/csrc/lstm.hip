// LSTM kernels for gfx950: the decoder nn.LSTMCell (model.py:437,514) and the encoder's packed
// bidirectional nn.LSTM (r2rmodel.py:2239-2243, 2339-2354).
//
// Bi-LSTM forward: the input projection for all timesteps is one MFMA GEMM (dasa_gemm_f32, done by
// the caller); the recurrence is L dependent step launches (one per timestep, both directions in one
// grid). For B <= 32 a step is fused: each workgroup owns 8 hidden units = 32 gate columns (i,f,g,o
// interleaved so the cell update is workgroup-local), its 4 waves split the K=H recurrent reduction
// with v_mfma_f32_32x32x2_f32 (batch rows padded to 32), reduce through LDS and apply the cell.
// W_hh (2 x 16 MB) is re-read every step and stays L2/MALL-resident.
// Packed-sequence semantics: a row is active at time t iff t < len[b]; inactive steps freeze the
// forward state, keep the backward state at zero, and emit zero outputs (pad_packed_sequence).
#include "common.h"
#include <cstdlib>
#include "lstm_internal.h"
#include "../../include/dasa_hip.h"

namespace {

__device__ __forceinline__ float tanh_(float x) { return tanhf(x); }

// ---------------------------------------------------------------- decoder LSTMCell
__global__ void lstm_cell_fwd_kernel(const float* __restrict__ gates, const float* __restrict__ c_prev,
                                     float* __restrict__ h, float* __restrict__ c, float* __restrict__ act,
                                     int B, int H) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx % H;
  const float* g = gates + (long)b * 4 * H;
  const float i = sigmoidf_(g[j]), f = sigmoidf_(g[H + j]), gg = tanh_(g[2 * H + j]), o = sigmoidf_(g[3 * H + j]);
  const float cn = f * c_prev[idx] + i * gg;
  c[idx] = cn;
  h[idx] = o * tanh_(cn);
  if (act) {
    float* a = act + (long)b * 4 * H;
    a[j] = i; a[H + j] = f; a[2 * H + j] = gg; a[3 * H + j] = o;
  }
}

__global__ void lstm_cell_bwd_kernel(const float* __restrict__ act, const float* __restrict__ c_prev,
                                     const float* __restrict__ c, const float* __restrict__ dh,
                                     const float* __restrict__ dc, float* __restrict__ dgates,
                                     float* __restrict__ dc_prev, int B, int H) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx % H;
  const float* a = act + (long)b * 4 * H;
  const float i = a[j], f = a[H + j], gg = a[2 * H + j], o = a[3 * H + j];
  const float tc = tanh_(c[idx]);
  const float dhv = dh ? dh[idx] : 0.f;
  const float dcv = (dc ? dc[idx] : 0.f) + dhv * o * (1.f - tc * tc);
  float* dg = dgates + (long)b * 4 * H;
  dg[j] = dcv * gg * i * (1.f - i);
  dg[H + j] = dcv * c_prev[idx] * f * (1.f - f);
  dg[2 * H + j] = dcv * i * (1.f - gg * gg);
  dg[3 * H + j] = dhv * tc * o * (1.f - o);
  if (dc_prev) dc_prev[idx] = dcv * f;
}

// ---------------------------------------------------------------- bi-LSTM recurrence
struct SeqArgs {
  const float* xproj;   // [B][L][2][4H]
  const float* whh0;    // [4H][H] forward direction
  const float* whh1;    // [4H][H] backward direction
  const int* len;       // [B]
  float* out;           // [B][L][2H]
  const float* hin;     // [2][B][H]
  float* hout;          // [2][B][H]
  float* c;             // [2][B][H]
  float* save_act;      // [L][2][B][4H] or NULL
  float* save_c;        // [L][2][B][H] or NULL
  const float* rec;     // [2][B][4H] (unfused path) or NULL
  int B, L, H;
};

__device__ __forceinline__ void cell_apply(const SeqArgs& a, int dir, int t, int b, int u, float g0, float g1,
                                           float g2, float g3) {
  const int H = a.H;
  const long sidx = ((long)dir * a.B + b) * H + u;
  const float* xp = a.xproj + (((long)b * a.L + t) * 2 + dir) * 4 * H;
  g0 += xp[u]; g1 += xp[H + u]; g2 += xp[2 * H + u]; g3 += xp[3 * H + u];
  float* outp = a.out + ((long)b * a.L + t) * 2 * H + dir * H + u;
  if (t < a.len[b]) {
    const float i = sigmoidf_(g0), f = sigmoidf_(g1), gg = tanh_(g2), o = sigmoidf_(g3);
    const float cn = f * a.c[sidx] + i * gg;
    const float hn = o * tanh_(cn);
    a.c[sidx] = cn;
    a.hout[sidx] = hn;
    *outp = hn;
    if (a.save_act) {
      float* sa = a.save_act + (((long)t * 2 + dir) * a.B + b) * 4 * H;
      sa[u] = i; sa[H + u] = f; sa[2 * H + u] = gg; sa[3 * H + u] = o;
      a.save_c[(((long)t * 2 + dir) * a.B + b) * H + u] = cn;
    }
  } else {
    a.hout[sidx] = a.hin[sidx];
    *outp = 0.f;
    if (a.save_act) {
      float* sa = a.save_act + (((long)t * 2 + dir) * a.B + b) * 4 * H;
      sa[u] = 0.f; sa[H + u] = 0.f; sa[2 * H + u] = 0.f; sa[3 * H + u] = 0.f;
      a.save_c[(((long)t * 2 + dir) * a.B + b) * H + u] = a.c[sidx];
    }
  }
}

// Fused step for B <= 32: grid (H/4, 2), 1024 threads. A workgroup owns 4 hidden units = 16 gate
// columns (i,f,g,o interleaved); its 16 waves split the K = H recurrent reduction (v_mfma_f32_16x16x4_f32,
// batch rows padded to 2 x 16) and reduce through LDS before the cell update.
constexpr int kFwdUnits = 4, kFwdWaves = 16;
__global__ __launch_bounds__(1024) void bilstm_step_fused_kernel(SeqArgs a, int s) {
  __shared__ float red[kFwdWaves][32][17];
  const int dir = blockIdx.y, u0 = blockIdx.x * kFwdUnits;
  const int H = a.H, B = a.B;
  const int t = dir == 0 ? s : a.L - 1 - s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i16 = lane & 15, kg = lane >> 4;
  // rows >= B are clamped to B-1 and zeroed by a select (no branch around the loads)
  const float* h0 = a.hin + ((long)dir * B + min(i16, B - 1)) * H;
  const float* h1 = a.hin + ((long)dir * B + min(16 + i16, B - 1)) * H;
  const bool r0 = i16 < B, r1 = 16 + i16 < B;
  const int q = i16 & 3, unit = u0 + (i16 >> 2);
  const float* wrow = (dir ? a.whh1 : a.whh0) + ((long)q * H + unit) * H;
  const int kq = H / kFwdWaves, k0 = w * kq;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int kb = k0; kb < k0 + kq; kb += 16) {
    const int ko = kb + 4 * kg;
    const float4 bv = *reinterpret_cast<const float4*>(wrow + ko);
    float4 a0 = *reinterpret_cast<const float4*>(h0 + ko);
    float4 a1 = *reinterpret_cast<const float4*>(h1 + ko);
    if (!r0) a0 = z;   // uniform per lane-row; component selects, no branch around the loads
    if (!r1) a1 = z;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, bv.x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bv.y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, bv.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bv.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, bv.z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bv.w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, bv.w, acc1, 0, 0, 0);
  }
  // 16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + reg
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w][4 * kg + r][i16] = acc0[r];
    red[w][16 + 4 * kg + r][i16] = acc1[r];
  }
  __syncthreads();
  if (threadIdx.x < 32 * kFwdUnits) {
    const int b = threadIdx.x / kFwdUnits, ul = threadIdx.x % kFwdUnits;
    if (b < B) {
      float g[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ww = 0; ww < kFwdWaves; ++ww)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) g[qq] += red[ww][b][4 * ul + qq];
      cell_apply(a, dir, t, b, u0 + ul, g[0], g[1], g[2], g[3]);
    }
  }
}

// Unfused step (any B): rec = h W_hh^T computed by dasa_gemm_f32 beforehand.
__global__ void bilstm_step_cell_kernel(SeqArgs a, int s) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = 2 * a.B * a.H;
  if (idx >= total) return;
  const int dir = idx / (a.B * a.H), rem = idx % (a.B * a.H), b = rem / a.H, u = rem % a.H;
  const int t = dir == 0 ? s : a.L - 1 - s;
  const float* rr = a.rec + ((long)dir * a.B + b) * 4 * a.H;
  cell_apply(a, dir, t, b, u, rr[u], rr[a.H + u], rr[2 * a.H + u], rr[3 * a.H + u]);
}

__global__ void fill_kernel(float* p, long n, float v) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void copy_kernel(const float* src, float* dst, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------- bi-LSTM BPTT
struct BpttArgs {
  const float* wt0;       // W_hh^T [H][4H] forward direction (transposed once per call)
  const float* wt1;
  const int* len;
  const float* save_act;  // [L][2][B][4H]
  const float* save_c;    // [L][2][B][H]
  const float* dout;      // [B][L][2H]
  float* dgates;          // [B][L][2][4H]
  float* dh;              // [2][B][H] carry
  float* dc;              // [2][B][H] carry
  int B, L, H;
};

// out[c][r] = in[r][c] for an [R][C] matrix, 32x32 LDS tiles.
__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, int R, int C) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < R && c < C) ? in[(long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (c < C && r < R) out[(long)c * R + r] = tile[tx][k];
  }
}

// BPTT step for B <= 32: grid (H/16, 2), 1024 threads. The workgroup owns 16 hidden units j: its 16
// waves split the K = 4H reduction rec[b][j] = sum_n dgates_prev[b][n] W_hh[n][j] (v_mfma 16x16x4 on
// W_hh^T so both operands stream K-contiguous float4s), then the cell backward for those units.
constexpr int kBwdUnits = 16, kBwdWaves = 16;
__global__ __launch_bounds__(1024) void bilstm_bptt_step_kernel(BpttArgs a, int s) {
  __shared__ float red[kBwdWaves][32][17];
  const int dir = blockIdx.y, j0 = blockIdx.x * kBwdUnits;
  const int H = a.H, B = a.B, L = a.L, G4 = 4 * H;
  const int t = dir == 0 ? (L - 1 - s) : s;
  const int tp = dir == 0 ? t + 1 : t - 1;  // step processed just before in BPTT order
  const bool tpv = tp >= 0 && tp < L;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i16 = lane & 15, kg = lane >> 4;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (tpv) {
    const bool r0 = i16 < B, r1 = 16 + i16 < B;
    const float* g0 = a.dgates + (((long)min(i16, B - 1) * L + tp) * 2 + dir) * G4;
    const float* g1 = a.dgates + (((long)min(16 + i16, B - 1) * L + tp) * 2 + dir) * G4;
    const float* wt = (dir ? a.wt1 : a.wt0) + (long)(j0 + i16) * G4;
    const int kq = G4 / kBwdWaves, k0 = w * kq;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int kb = k0; kb < k0 + kq; kb += 16) {
      const int ko = kb + 4 * kg;
      const float4 bv = *reinterpret_cast<const float4*>(wt + ko);
      float4 a0 = *reinterpret_cast<const float4*>(g0 + ko);
      float4 a1 = *reinterpret_cast<const float4*>(g1 + ko);
      if (!r0) a0 = z;
      if (!r1) a1 = z;
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bv.x, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, bv.x, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bv.y, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, bv.y, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bv.z, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, bv.z, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bv.w, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, bv.w, acc1, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w][4 * kg + r][i16] = acc0[r];
    red[w][16 + 4 * kg + r][i16] = acc1[r];
  }
  __syncthreads();
  if (threadIdx.x < 32 * kBwdUnits) {
    const int b = threadIdx.x / kBwdUnits, jl = threadIdx.x % kBwdUnits, j = j0 + jl;
    if (b < B) {
      float rec = 0.f;
#pragma unroll
      for (int i = 0; i < kBwdWaves; ++i) rec += red[i][b][jl];
      const long sidx = ((long)dir * B + b) * H + j;
      float* dg = a.dgates + (((long)b * L + t) * 2 + dir) * G4;
      if (t < a.len[b]) {
        const float G = rec + a.dout[((long)b * L + t) * 2 * H + dir * H + j] + a.dh[sidx];
        const float* sa = a.save_act + (((long)t * 2 + dir) * B + b) * G4;
        const float i_ = sa[j], f_ = sa[H + j], g_ = sa[2 * H + j], o_ = sa[3 * H + j];
        const float ct = a.save_c[(((long)t * 2 + dir) * B + b) * H + j];
        const int tq = dir == 0 ? t - 1 : t + 1;  // previous step in forward order
        const float cp = (tq >= 0 && tq < L) ? a.save_c[(((long)tq * 2 + dir) * B + b) * H + j] : 0.f;
        const float tc = tanh_(ct);
        const float dcv = a.dc[sidx] + G * o_ * (1.f - tc * tc);
        dg[j] = dcv * g_ * i_ * (1.f - i_);
        dg[H + j] = dcv * cp * f_ * (1.f - f_);
        dg[2 * H + j] = dcv * i_ * (1.f - g_ * g_);
        dg[3 * H + j] = G * tc * o_ * (1.f - o_);
        a.dc[sidx] = dcv * f_;
        a.dh[sidx] = 0.f;
      } else {
        dg[j] = 0.f; dg[H + j] = 0.f; dg[2 * H + j] = 0.f; dg[3 * H + j] = 0.f;
        a.dh[sidx] = rec + a.dh[sidx];
      }
    }
  }
}

// BPTT cell step for any B (the recurrent product rec[dir][b][j] was computed by dasa_gemm_f32).
// Carries dh/dc [2][B][H] live in the workspace; same math as the fused step kernel above.
__global__ void bilstm_bptt_cell_kernel(BpttArgs a, const float* __restrict__ rec, int s) {
  const long total = 2L * a.B * a.H;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int H = a.H, B = a.B, L = a.L, G4 = 4 * H;
  const int dir = (int)(idx / ((long)B * H));
  const int rem = (int)(idx % ((long)B * H)), b = rem / H, j = rem % H;
  const int t = dir == 0 ? (L - 1 - s) : s;
  const float r = s > 0 ? rec[idx] : 0.f;
  float* dg = a.dgates + (((long)b * L + t) * 2 + dir) * G4;
  if (t < a.len[b]) {
    const float G = r + a.dout[((long)b * L + t) * 2 * H + dir * H + j] + a.dh[idx];
    const float* sa = a.save_act + (((long)t * 2 + dir) * B + b) * G4;
    const float i_ = sa[j], f_ = sa[H + j], g_ = sa[2 * H + j], o_ = sa[3 * H + j];
    const float ct = a.save_c[(((long)t * 2 + dir) * B + b) * H + j];
    const int tq = dir == 0 ? t - 1 : t + 1;
    const float cp = (tq >= 0 && tq < L) ? a.save_c[(((long)tq * 2 + dir) * B + b) * H + j] : 0.f;
    const float tc = tanh_(ct);
    const float dcv = a.dc[idx] + G * o_ * (1.f - tc * tc);
    dg[j] = dcv * g_ * i_ * (1.f - i_);
    dg[H + j] = dcv * cp * f_ * (1.f - f_);
    dg[2 * H + j] = dcv * i_ * (1.f - g_ * g_);
    dg[3 * H + j] = G * tc * o_ * (1.f - o_);
    a.dc[idx] = dcv * f_;
    a.dh[idx] = 0.f;
  } else {
    dg[j] = 0.f; dg[H + j] = 0.f; dg[2 * H + j] = 0.f; dg[3 * H + j] = 0.f;
    a.dh[idx] = r + a.dh[idx];
  }
}

// hprev[dir][b][t][:] = the recurrent input of step t: fwd out[b][t-1][0:H], bwd out[b][t+1][H:2H], 0 at the ends.
__global__ void bilstm_hprev_kernel(const float* __restrict__ out, float* __restrict__ hprev, int B, int L, int H) {
  const long total = 2L * B * L * H;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int j = (int)(i % H);
    long r = i / H;
    const int t = (int)(r % L);
    r /= L;
    const int b = (int)(r % B), dir = (int)(r / B);
    const int ts = dir == 0 ? t - 1 : t + 1;
    hprev[i] = (ts >= 0 && ts < L) ? out[((long)b * L + ts) * 2 * H + dir * H + j] : 0.f;
  }
}

inline int cdivi(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace

extern "C" int dasa_bilstm_hprev(const float* out, float* hprev, int32_t B, int32_t L, int32_t H, void* stream) {
  if (B <= 0 || L <= 0) return 0;
  long total = 2L * B * L * H;
  int grid = cdivi(total, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(bilstm_hprev_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, out, hprev, B, L, H);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_lstm_cell_fwd(const float* gates, const float* c_prev, float* h, float* c, float* act_save,
                                  int32_t B, int32_t H, void* stream) {
  if (B <= 0 || H <= 0) return 0;
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(cdivi((long)B * H, 256)), dim3(256), 0, (hipStream_t)stream,
                     gates, c_prev, h, c, act_save, B, H);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_lstm_cell_bwd(const float* act_save, const float* c_prev, const float* c, const float* dh,
                                  const float* dc, float* dgates, float* dc_prev, int32_t B, int32_t H,
                                  void* stream) {
  if (B <= 0 || H <= 0) return 0;
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(cdivi((long)B * H, 256)), dim3(256), 0, (hipStream_t)stream,
                     act_save, c_prev, c, dh, dc, dgates, dc_prev, B, H);
  DASA_CHECK_LAUNCH();
  return 0;
}

// 0 = automatic (persistent recurrence when eligible, else step kernels), 1 = step kernels only,
// 2 = persistent only (error when not eligible). DASA_LSTM_MODE sets the initial value.
static int g_lstm_mode = -1;
static int lstm_mode() {
  if (g_lstm_mode < 0) {
    const char* e = getenv("DASA_LSTM_MODE");
    g_lstm_mode = e ? atoi(e) : 0;
  }
  return g_lstm_mode;
}
extern "C" int dasa_bilstm_set_mode(int mode) {
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  g_lstm_mode = mode;
  return 0;
}

// Step path at B > 32 (configs[4]'s B = 256 rollout, or DASA_LSTM_MODE=1): W_hh of both directions is converted
// ONCE per call into the workspace — three bf16 planes [dir][plane][4H][H] for the bf16x6 fp32 GEMM, or one bf16
// copy [dir][4H][H] in bf16 mode (dasa_bilstm_fwd_bf16) — and each timestep's recurrent product of both
// directions is ONE batched GEMM (batch = direction) instead of two native fp32 launches.
static bool step_gemm_path(int B, int H) { return B > 32 && (lstm_mode() == 1 || !bilstm_persist_fwd_ok(B, H)); }
static long step_planes_floats(int H) { return 12L * H * H; }   // 2 dirs x 3 planes x 4H x H bf16

static int g_fwd_bf16 = 0;
extern "C" int dasa_bilstm_fwd_bf16(int32_t on) {
  const int prev = g_fwd_bf16;
  if (on >= 0) g_fwd_bf16 = on ? 1 : 0;
  return prev;
}

extern "C" int64_t dasa_bilstm_workspace(int32_t B, int32_t H) {
  const long base = 6L * B * H;
  long n = B <= 32 ? base : base + 8L * B * H;
  if (step_gemm_path(B, H)) n += step_planes_floats(H);
  return (int64_t)(n * sizeof(float));
}

extern "C" int dasa_bilstm_fwd(const float* xproj, const float* whh_fwd, const float* whh_bwd,
                               const int32_t* lengths, float* out, float* h_n, float* c_n, float* save_act,
                               float* save_c, int32_t B, int32_t L, int32_t H, float* ws, void* stream) {
  if (B <= 0 || L <= 0) return 0;
  if ((H % 256) || !ws || (((uintptr_t)whh_fwd | (uintptr_t)whh_bwd) & 15) ||
      (save_act != nullptr) != (save_c != nullptr))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long S = 2L * B * H;
  float* h0 = ws;
  float* h1 = ws + S;
  float* c = ws + 2 * S;
  float* rec = ws + 3 * S;
  hipLaunchKernelGGL(fill_kernel, dim3(cdivi(3 * S, 256)), dim3(256), 0, st, ws, 3 * S, 0.f);
  DASA_CHECK_LAUNCH();
  const int mode = lstm_mode();
  if (mode != 1 && bilstm_persist_fwd_ok(B, H)) {
    // ws: [0, 2S) = the [parity][dir][B][H] state hand-off, ws + 2S = zeroed barrier words
    const int rc = bilstm_persist_fwd(xproj, whh_fwd, whh_bwd, lengths, out, h_n, c_n, save_act, save_c, B, L, H,
                                      ws, reinterpret_cast<unsigned*>(ws + 2 * S), st);
    if (rc == 0 || mode == 2) return rc;
  } else if (mode == 2) {
    return (int)hipErrorInvalidValue;
  }
  SeqArgs a{xproj, whh_fwd, whh_bwd, lengths, out, h0, h1, c, save_act, save_c, nullptr, B, L, H};
  // the batched recurrent product of the step path (above): planes after the recurrent-gate buffer
  const bool bf = g_fwd_bf16 != 0, x6 = !bf && bilstm_fwd_x6_on();
  const bool planes = step_gemm_path(B, H) && (bf || x6) && H % 64 == 0;
  uint16_t* wp = reinterpret_cast<uint16_t*>(rec + 8L * B * H);
  const long WH = 4L * H * H;   // elements of one direction's W_hh
  if (planes) {
    int rc = 0;
    if (bf) {
      rc = dasa_f32_to_bf16(whh_fwd, wp, WH, stream);
      if (!rc) rc = dasa_f32_to_bf16(whh_bwd, wp + WH, WH, stream);
    } else {
      rc = dasa_f32_split3_bf16(whh_fwd, H, wp, 4 * H, H, stream);
      if (!rc) rc = dasa_f32_split3_bf16(whh_bwd, H, wp + 3 * WH, 4 * H, H, stream);
    }
    if (rc) return rc;
  }
  for (int s = 0; s < L; ++s) {
    a.hin = (s & 1) ? h1 : h0;
    a.hout = (s & 1) ? h0 : h1;
    if (B <= 32) {
      hipLaunchKernelGGL(bilstm_step_fused_kernel, dim3(H / kFwdUnits, 2), dim3(1024), 0, st, a, s);
      DASA_CHECK_LAUNCH();
    } else if (planes) {
      dasa_gemm_desc d{};
      d.M = B; d.N = 4 * H; d.K = H; d.batch = 2; d.opA = 0; d.opB = 1;
      d.A = a.hin; d.lda = H; d.strideA = (long)B * H;
      d.B = reinterpret_cast<const float*>(wp); d.ldb = H; d.strideB = bf ? WH : 3 * WH;
      d.C = rec; d.ldc = 4 * H; d.strideC = 4L * B * H;
      d.alpha = 1.f; d.beta = 0.f;
      const int rc = bf ? dasa_gemm_bf16_ex(&d, 0, stream) : dasa_gemm_f32x6_ws(&d, WH, nullptr, 0, stream);
      if (rc) return rc;
      a.rec = rec;
      hipLaunchKernelGGL(bilstm_step_cell_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, a, s);
      DASA_CHECK_LAUNCH();
    } else {
      for (int dir = 0; dir < 2; ++dir) {
        dasa_gemm_desc d{};
        d.M = B; d.N = 4 * H; d.K = H; d.batch = 1; d.opA = 0; d.opB = 1;
        d.A = a.hin + (long)dir * B * H; d.lda = H;
        d.B = dir ? whh_bwd : whh_fwd; d.ldb = H;
        d.C = rec + (long)dir * 4 * B * H; d.ldc = 4 * H;
        d.alpha = 1.f; d.beta = 0.f;
        int rc = dasa_gemm_f32(&d, nullptr, 0, stream);
        if (rc) return rc;
      }
      a.rec = rec;
      hipLaunchKernelGGL(bilstm_step_cell_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, a, s);
      DASA_CHECK_LAUNCH();
    }
  }
  const float* hfin = (L & 1) ? h1 : h0;
  if (h_n) {
    hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, hfin, h_n, S);
    DASA_CHECK_LAUNCH();
  }
  if (c_n) {
    hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, (const float*)c, c_n, S);
    DASA_CHECK_LAUNCH();
  }
  return 0;
}

// Large-batch BPTT: the per-timestep recurrent product of both directions as ONE batched NT GEMM
// (rec[dir] = dgates_prev[dir] . W_hh[dir], with W_hh^T staged K-contiguous once per call), so it
// takes the 64-deep K / stream-K kernels (gemm.hip) with its own zero-counter workspace.
static dasa_gemm_desc bptt_rec_desc(int B, int L, int H) {
  dasa_gemm_desc d{};
  d.M = B; d.N = H; d.K = 4 * H; d.batch = 2; d.opA = 0; d.opB = 1;
  d.lda = (long)L * 2 * 4 * H; d.ldb = 4 * H; d.ldc = H;
  d.strideB = 4L * H * H; d.strideC = (long)B * H;
  d.alpha = 1.f; d.beta = 0.f;
  return d;
}
// The recurrent product on the bf16x6 fp32 GEMM (dasa_gemm_f32x6_ws: fp32-accurate, 1.5-2x the native
// fp32 MFMA kernels on these few-tile long-K shapes through its split-K form) with W_hh^T pre-split into
// three bf16 planes [3][2][H][4H] once per call. DASA_BPTT_X6=0 (or DASA_GEMM_EMU=0) keeps dasa_gemm_f32.
static int g_bptt_x6 = -1;
static bool bptt_x6() {
  if (g_bptt_x6 < 0) {
    const char* e = getenv("DASA_BPTT_X6");
    const char* g = getenv("DASA_GEMM_EMU");
    g_bptt_x6 = !(e && e[0] == '0') && !(g && g[0] == '0');
  }
  return g_bptt_x6 != 0;
}
extern "C" int dasa_bilstm_bptt_x6(int32_t on) {
  const int prev = bptt_x6() ? 1 : 0;
  if (on >= 0) g_bptt_x6 = on ? 1 : 0;
  return prev;
}
static long bptt_gemm_ws_floats(int B, int L, int H) {
  dasa_gemm_desc d = bptt_rec_desc(B, L, H);
  const int64_t f = dasa_gemm_f32_workspace(&d), x = dasa_gemm_f32x6_workspace(&d);
  return ((f > x ? f : x) + 15) / 4 + 4;
}

extern "C" int64_t dasa_bilstm_bwd_workspace(int32_t B, int32_t H) {
  if (B > 32)   // carries + rec, W_hh^T of both directions (fp32 + three bf16 planes), GEMM workspace
    return (int64_t)((6L * B * H + 8L * H * H + 12L * H * H + 16 + bptt_gemm_ws_floats(B, 1, H)) * sizeof(float));
  return (int64_t)((4L * B * H + 8L * H * H) * sizeof(float));
}

extern "C" int dasa_bilstm_bwd(const float* whh_fwd, const float* whh_bwd, const int32_t* lengths,
                               const float* save_act, const float* save_c, const float* dout, const float* dh_n,
                               const float* dc_n, float* dgates, int32_t B, int32_t L, int32_t H, float* ws,
                               void* stream) {
  if (B <= 0 || L <= 0) return 0;
  if ((H % 64) || !ws || !save_act || !save_c || !dout || ((uintptr_t)ws & 15))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long S = 2L * B * H;
  if (B > 32) {
    // Large batch (e.g. every rollout step's sequences of one optimizer step, batched): per timestep
    // one MFMA GEMM per direction for rec = dgates_prev . W_hh, then the cell kernel.
    float* dh = ws;
    float* dc = ws + S;
    float* rec = ws + 2 * S;
    if (dh_n) hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dh_n, dh, S);
    else hipLaunchKernelGGL(fill_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dh, S, 0.f);
    DASA_CHECK_LAUNCH();
    if (dc_n) hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dc_n, dc, S);
    else hipLaunchKernelGGL(fill_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dc, S, 0.f);
    DASA_CHECK_LAUNCH();
    float* wt = rec + S;
    wt += (16 - ((uintptr_t)wt & 15) / 4) % 4;            // 16-B aligned W_hh^T [2][H][4H]
    uint16_t* planes = reinterpret_cast<uint16_t*>(wt + 8L * H * H);   // [3][2][H][4H] bf16, 16-B aligned
    float* gws = wt + 8L * H * H + 12L * H * H;
    gws += (16 - ((uintptr_t)gws & 15) / 4) % 4;
    const long gws_floats = bptt_gemm_ws_floats(B, L, H) - 4;
    hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, st, gws, 16384L, 0.f);   // GEMM arrival counters
    DASA_CHECK_LAUNCH();
    hipLaunchKernelGGL(transpose_kernel, dim3(H / 32, 4 * H / 32), dim3(256), 0, st, whh_fwd, wt, 4 * H, H);
    DASA_CHECK_LAUNCH();
    hipLaunchKernelGGL(transpose_kernel, dim3(H / 32, 4 * H / 32), dim3(256), 0, st, whh_bwd, wt + 4L * H * H,
                       4 * H, H);
    DASA_CHECK_LAUNCH();
    const bool x6 = bptt_x6();
    if (x6) {
      const int rc = dasa_f32_split3_bf16(wt, 4L * H, planes, 2 * H, 4 * H, stream);
      if (rc) return rc;
    }
    BpttArgs a{nullptr, nullptr, lengths, save_act, save_c, dout, dgates, dh, dc, B, L, H};
    for (int s = 0; s < L; ++s) {
      if (s > 0) {   // both directions in one launch: dir 0 reads step t+1 = L-s, dir 1 step t-1 = s-1
        dasa_gemm_desc d = bptt_rec_desc(B, L, H);
        const long a0 = ((long)(L - s) * 2 + 0) * 4 * H, a1 = ((long)(s - 1) * 2 + 1) * 4 * H;
        d.A = dgates + a0;
        d.strideA = a1 - a0;
        d.C = rec;
        int rc;
        if (x6) {
          d.B = reinterpret_cast<const float*>(planes);   // hi plane; mid / lo 8H^2 on, direction 1 at +4H^2
          rc = dasa_gemm_f32x6_ws(&d, 8L * H * H, gws, gws_floats * (int64_t)sizeof(float), stream);
        } else {
          d.B = wt;
          rc = dasa_gemm_f32(&d, gws, gws_floats * (int64_t)sizeof(float), stream);
        }
        if (rc) return rc;
      }
      hipLaunchKernelGGL(bilstm_bptt_cell_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, a, (const float*)rec, s);
      DASA_CHECK_LAUNCH();
    }
    return 0;
  }
  const int mode = lstm_mode();
  if (mode != 1 && bilstm_persist_ok(B, H)) {
    hipLaunchKernelGGL(fill_kernel, dim3(2), dim3(256), 0, st, ws, 512L, 0.f);   // barrier words (sharded)
    DASA_CHECK_LAUNCH();
    const int rc = bilstm_persist_bwd(whh_fwd, whh_bwd, lengths, save_act, save_c, dout, dh_n, dc_n, dgates, B, L,
                                      H, reinterpret_cast<unsigned*>(ws), st);
    if (rc == 0 || mode == 2) return rc;
  } else if (mode == 2) {
    return (int)hipErrorInvalidValue;
  }
  float* dh = ws;
  float* dc = ws + S;
  float* wt0 = ws + 2 * S;
  wt0 += (16 - ((uintptr_t)wt0 & 15) / 4) % 4;   // 16-B align (ws budget has slack: 8H^2 >> 3)
  float* wt1 = wt0 + 4L * H * H;
  if (dh_n) hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dh_n, dh, S);
  else hipLaunchKernelGGL(fill_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dh, S, 0.f);
  DASA_CHECK_LAUNCH();
  if (dc_n) hipLaunchKernelGGL(copy_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dc_n, dc, S);
  else hipLaunchKernelGGL(fill_kernel, dim3(cdivi(S, 256)), dim3(256), 0, st, dc, S, 0.f);
  DASA_CHECK_LAUNCH();
  hipLaunchKernelGGL(transpose_kernel, dim3(H / 32, 4 * H / 32), dim3(256), 0, st, whh_fwd, wt0, 4 * H, H);
  DASA_CHECK_LAUNCH();
  hipLaunchKernelGGL(transpose_kernel, dim3(H / 32, 4 * H / 32), dim3(256), 0, st, whh_bwd, wt1, 4 * H, H);
  DASA_CHECK_LAUNCH();
  BpttArgs a{wt0, wt1, lengths, save_act, save_c, dout, dgates, dh, dc, B, L, H};
  for (int s = 0; s < L; ++s) {
    hipLaunchKernelGGL(bilstm_bptt_step_kernel, dim3(H / kBwdUnits, 2), dim3(1024), 0, st, a, s);
    DASA_CHECK_LAUNCH();
  }
  return 0;
}
