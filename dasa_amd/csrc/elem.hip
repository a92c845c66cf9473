// Elementwise kernels of the training path (backward of fused GEMM epilogues, DGAdaChannel gate).
// All are HBM-bound streaming kernels over [rows][cols] blocks with arbitrary row strides, so they
// can address the RGB part [..., :2048] of a 2176-stride feature block in place.
#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

inline int cdivi(long a, long b) { return (int)((a + b - 1) / b); }
inline int grid_for(long n) {
  int g = cdivi(n, 256);
  return g > 16384 ? 16384 : (g < 1 ? 1 : g);
}

// Vectorised 2-D streaming: thread = one float4 column quad of RPT consecutive rows; every input
// quad of the RPT rows is loaded (rows clamped) before any result is stored, so each thread keeps
// RPT x NIN 16-B loads in flight. A per-column vector (noise, scale) is an input with ld = 0.
// Used whenever cols % 4 == 0 and every base / ld is 16-B aligned (the policy's feature blocks).
template <int NIN>
struct Ew4Args {
  const float* in[NIN];
  long ld[NIN];
  float* out;
  long ldo;
  int rows, cols4, cols;
  int flag;   // op-specific (the gate's noise present); ops carry no state of their own (a stateful
              // functor argument is promoted to per-thread LDS by hipcc and costs 5-10x)
  float p;
  uint64_t seed;
  const uint64_t* seed_src;   // eff_seed(): device seed source of a graph-captured launch, or null
};

__device__ __forceinline__ float4 mul4(const float4 a, const float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}

template <int NIN, int RPT, class Op>
__global__ __launch_bounds__(256) void ew4_kernel(Ew4Args<NIN> a, Op op) {
  const int c4 = blockIdx.x * 256 + threadIdx.x;
  if (c4 >= a.cols4) return;
  const int r0 = blockIdx.y * RPT;
  float4 v[RPT][NIN];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const long r = min(r0 + k, a.rows - 1);
#pragma unroll
    for (int i = 0; i < NIN; ++i) v[k][i] = reinterpret_cast<const float4*>(a.in[i] + r * a.ld[i])[c4];
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = r0 + k;
    if (r < a.rows) reinterpret_cast<float4*>(a.out + (long)r * a.ldo)[c4] = op(v[k], r, c4, a);
  }
}

struct AdaFwdOp {   // out = s * f (* noise)
  template <class A> __device__ float4 operator()(const float4 (&v)[3], int, int, const A& a) const {
    const float4 o = mul4(v[0], v[1]);
    return a.flag ? mul4(o, v[2]) : o;
  }
};
struct AdaBwdOp {   // dz = dout * f * s * (1 - s) (* noise)
  template <class A> __device__ float4 operator()(const float4 (&v)[4], int, int, const A& a) const {
    const float4 s = v[1];
    float4 o = mul4(mul4(v[0], v[2]), make_float4(s.x * (1.f - s.x), s.y * (1.f - s.y), s.z * (1.f - s.z),
                                                   s.w * (1.f - s.w)));
    return a.flag ? mul4(o, v[3]) : o;
  }
};
struct MulOp {
  template <class A> __device__ float4 operator()(const float4 (&v)[2], int, int, const A&) const { return mul4(v[0], v[1]); }
};
struct AddOp {
  template <class A> __device__ float4 operator()(const float4 (&v)[2], int, int, const A&) const {
    return make_float4(v[0].x + v[1].x, v[0].y + v[1].y, v[0].z + v[1].z, v[0].w + v[1].w);
  }
};
struct CopyOp {
  template <class A> __device__ float4 operator()(const float4 (&v)[1], int, int, const A&) const { return v[0]; }
};
struct DropOp {     // same (seed, logical index r * cols + c) mask as the scalar dropout kernel
  template <class A> __device__ float4 operator()(const float4 (&v)[1], int r, int c4, const A& a) const {
    const uint64_t i = (uint64_t)r * a.cols + 4 * c4;
    const uint64_t sd = eff_seed(a.seed, a.seed_src);
    return make_float4(v[0].x * dasa_dropout_scale(a.p, sd, i), v[0].y * dasa_dropout_scale(a.p, sd, i + 1),
                       v[0].z * dasa_dropout_scale(a.p, sd, i + 2), v[0].w * dasa_dropout_scale(a.p, sd, i + 3));
  }
};

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int NIN, class Op>
bool try_ew4(const float* const (&in)[NIN], const long (&ld)[NIN], float* out, long ldo, int rows, int cols, Op op,
             hipStream_t st, float p = 0.f, uint64_t seed = 0, int flag = 0) {
  if (cols & 3 || !al16(out) || (ldo & 3)) return false;
  for (int i = 0; i < NIN; ++i)
    if (!al16(in[i]) || (ld[i] & 3)) return false;
  Ew4Args<NIN> a;
  for (int i = 0; i < NIN; ++i) { a.in[i] = in[i]; a.ld[i] = ld[i]; }
  a.out = out; a.ldo = ldo; a.rows = rows; a.cols4 = cols / 4; a.cols = cols; a.p = p; a.seed = seed;
  a.seed_src = p > 0.f ? dasa_seed_src_host() : nullptr;
  a.flag = flag;
  // 4 rows per thread once there are enough rows to fill the chip several times over; below that
  // one row per thread (more waves in flight beats more loads per wave there)
  const int rpt = (long)rows * a.cols4 >= (long)256 * 256 * 16 ? 4 : 1;
  const dim3 grid((a.cols4 + 255) / 256, (rows + rpt - 1) / rpt);
  if (grid.y > 65535) return false;
  const dim3 block(a.cols4 < 256 ? ((a.cols4 + 63) / 64) * 64 : 256);
  if (rpt == 4) hipLaunchKernelGGL((ew4_kernel<NIN, 4, Op>), grid, block, 0, st, a, op);
  else hipLaunchKernelGGL((ew4_kernel<NIN, 1, Op>), grid, block, 0, st, a, op);
  return true;
}

// DGAdaChannel (agent_dg.py:1537-1547, a_type sigmoid, ab_type a): out = s * f * noise[c]
__global__ void ada_gate_fwd_kernel(const float* s, long lds, const float* f, long ldf, const float* noise, float* out,
                                    long ldo, int rows, int cols) {
  const long total = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    float v = s[r * lds + c] * f[r * ldf + c];
    if (noise) v *= noise[c];
    out[r * ldo + c] = v;
  }
}

// dz = dout * f * noise * s * (1 - s)   (grad of the a_fc pre-activation)
__global__ void ada_gate_bwd_kernel(const float* dout, long lddo, const float* s, long lds, const float* f, long ldf,
                                    const float* noise, float* dz, long ldz, int rows, int cols) {
  const long total = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    const float sv = s[r * lds + c];
    float v = dout[r * lddo + c] * f[r * ldf + c] * sv * (1.f - sv);
    if (noise) v *= noise[c];
    dz[r * ldz + c] = v;
  }
}

// dx = dy * act'(.) given the activation OUTPUT y (relu/tanh/sigmoid) or the INPUT x (gelu).
__global__ void act_bwd_kernel(const float* yx, const float* dy, float* dx, long n, int act) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = yx[i], g = dy[i];
    float d;
    switch (act) {
      case DASA_ACT_RELU: d = v > 0.f ? g : 0.f; break;
      case DASA_ACT_TANH: d = g * (1.f - v * v); break;
      case DASA_ACT_SIGMOID: d = g * v * (1.f - v); break;
      case DASA_ACT_GELU: d = g * gelu_erf_grad(v); break;
      default: d = g;
    }
    dx[i] = d;
  }
}

__global__ void act_fwd_kernel(const float* x, float* y, long n, int act) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = x[i];
    float o;
    switch (act) {
      case DASA_ACT_RELU: o = fmaxf(v, 0.f); break;
      case DASA_ACT_TANH: o = tanhf(v); break;
      case DASA_ACT_SIGMOID: o = sigmoidf_(v); break;
      case DASA_ACT_GELU: o = gelu_erf(v); break;
      default: o = v;
    }
    y[i] = o;
  }
}

// out[r][c] = a[r][c] + b[r][c] (strided; used to merge split-column gradients)
__global__ void add2d_kernel(const float* a, long lda, const float* b, long ldb, float* out, long ldo, int rows,
                             int cols) {
  const long total = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[r * ldo + c] = a[r * lda + c] + b[r * ldb + c];
  }
}

// out[r][c] = x[r][c] * scale[c] (the shared env-drop mask, agent_dg.py:731-736, 780-785)
__global__ void colscale_kernel(const float* x, long ldx, const float* scale, float* out, long ldo, int rows, int cols) {
  const long total = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[r * ldo + c] = x[r * ldx + c] * scale[c];
  }
}

// out[r][c] = x[r][c] (strided copy; the angle columns of the AdaIN output)
__global__ void copy2d_kernel(const float* x, long ldx, float* out, long ldo, int rows, int cols) {
  const long total = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[r * ldo + c] = x[r * ldx + c];
  }
}

// Observation gather (agent_dg.py:286-323 on a device-resident feature store): out row r =
// [ta[ia[r]] (Fa wide, zeros if ia[r] < 0) | tb[ib[r]] (Fb wide, zeros if ib[r] < 0)]. One wave per row.
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ ta, const int* __restrict__ ia,
                                                          int Fa, const float* __restrict__ tb,
                                                          const int* __restrict__ ib, int Fb, float* __restrict__ out,
                                                          int R) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const int a = ia[r], b = ib ? ib[r] : -1;
  DASA_DCHECK(a >= -1 && b >= -1, 32);
  float4* o = reinterpret_cast<float4*>(out + (long)r * (Fa + Fb));
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* pa = a >= 0 ? reinterpret_cast<const float4*>(ta + (long)a * Fa) : nullptr;
  for (int c = lane; c < Fa / 4; c += 64) o[c] = pa ? pa[c] : z;
  const float4* pb = b >= 0 ? reinterpret_cast<const float4*>(tb + (long)b * Fb) : nullptr;
  for (int c = lane; c < Fb / 4; c += 64) o[Fa / 4 + c] = pb ? pb[c] : z;
}

}  // namespace

extern "C" int dasa_gather_rows(const float* ta, const int32_t* ia, int32_t Fa, const float* tb, const int32_t* ib,
                                int32_t Fb, float* out, int32_t R, void* stream) {
  if (R <= 0) return 0;
  if ((Fa & 3) || (Fb & 3)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(cdivi(R, 4)), dim3(256), 0, (hipStream_t)stream, ta, ia, Fa, tb, ib, Fb,
                     out, R);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_ada_gate_fwd(const float* s, int64_t lds, const float* f, int64_t ldf, const float* noise,
                                 float* out, int64_t ldo, int32_t rows, int32_t cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const float* in[3] = {s, f, noise ? noise : s};
    const long ld[3] = {(long)lds, (long)ldf, 0};
    if (try_ew4<3>(in, ld, out, (long)ldo, rows, cols, AdaFwdOp{}, (hipStream_t)stream, 0.f, 0, noise != nullptr)) {
      DASA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL(ada_gate_fwd_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, s,
                     (long)lds, f, (long)ldf, noise, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_ada_gate_bwd(const float* dout, int64_t lddo, const float* s, int64_t lds, const float* f,
                                 int64_t ldf, const float* noise, float* dz, int64_t ldz, int32_t rows, int32_t cols,
                                 void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const float* in[4] = {dout, s, f, noise ? noise : s};
    const long ld[4] = {(long)lddo, (long)lds, (long)ldf, 0};
    if (try_ew4<4>(in, ld, dz, (long)ldz, rows, cols, AdaBwdOp{}, (hipStream_t)stream, 0.f, 0, noise != nullptr)) {
      DASA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL(ada_gate_bwd_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, dout,
                     (long)lddo, s, (long)lds, f, (long)ldf, noise, dz, (long)ldz, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_act_bwd(const float* y_or_x, const float* dy, float* dx, int64_t n, int32_t act, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, y_or_x, dy, dx, (long)n,
                     act);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_act_fwd(const float* x, float* y, int64_t n, int32_t act, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, (long)n, act);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_add2d(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int64_t ldo,
                          int32_t rows, int32_t cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const float* in[2] = {a, b};
    const long ld[2] = {(long)lda, (long)ldb};
    if (try_ew4<2>(in, ld, out, (long)ldo, rows, cols, AddOp{}, (hipStream_t)stream)) {
      DASA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL(add2d_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, a, (long)lda,
                     b, (long)ldb, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_colscale(const float* x, int64_t ldx, const float* scale, float* out, int64_t ldo, int32_t rows,
                             int32_t cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const float* in[2] = {x, scale};
    const long ld[2] = {(long)ldx, 0};
    if (try_ew4<2>(in, ld, out, (long)ldo, rows, cols, MulOp{}, (hipStream_t)stream)) {
      DASA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL(colscale_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, x,
                     (long)ldx, scale, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_copy2d(const float* x, int64_t ldx, float* out, int64_t ldo, int32_t rows, int32_t cols,
                           void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const float* in[1] = {x};
    const long ld[1] = {(long)ldx};
    if (try_ew4<1>(in, ld, out, (long)ldo, rows, cols, CopyOp{}, (hipStream_t)stream)) {
      DASA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL(copy2d_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, x, (long)ldx,
                     out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

// Vector path of dasa_dropout_fwd (bert.hip): false when the block is not float4-aligned.
__attribute__((visibility("hidden"))) bool dasa_dropout_vec(const float* x, long ldx, float* y, long ldy, int rows, int cols, float p, uint64_t seed,
                      hipStream_t st) {
  const float* in[1] = {x};
  const long ld[1] = {ldx};
  return try_ew4<1>(in, ld, y, ldy, rows, cols, DropOp{}, st, p, seed);
}

// ---- device seed source for graph-captured dropout (include/dasa_hip.h) ----------------------------
namespace {
const uint64_t* g_seed_src = nullptr;
__global__ void seed_bump_kernel(uint64_t* ctr) {
  if (threadIdx.x == 0) ctr[0] += 1;
}
}  // namespace

__attribute__((visibility("hidden"))) const uint64_t* dasa_seed_src_host() { return g_seed_src; }

extern "C" int dasa_set_seed_source(const uint64_t* dev_counter) {
  g_seed_src = dev_counter;
  return 0;
}

extern "C" int dasa_seed_bump(uint64_t* dev_counter, void* stream) {
  if (!dev_counter) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seed_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_counter);
  DASA_CHECK_LAUNCH();
  return 0;
}
