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
  hipLaunchKernelGGL(ada_gate_fwd_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, s,
                     (long)lds, f, (long)ldf, noise, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_ada_gate_bwd(const float* dout, int64_t lddo, const float* s, int64_t lds, const float* f,
                                 int64_t ldf, const float* noise, float* dz, int64_t ldz, int32_t rows, int32_t cols,
                                 void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
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
  hipLaunchKernelGGL(add2d_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, a, (long)lda,
                     b, (long)ldb, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_colscale(const float* x, int64_t ldx, const float* scale, float* out, int64_t ldo, int32_t rows,
                             int32_t cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  hipLaunchKernelGGL(colscale_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, x,
                     (long)ldx, scale, out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_copy2d(const float* x, int64_t ldx, float* out, int64_t ldo, int32_t rows, int32_t cols,
                           void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  hipLaunchKernelGGL(copy2d_kernel, dim3(grid_for((long)rows * cols)), dim3(256), 0, (hipStream_t)stream, x, (long)ldx,
                     out, (long)ldo, rows, cols);
  DASA_CHECK_LAUNCH();
  return 0;
}
