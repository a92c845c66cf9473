// Sustained fp32 MFMA ceiling probe: every wave runs a long chain of v_mfma_f32_32x32x2_f32 on
// 4 independent accumulators (register operands only), so the measured rate is the clock the chip
// holds under a full-chip fp32 MFMA load, not a memory effect.
#include <hip/hip_runtime.h>
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float seed) {
  floatx16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
  float x = seed * (threadIdx.x + 1), y = seed * (blockIdx.x + 1);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, y, a3, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += a0[r] + a1[r] + a2[r] + a3[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

extern "C" int mfma_peak_launch(float* out, int blocks, int iters, void* stream) {
  hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1e-3f);
  return (int)hipGetLastError();
}
