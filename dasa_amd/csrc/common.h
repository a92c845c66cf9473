// Shared device helpers for the DASA gfx950 kernels.
// Wave = 64 lanes on CDNA4; every reduction below is written for 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DASA_WAVE 64

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define DASA_CHECK_LAUNCH()                                   \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return (int)_e;                     \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 64*NW; `red` must hold NW floats.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// Exact-erf GELU, matching vilmodel.py:125-131 (x * 0.5 * (1 + erf(x / sqrt(2)))).
__device__ __forceinline__ float gelu_erf(float x) { return x * 0.5f * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Counter-based dropout RNG: stateless, so a kernel can regenerate the same keep-mask in its backward
// from (seed, index). Two rounds of a 32-bit avalanche mixer (lowbias32) over the index halves, keyed by
// the seed halves: 32-bit multiplies only (r05: the splitmix64 finaliser's 64-bit multiplies were ≈15 of
// the language MHA's ≈80 µs per launch; this form 39.0-39.5 -> 37.4-38.4 µs, profiles/r05/z/).
__device__ __forceinline__ uint32_t dasa_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float dasa_uniform(uint64_t seed, uint64_t idx) {
  uint32_t h = dasa_mix32((uint32_t)idx ^ (uint32_t)seed);
  h = dasa_mix32(h ^ (uint32_t)(seed >> 32) ^ ((uint32_t)(idx >> 32) * 0x9E3779B9U));
  return (float)(h >> 8) * (1.0f / 16777216.0f);  // [0,1)
}
// Dropout seed of one launch: the host seed, re-keyed by the 64-bit value at `src` when the launch
// was recorded with a device seed source (dasa_set_seed_source, used around hipGraph capture), so
// every replay of a captured graph draws fresh masks after dasa_seed_bump advanced the value.
__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t* src) {
  return src ? seed ^ (*src * 0xD1B54A32D192ED03ull) : seed;
}
// Host side: the seed source recorded into dropout launches (nullptr = plain host seeds).
__attribute__((visibility("hidden"))) const uint64_t* dasa_seed_src_host();
// Host side: the library's device error word (dasa_set_error_word; bits: 1 bi-LSTM forward, 2 bi-LSTM
// BPTT, 4 attention group barrier) and the forced-timeout test hook (dasa_persist_force_timeout).
__attribute__((visibility("hidden"))) unsigned* dasa_err_word_host();
__attribute__((visibility("hidden"))) int dasa_force_timeout_host();

// ---- debug build (dasa_amd/build.py --debug: -DDASA_DEBUG, host ASan + UBSan) ----------------------
// DASA_DCHECK(cond, bit): a device-side check of an input invariant the kernel relies on (an index in
// range, a launch shape the kernel assumes). In the debug library a failed check ORs `bit` into the
// library's error word (dasa_set_error_word; the host raises at its next ops.check_device_errors()) and
// the thread leaves the kernel — no trap, no fault. `cond` must be uniform over a workgroup wherever the
// kernel has a barrier after the check. Compiled out of the release library. Bits: 16 policy head
// target / forced action, 32 gather index, 64 sequence length, 128 attention launch shape.
#ifdef DASA_DEBUG
namespace {
__device__ unsigned* g_dbg_err = nullptr;   // per translation unit, set by dasa_set_error_word
}
__attribute__((visibility("hidden"))) void dasa_dbg_register(void (*setter)(unsigned*));
namespace {
inline void dasa_dbg_set_err(unsigned* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_err), &p, sizeof(p)); }
[[maybe_unused]] const int dasa_dbg_registered = (dasa_dbg_register(dasa_dbg_set_err), 0);
}
#define DASA_DCHECK(cond, bit)                          \
  do {                                                  \
    if (!(cond)) {                                      \
      unsigned* _w = g_dbg_err;                         \
      if (_w) atomicOr(_w, (unsigned)(bit));            \
      return;                                           \
    }                                                   \
  } while (0)
#else
#define DASA_DCHECK(cond, bit) \
  do {                         \
  } while (0)
#endif

__device__ __forceinline__ float dasa_dropout_scale(float p, uint64_t seed, uint64_t idx) {
  if (p <= 0.f) return 1.f;
  return dasa_uniform(seed, idx) >= p ? 1.f / (1.f - p) : 0.f;
}
