// Minimal reproducer for the r05 row-split finding: do packed-FP32 VALU results
// (v_pk_fma_f32) come back wrong while a bf16x6 form-20 GEMM workgroup starts on the same CU?
//
// The kernel has the geometry of the r04/r05 row-split SoftDot forward it stands in for (attn_fwd_kernel at
// B = 20, N = 80, D = 2048: one 512-thread workgroup per (batch row, 16-row block), each thread the dot
// products of 16 rows with its float4 of q). Every row pair (2k, 2k+1) is accumulated TWICE in the same k
// order from the same registers: once as a packed chain (v_pk_fma_f32, row 2k in the low half, 2k+1 in the
// high half — the instruction the compiler emitted for the r04 kernel) and once as two scalar chains
// (v_fma_f32). Both are single-rounding fmas in the same order, so the two must agree bit for bit; the host
// also compares each against the quiet run's bits (no side GEMM), which tells which of the two went wrong.
// Both forms are inline asm so no compiler flag (the library builds without packed FP32) changes them.
// Writes only through vector stores / vector atomics. Built by tools/pk_fp32_repro.py (hipcc, gfx950).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) {
  f2 d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ float sc_fma(float a, float b, float c) {
  float d;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

__device__ __forceinline__ float sc_mul(float a, float b) {
  float d;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

// the row-split kernel's dot (attn.hip dot4): x.w*q.w first, then fmas of z, y, x — written in plain C so that
// this file's default hipcc build (SLP on) packs it exactly as it packed the r04 kernel (v_pk_mul_f32, then
// v_pk_fma_f32 with op_sel / op_sel_hi broadcasts of q)
__device__ __forceinline__ float dot4c(const float4 a, const float4 b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}
__device__ __forceinline__ float dot4s(const float4 a, const float4 b) {   // the same order, scalar asm
  return sc_fma(a.x, b.x, sc_fma(a.y, b.y, sc_fma(a.z, b.z, sc_mul(a.w, b.w))));
}

// x [B][N][D], q [B][D]; outputs per (call slot): pk / sc [B][nblk][16][T] (T = D / 4 threads per workgroup),
// and bad[0] += number of (thread, row) whose packed and scalar results differ, bad[1 + lane] per lane.
// MODE 0: the packed chains as inline asm (no op_sel); MODE 1: compiler-packed dot4 over rows loaded the way
// the r05 row-split kernel loads them (one buffer_load_dwordx4 per row, shared offset VGPR, row offset in an
// SGPR) — the r04/r05 instruction stream itself.
template <int MODE>
__global__ __launch_bounds__(1024) void pk_rows_kernel(const float* __restrict__ x, const float* __restrict__ q,
                                                       float* __restrict__ pk, float* __restrict__ sc,
                                                       unsigned* __restrict__ bad, int N, int D) {
  const int T = D / 4, t = threadIdx.x, b = blockIdx.y, blk = blockIdx.x, lane = t & 63;
  const int nblk = gridDim.x;
  const float4 qv = reinterpret_cast<const float4*>(q + (long)b * D)[t];
  float4 xv[16];
  if (MODE == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = min(blk * 16 + r, N - 1);
      xv[r] = reinterpret_cast<const float4*>(x + ((long)b * N + row) * D)[t];
    }
  } else {
    const float* rows = x + ((long)b * N + blk * 16) * D;
    const int nr = min(16, N - blk * 16);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows), 0, 0x7fffffff,
                                                                        0x00020000);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const auto u = __builtin_amdgcn_raw_buffer_load_b128(rr, t * 16, __builtin_amdgcn_readfirstlane(min(r, nr - 1) * D * 4), 0);
      xv[r] = __builtin_bit_cast(float4, u);
    }
  }
  float vp[16], vs[16];
  if (MODE == 0) {
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f2 acc = {0.f, 0.f};
      acc = pk_fma(f2{xv[r].x, xv[r + 1].x}, f2{qv.x, qv.x}, acc);
      acc = pk_fma(f2{xv[r].y, xv[r + 1].y}, f2{qv.y, qv.y}, acc);
      acc = pk_fma(f2{xv[r].z, xv[r + 1].z}, f2{qv.z, qv.z}, acc);
      acc = pk_fma(f2{xv[r].w, xv[r + 1].w}, f2{qv.w, qv.w}, acc);
      vp[r] = acc.x;
      vp[r + 1] = acc.y;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float s = 0.f;
        s = sc_fma(xv[r + h].x, qv.x, s);
        s = sc_fma(xv[r + h].y, qv.y, s);
        s = sc_fma(xv[r + h].z, qv.z, s);
        s = sc_fma(xv[r + h].w, qv.w, s);
        vs[r + h] = s;
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) vp[r] = dot4c(xv[r], qv);
#pragma unroll
    for (int r = 0; r < 16; ++r) vs[r] = dot4s(xv[r], qv);
  }
  const long base = ((long)b * nblk + blk) * 16 * T;
  unsigned nbad = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    pk[base + (long)r * T + t] = vp[r];
    sc[base + (long)r * T + t] = vs[r];
    nbad += __float_as_uint(vp[r]) != __float_as_uint(vs[r]);
  }
  if (nbad) {
    atomicAdd(bad, nbad);
    atomicAdd(bad + 1 + lane, nbad);
  }
}

extern "C" int pk_rows_launch(const float* x, const float* q, float* pk, float* sc, unsigned* bad, int B, int N,
                              int D, int mode, void* stream) {
  if (B <= 0 || N <= 0 || D != 2048 || mode < 0 || mode > 1) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((N + 15) / 16), (unsigned)B);
  if (mode == 0)
    hipLaunchKernelGGL(pk_rows_kernel<0>, grid, dim3(D / 4), 0, (hipStream_t)stream, x, q, pk, sc, bad, N, D);
  else
    hipLaunchKernelGGL(pk_rows_kernel<1>, grid, dim3(D / 4), 0, (hipStream_t)stream, x, q, pk, sc, bad, N, D);
  return (int)hipGetLastError();
}
