// Batched strided copies: the static-buffer traffic around every replayed graph (a captured training
// step's inputs copied into its padded static buffers, its outputs copied out; graph.py) as ONE launch
// instead of one hipMemcpyAsync / blit kernel per tensor. r05 trace of the cfg2 iteration: 2214
// `__amd_rocclr_copyBuffer` launches (≈32 per decision step, 12.7 ms of 5.7-µs blits) and the host
// gaps between them were the largest idle item left after the backward capture.
//
// A segment copies a [n0][n1][bytes] block between two byte-strided layouts (every tensor the graphs
// exchange is at most 3-D with a contiguous innermost dimension). Workgroup (x, y = segment): the
// segment's 16-B (or, for unaligned segments, 4-B) units split over gridDim.x workgroups of 256
// threads, grid-stride. Pure data movement, HBM-bound.
#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

struct CopyArgs {
  dasa_copy_seg seg[DASA_COPY_MAX_SEGS];
  int n;
};

template <typename U>
__device__ __forceinline__ void copy_seg(const dasa_copy_seg& s, long first, long step) {
  const long per_row = s.row_bytes / (long)sizeof(U);
  const long total = (long)s.n0 * s.n1 * per_row;
  const char* src = reinterpret_cast<const char*>(s.src);
  char* dst = reinterpret_cast<char*>(s.dst);
  for (long u = first; u < total; u += step) {
    const long r = u / per_row, e = u - r * per_row;
    const long i0 = r / s.n1, i1 = r - i0 * s.n1;
    const U v = *reinterpret_cast<const U*>(src + i0 * s.src_s0 + i1 * s.src_s1 + e * (long)sizeof(U));
    *reinterpret_cast<U*>(dst + i0 * s.dst_s0 + i1 * s.dst_s1 + e * (long)sizeof(U)) = v;
  }
}

__global__ __launch_bounds__(256) void copy_segments_kernel(CopyArgs a) {
  const int k = blockIdx.y;
  if (k >= a.n) return;
  const dasa_copy_seg& s = a.seg[k];
  const long first = (long)blockIdx.x * 256 + threadIdx.x, step = (long)gridDim.x * 256;
  const bool v16 = ((s.row_bytes | s.src_s0 | s.src_s1 | s.dst_s0 | s.dst_s1) & 15) == 0 &&
                   (((uintptr_t)s.src | (uintptr_t)s.dst) & 15) == 0;
  if (v16) {
    copy_seg<uint4>(s, first, step);
  } else if (((s.row_bytes | s.src_s0 | s.src_s1 | s.dst_s0 | s.dst_s1) & 3) == 0 &&
             (((uintptr_t)s.src | (uintptr_t)s.dst) & 3) == 0) {
    copy_seg<unsigned>(s, first, step);
  } else {
    copy_seg<unsigned char>(s, first, step);
  }
}

}  // namespace

extern "C" int dasa_copy_segments(const dasa_copy_seg* segs, int32_t n, void* stream) {
  if (n < 0 || n > DASA_COPY_MAX_SEGS || (n > 0 && !segs)) return (int)hipErrorInvalidValue;
  CopyArgs a{};
  long most = 0;
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const dasa_copy_seg& s = segs[i];
    if (s.n0 < 0 || s.n1 < 0 || s.row_bytes < 0) return (int)hipErrorInvalidValue;
    const long units = (long)s.n0 * s.n1 * s.row_bytes / 16 + 1;
    if ((long)s.n0 * s.n1 * s.row_bytes == 0) continue;
    if (!s.src || !s.dst) return (int)hipErrorInvalidValue;
    a.seg[m++] = s;
    most = units > most ? units : most;
  }
  a.n = m;
  if (m == 0) return 0;
  long gx = (most + 255) / 256;
  if (gx > 256) gx = 256;   // grid-stride beyond 256 x 256 threads per segment
  hipLaunchKernelGGL(copy_segments_kernel, dim3((unsigned)gx, (unsigned)m), dim3(256), 0, (hipStream_t)stream, a);
  DASA_CHECK_LAUNCH();
  return 0;
}
