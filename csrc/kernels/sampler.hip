// Greedy sampler: per-row argmax over the vocabulary (ties -> smallest index,
// numpy semantics). Replaces the host-side np.argmax of the reference
// (node.py:61,190), done per row instead of over the flattened batch.
#include "common.h"

namespace dnn {

template <bool F32>
__global__ __launch_bounds__(256) void argmax_rows_kernel(const void* __restrict__ xv, int ld, int M, int N,
                                                          int* __restrict__ out) {
  const int row = blockIdx.x;
  if (row >= M) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if (F32) {
    const float* x = reinterpret_cast<const float*>(xv) + (size_t)row * ld;
    for (int i = threadIdx.x; i < N; i += 256) {
      const float v = x[i];
      if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    }
  } else {
    const bf16_t* x = reinterpret_cast<const bf16_t*>(xv) + (size_t)row * ld;
    const int n8 = (N / 8) * 8;
    for (int i = threadIdx.x * 8; i < n8; i += 256 * 8) {
      const bf16x8 p = *reinterpret_cast<const bf16x8*>(x + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = bf2f_s(p[j]);
        if (v > best) { best = v; bi = i + j; }
      }
    }
    for (int i = n8 + threadIdx.x; i < N; i += 256) {
      const float v = bf2f(x[i]);
      if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = best; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (sv[w] > best || (sv[w] == best && si[w] < bi)) { best = sv[w]; bi = si[w]; }
    out[row] = bi;
  }
}

}  // namespace dnn

using namespace dnn;

extern "C" int dnn_argmax_rows(const void* x, int ld, int M, int N, int* out, int f32in, hipStream_t st) {
  if (M <= 0) return 0;
  if (!f32in && (ld % 8) != 0) return -1;
  if (f32in) hipLaunchKernelGGL((argmax_rows_kernel<true>), dim3(M), dim3(256), 0, st, x, ld, M, N, out);
  else hipLaunchKernelGGL((argmax_rows_kernel<false>), dim3(M), dim3(256), 0, st, x, ld, M, N, out);
  return (int)hipGetLastError();
}
