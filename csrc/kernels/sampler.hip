// Greedy sampler: per-row argmax over the vocabulary (ties -> smallest index,
// numpy semantics). Replaces the host-side np.argmax of the reference
// (node.py:61,190), done per row instead of over the flattened batch.
#include "common.h"

namespace dnn {

// One workgroup per row.  bf16 rows: every thread issues all of its 16-B loads
// before the first compare (NV per lane, unrolled), so a row costs one memory
// round trip instead of one per 2048-element sweep (Llama-3's 128K vocabulary
// at batch 1: one 1024-thread workgroup, 16 loads per lane).  Decode step tail
// fused in: the token also goes to `out2` (the next step's input ids) and
// `pos_inc[row]` advances by one, so the sampled id, the input-id copy and the
// position update are one launch instead of three.
__device__ __forceinline__ void argmax_merge(float& best, int& bi, float v, int i) {
  if (v > best || (v == best && i < bi)) { best = v; bi = i; }
}

// Token history (multi-step decode graphs): `hist[row * hist_ld + pos]` gets
// the sampled id at the row's position before the advance, so K decode steps
// replayed as one graph leave every step's token in device memory (no host
// bookkeeping per step); positions outside [0, hist_ld) are not written.
__device__ __forceinline__ void step_tail(int row, int bi, int* out, int* out2, int* pos_inc, int* hist,
                                          int hist_ld) {
  out[row] = bi;
  if (out2 != nullptr) out2[row] = bi;
  if (pos_inc != nullptr) {
    const int p = pos_inc[row];
    if (hist != nullptr && p >= 0 && p < hist_ld) hist[(size_t)row * hist_ld + p] = bi;
    pos_inc[row] = p + 1;
  }
}

template <bool F32, int TH, int NV>
__global__ __launch_bounds__(TH) void argmax_rows_kernel(const void* __restrict__ xv, int ld, int M, int N,
                                                         int* __restrict__ out, int* __restrict__ out2,
                                                         int* __restrict__ pos_inc, int* __restrict__ hist,
                                                         int hist_ld) {
  const int row = blockIdx.x;
  if (row >= M) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if constexpr (F32) {
    const float* x = reinterpret_cast<const float*>(xv) + (size_t)row * ld;
    for (int i = threadIdx.x; i < N; i += TH) argmax_merge(best, bi, x[i], i);
  } else {
    const bf16_t* x = reinterpret_cast<const bf16_t*>(xv) + (size_t)row * ld;
    const int n8 = (N / 8) * 8;
    // full sweeps of TH x 8 elements, NV at a time with every load in flight
    for (int base = 0; base < n8; base += NV * TH * 8) {
      bf16x8 p[NV];
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int i = base + (u * TH + threadIdx.x) * 8;
        p[u] = i < n8 ? *reinterpret_cast<const bf16x8*>(x + i) : bf16x8{};
      }
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int i = base + (u * TH + threadIdx.x) * 8;
        if (i < n8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float v = bf2f_s(p[u][j]);
            if (v > best) { best = v; bi = i + j; }  // ascending i per lane: strict > keeps the first
          }
        }
      }
    }
    for (int i = n8 + threadIdx.x; i < N; i += TH) argmax_merge(best, bi, bf2f(x[i]), i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_merge(best, bi, ov, oi);
  }
  __shared__ float sv[TH / 64];
  __shared__ int si[TH / 64];
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = best; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < TH / 64; ++w) argmax_merge(best, bi, sv[w], si[w]);
    bi = bi == 0x7fffffff ? 0 : bi;  // all-NaN row: token 0
    step_tail(row, bi, out, out2, pos_inc, hist, hist_ld);
  }
}

// Row split (small batches): one workgroup per row leaves most of the chip
// idle (GPT-2 B = 64: 64 workgroups, 12.6 us for 6.4 MB; Llama-3 B = 1: one
// CU reads the 128K-entry row, 24 us).  argmax_part_kernel: grid (S, M), each
// workgroup takes one contiguous segment of a row (all of its 16-B loads in
// flight) and writes {value bits, index} of its winner; argmax_final_kernel:
// one wave per row merges the S partials (ties -> smallest index) and does the
// decode step tail (ids copy, position advance).
template <int NV>
__global__ __launch_bounds__(256) void argmax_part_kernel(const bf16_t* __restrict__ x, int ld, int N, int seg,
                                                          int2* __restrict__ part) {
  const int s = blockIdx.x, row = blockIdx.y, S = gridDim.x;
  const int lo = s * seg, hi = min(N, lo + seg);
  const bf16_t* xr = x + (size_t)row * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int hi8 = lo + ((hi - lo) / 8) * 8;  // seg and lo are multiples of 8
  for (int base = lo; base < hi8; base += NV * 256 * 8) {
    bf16x8 p[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = base + (u * 256 + (int)threadIdx.x) * 8;
      p[u] = i < hi8 ? *reinterpret_cast<const bf16x8*>(xr + i) : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = base + (u * 256 + (int)threadIdx.x) * 8;
      if (i < hi8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f_s(p[u][j]);
          if (v > best) { best = v; bi = i + j; }
        }
      }
    }
  }
  for (int i = hi8 + (int)threadIdx.x; i < hi; i += 256) argmax_merge(best, bi, bf2f(xr[i]), i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_merge(best, bi, ov, oi);
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = best; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) argmax_merge(best, bi, sv[w], si[w]);
    part[(size_t)row * S + s] = make_int2(__float_as_int(best), bi);
  }
}

__global__ __launch_bounds__(256) void argmax_final_kernel(const int2* __restrict__ part, int S, int M,
                                                           int* __restrict__ out, int* __restrict__ out2,
                                                           int* __restrict__ pos_inc, int* __restrict__ hist,
                                                           int hist_ld) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int s = lane; s < S; s += 64) {
    const int2 p = part[(size_t)row * S + s];
    argmax_merge(best, bi, __int_as_float(p.x), p.y);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_merge(best, bi, ov, oi);
  }
  if (lane == 0) {
    bi = bi == 0x7fffffff ? 0 : bi;  // all-NaN row: token 0
    step_tail(row, bi, out, out2, pos_inc, hist, hist_ld);
  }
}

// ---------------------------------------------------------------------------
// Stochastic sampler: temperature + top-k via the Gumbel-max trick
//   token = argmax_{i in topk} ( x_i / T + G_i ),  G_i = -log(-log(U_i))
// which draws exactly from softmax(x / T) restricted to the k largest logits.
// One 1024-thread workgroup per row keeps the whole bf16 row in VGPRs (NV x 16 B
// per lane: 128K-entry vocabularies fit), finds the k-th largest logit by a
// 16-step bisection over the order-preserving 16-bit key (block-wide counts,
// no atomics), then takes the Gumbel-max over the survivors.  U_i is a
// counter-based hash of (seed, row, step[row], i): no RNG state, so one captured
// HIP graph serves every decode step (step = the row's position, in device
// memory) and the result is reproducible.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bf16_key(short v) {
  const uint32_t u = (uint16_t)v;
  return (u & 0x8000u) ? (~u & 0xFFFFu) : (u | 0x8000u);
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float key_to_f(uint32_t k) {
  const uint32_t u = (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu);
  return __uint_as_float(u << 16);
}

template <int NV, int TH>
__global__ __launch_bounds__(TH) void sample_topk_kernel(const bf16_t* __restrict__ x, int ld, int M, int N,
                                                           int* __restrict__ out, float inv_temp, int topk,
                                                           uint32_t seed, const int* __restrict__ step) {
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* xr = x + (size_t)row * ld;
  // the row lives in VGPRs as packed 16-bit order-preserving keys (2 per dword)
  uint32_t kw[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i0 = (tid + TH * j) * 8;
    bf16x8 p;
    if (i0 + 8 <= N) {
      p = *reinterpret_cast<const bf16x8*>(xr + i0);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) p[e] = (short)(i0 + e < N ? xr[i0 + e] : (bf16_t)0xFF80u);  // -inf pad
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) kw[j][e] = bf16_key(p[2 * e]) | (bf16_key(p[2 * e + 1]) << 16);
  }
  __shared__ int red[16];
  __shared__ float bv[16];
  __shared__ int bi_s[16];
  uint32_t thr = 0;
  if (topk > 0 && topk < N) {
    for (int bit = 15; bit >= 0; --bit) {
      const uint32_t cand = thr | (1u << bit);
      int c = 0;
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t w = kw[j][e];
          asm volatile("" : "+v"(w));  // keep the unpack inside the loop (no hoisted 2x copy)
          c += ((w & 0xFFFFu) >= cand ? 1 : 0) + ((w >> 16) >= cand ? 1 : 0);
        }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) red[wave] = c;
      __syncthreads();
      int tot = 0;
#pragma unroll
      for (int w = 0; w < TH / 64; ++w) tot += red[w];
      __syncthreads();
      if (tot >= topk) thr = cand;
    }
  }
  const uint32_t st = step != nullptr ? (uint32_t)step[row] : 0u;
  const uint32_t base = mix32(seed ^ mix32((uint32_t)row * 0x9E3779B9u ^ mix32(st + 0x632BE5ABu)));
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = (tid + TH * j) * 8 + e;
      const uint32_t k = (kw[j][e >> 1] >> ((e & 1) * 16)) & 0xFFFFu;
      if (i < N && k >= thr) {
        const uint32_t h = mix32(base ^ (uint32_t)i * 0x85EBCA6Bu);
        const float u = ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
        const float sc = key_to_f(k) * inv_temp - __logf(-__logf(u));
        if (sc > best) { best = sc; bi = i; }
      }
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) { bv[wave] = best; bi_s[wave] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < TH / 64; ++w)
      if (bv[w] > best || (bv[w] == best && bi_s[w] < bi)) { best = bv[w]; bi = bi_s[w]; }
    out[row] = bi == 0x7fffffff ? 0 : bi;
  }
}

}  // namespace dnn

using namespace dnn;

extern "C" int dnn_sample_topk(const void* x, int ld, int M, int N, int* out, float temperature, int topk,
                               unsigned seed, const int* step, hipStream_t st) {
  if (M <= 0) return 0;
  if (!(temperature > 0.f) || (ld % 8) != 0) return -1;
  const int nv = (N + 8 * 1024 - 1) / (8 * 1024);
  const float it = 1.f / temperature;
#define SAMP(NVV, THV)                                                                                               \
  {                                                                                                                  \
    hipLaunchKernelGGL((sample_topk_kernel<NVV, THV>), dim3(M), dim3(THV), 0, st, (const bf16_t*)x, ld, M, N, out, it, \
                       topk, (uint32_t)seed, step);                                                                  \
    return (int)hipGetLastError();                                                                                   \
  }
  // <= 64K entries: 1024 threads, <= 8 vectors each; larger vocabularies (Llama-3
  // 128K): 512 threads x 32 vectors (128 key VGPRs of a 256 budget)
  if (nv <= 1) SAMP(1, 1024)
  if (nv <= 2) SAMP(2, 1024)
  if (nv <= 4) SAMP(4, 1024)
  if (nv <= 8) SAMP(8, 1024)
  if (nv <= 16) SAMP(32, 512)
#undef SAMP
  return -2;  // vocabulary > 128K entries
}

// The second pass of a row-split argmax whose partials another kernel wrote
// (part[row * S + s]; gemm_head.h writes one per workgroup), with the decode
// step tail.
extern "C" int dnn_argmax_final(const void* part, int S, int M, int* out, int* out2, int* pos_inc, hipStream_t st,
                                int* hist, int hist_ld) {
  if (M <= 0) return 0;
  if (S <= 0 || part == nullptr) return -1;
  if (hist != nullptr && (pos_inc == nullptr || hist_ld <= 0)) return -1;
  hipLaunchKernelGGL(argmax_final_kernel, dim3((M + 3) / 4), dim3(256), 0, st, (const int2*)part, S, M, out, out2,
                     pos_inc, hist, hist_ld);
  return (int)hipGetLastError();
}

// part (optional, >= M * 64 int2): workspace of the row-split path (bf16 rows,
// fewer than 512 rows x segments otherwise); nullptr = one workgroup per row.
extern "C" int dnn_argmax_rows(const void* x, int ld, int M, int N, int* out, int f32in, hipStream_t st,
                               int* out2, int* pos_inc, void* part, int* hist, int hist_ld) {
  if (M <= 0) return 0;
  if (!f32in && (ld % 8) != 0) return -1;
  if (hist != nullptr && (pos_inc == nullptr || hist_ld <= 0)) return -1;
  if (!f32in && part != nullptr && M < 256) {
    // segments per row: ~512 workgroups in all, >= 2048 entries per segment
    int S = (512 + M - 1) / M;
    S = S > 64 ? 64 : S;
    const int maxS = (N + 2047) / 2048;
    S = S > maxS ? maxS : S;
    if (S >= 2) {
      const int seg = ((N + S - 1) / S + 7) / 8 * 8;
      S = (N + seg - 1) / seg;
      const int nv = (seg + 2047) / 2048;  // 16-B vectors per thread per sweep
      if (nv <= 2) {
        hipLaunchKernelGGL((argmax_part_kernel<2>), dim3(S, M), dim3(256), 0, st, (const bf16_t*)x, ld, N, seg,
                           (int2*)part);
      } else {
        hipLaunchKernelGGL((argmax_part_kernel<4>), dim3(S, M), dim3(256), 0, st, (const bf16_t*)x, ld, N, seg,
                           (int2*)part);
      }
      hipLaunchKernelGGL(argmax_final_kernel, dim3((M + 3) / 4), dim3(256), 0, st, (const int2*)part, S, M, out, out2,
                         pos_inc, hist, hist_ld);
      return (int)hipGetLastError();
    }
  }
  if (f32in) {
    hipLaunchKernelGGL((argmax_rows_kernel<true, 256, 1>), dim3(M), dim3(256), 0, st, x, ld, M, N, out, out2, pos_inc,
                       hist, hist_ld);
  } else if (M <= 16) {
    // few rows: a wide workgroup per row (Llama-3 128K vocabulary: 16 loads per lane)
    hipLaunchKernelGGL((argmax_rows_kernel<false, 1024, 16>), dim3(M), dim3(1024), 0, st, x, ld, M, N, out, out2,
                       pos_inc, hist, hist_ld);
  } else {
    hipLaunchKernelGGL((argmax_rows_kernel<false, 256, 8>), dim3(M), dim3(256), 0, st, x, ld, M, N, out, out2,
                       pos_inc, hist, hist_ld);
  }
  return (int)hipGetLastError();
}
