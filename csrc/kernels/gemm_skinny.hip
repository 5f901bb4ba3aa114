// Skinny (decode-sized, M <= 64) GEMMs: weight streaming at HBM rate.
//
//   C[M,N] = act(A[M,K] . W[N,K]^T * (sa[m] sw[n]) + bias[n]) (+ R[M,N])
//
// In decode every projection is a GEMV-like product: the whole weight matrix is
// read once per step and the activations are a few KiB, so the roofline is HBM
// bandwidth and the enemy is latency (guide §5 table, "GEMV / M <= 16": load
// straight to VGPRs, deep unroll, late vmcnt — no LDS round trip for W).
//
// Layout: a workgroup owns NT x 16 output columns and KS waves that split K
// into contiguous slices; every wave streams its slice in chunks of 64 B per
// row (16 B per lane: 4 lane groups x 16 B), issuing U chunks of W and of the
// (L2-resident) A rows before the first MFMA, so U x 1 KiB of weights per wave
// is in flight.  The KS partial sums meet in LDS; the epilogue is the shared
// transposed-accumulator one (gemm_epilogue.h): bias / act / residual / SwiGLU
// (NT = 2: gate and up tile of the packed gate|up weight in one workgroup).
//
// bf16: one v_mfma_f32_16x16x32_bf16 per 16-B chunk.  fp8 (OCP e4m3fn weights
// and per-token-quantised activations, ops/fp8.py): two
// v_mfma_f32_16x16x32_fp8_fp8 per chunk (the k order inside a chunk is the same
// permutation for A and W, so the dot product is unchanged); the weight bytes
// and so the step time halve.  KS is chosen on the host so that N/16 x KS waves
// cover the CUs.
#include "gemm_epilogue.h"

namespace dnn {

template <bool FP8>
__device__ __forceinline__ f32x4 sk_mma(const i32x4& w, const i32x4& a, f32x4 acc) {
  if constexpr (FP8) {
    const long w0 = ((long)(uint32_t)w[1] << 32) | (uint32_t)w[0];
    const long w1 = ((long)(uint32_t)w[3] << 32) | (uint32_t)w[2];
    const long a0 = ((long)(uint32_t)a[1] << 32) | (uint32_t)a[0];
    const long a1 = ((long)(uint32_t)a[3] << 32) | (uint32_t)a[2];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w0, a0, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w1, a1, acc, 0, 0, 0);
  } else {
    bf16x8 wb, ab;
    __builtin_memcpy(&wb, &w, 16);
    __builtin_memcpy(&ab, &a, 16);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb, ab, acc, 0, 0, 0);
  }
}

template <int ACT, bool OUT_F32, int MT, int NT, bool FP8, int U>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const uint8_t* __restrict__ A, int lda_b,
                                                           const float* __restrict__ sa, const uint8_t* __restrict__ W,
                                                           int ldw_b, const float* __restrict__ sw,
                                                           void* __restrict__ Cv, int ldc,
                                                           const float* __restrict__ bias,
                                                           const bf16_t* __restrict__ R, int ldr, int M, int N,
                                                           int kbytes) {
  extern __shared__ __attribute__((aligned(16))) f32x4 sk_red[];  // [KS][NT*MT][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, KS = blockDim.x >> 6;
  const int n0 = blockIdx.x * (16 * NT);
  const int lg = (lane >> 4) * 16;  // byte offset of this lane group inside a 64-B chunk

  const uint8_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int n = n0 + j * 16 + (lane & 15);
    n = n < N ? n : N - 1;
    wp[j] = W + (size_t)n * ldw_b + lg;
  }
  const uint8_t* ap[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    int m = t * 16 + (lane & 15);
    m = m < M ? m : M - 1;
    ap[t] = A + (size_t)m * lda_b + lg;
  }
  f32x4 acc[NT][MT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = kbytes >> 6;
  const int per = (nch + KS - 1) / KS;
  const int c0 = wave * per, c1 = min(nch, c0 + per);
  int c = c0;
  for (; c + U <= c1; c += U) {
    i32x4 wv[NT][U], av[MT][U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) wv[j][u] = *reinterpret_cast<const i32x4*>(wp[j] + (size_t)(c + u) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) av[t][u] = *reinterpret_cast<const i32x4*>(ap[t] + (size_t)(c + u) * 64);
    // keep every load of the batch ahead of the first MFMA (the scheduler would
    // otherwise interleave them and wait vmcnt(0) per chunk: 1-2 loads in flight)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[j][t] = sk_mma<FP8>(wv[j][u], av[t][u], acc[j][t]);
  }
  for (; c < c1; ++c) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const i32x4 w = *reinterpret_cast<const i32x4*>(wp[j] + (size_t)c * 64);
#pragma unroll
      for (int t = 0; t < MT; ++t)
        acc[j][t] = sk_mma<FP8>(w, *reinterpret_cast<const i32x4*>(ap[t] + (size_t)c * 64), acc[j][t]);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) sk_red[(wave * NT * MT + j * MT + t) * 64 + lane] = acc[j][t];
  __syncthreads();

  // reduction over the KS waves + epilogue: wave w finishes M tiles t = w, w+KS, ...
  const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
  for (int t = wave; t < MT; t += KS) {
    f32x4 s[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      s[j] = sk_red[(j * MT + t) * 64 + lane];
      for (int w = 1; w < KS; ++w) s[j] += sk_red[(w * NT * MT + j * MT + t) * 64 + lane];
    }
    const int m = t * 16 + (lane & 15);
    const float rs = (FP8 && m < M) ? sa[m] : 1.f;
    if constexpr (ACT == ACT_SILU_MUL) {
      static_assert(NT % 2 == 0, "SwiGLU needs gate/up tile pairs");
#pragma unroll
      for (int jp = 0; jp < NT; jp += 2) {
        if constexpr (FP8) {
          const int ng = n0 + jp * 16 + (lane >> 4) * 4, nu = ng + 16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[jp][r] *= rs * (ng + r < N ? sw[ng + r] : 0.f);
            s[jp + 1][r] *= rs * (nu + r < N ? sw[nu + r] : 0.f);
          }
        }
        epi_silu_t4<OUT_F32>(s[jp], s[jp + 1], m, (n0 + jp * 16) / 2 + (lane >> 4) * 4, M, N / 2, Cv, ldc, vec);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NT; ++j)
        epi_t4<ACT, OUT_F32>(s[j], m, n0 + j * 16 + (lane >> 4) * 4, M, N, Cv, ldc, bias, R, ldr, vec,
                             FP8 ? sw : nullptr, rs);
    }
  }
}

}  // namespace dnn

using namespace dnn;

// Waves per workgroup: enough workgroups x waves to cover the 256 CUs (x4 SIMDs)
// while every wave keeps >= 2 chunks of K.
static int skinny_ks(int groups, int nch) {
  int ks = groups <= 256 ? 8 : 4;
  while (ks > 1 && nch / ks < 2) ks >>= 1;
  return ks;
}

// Per chunk a wave issues NT weight loads and MT activation loads (L2) for
// NT x MT MFMAs: NT grows with MT so the activation re-reads stay <= the
// weight bytes.  U = chunks in flight, sized for <= 256 VGPRs at 8 waves/WG.
template <int ACT, bool F32, bool FP8, int MT, int NT, int U>
static int launch_skinny_cfg(const void* A, int lda_b, const float* sa, const void* W, int ldw_b, const float* sw,
                             void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                             hipStream_t st) {
  const int groups = (N + 16 * NT - 1) / (16 * NT);
  const int ks = skinny_ks(groups, kbytes / 64);
  const size_t smem = (size_t)ks * NT * MT * 64 * sizeof(f32x4);
  hipLaunchKernelGGL((gemm_skinny_kernel<ACT, F32, MT, NT, FP8, U>), dim3(groups), dim3(64 * ks), smem, st,
                     (const uint8_t*)A, lda_b, sa, (const uint8_t*)W, ldw_b, sw, C, ldc, bias, (const bf16_t*)R, ldr,
                     M, N, kbytes);
  return (int)hipGetLastError();
}

template <int ACT, bool F32, bool FP8, int MT, int U4>
static int launch_skinny_mt(const void* A, int lda_b, const float* sa, const void* W, int ldw_b, const float* sw,
                            void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                            hipStream_t st) {
  // widest column tile that still leaves >= 128 workgroups (small N: latency-bound, keep the waves)
  if (N >= 128 * 64)
    return launch_skinny_cfg<ACT, F32, FP8, MT, 4, U4>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R, ldr, M, N, kbytes,
                                                        st);
  if (ACT == ACT_SILU_MUL || N >= 128 * 32)
    return launch_skinny_cfg<ACT, F32, FP8, MT, 2, (MT >= 4 ? 4 : 8)>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias,
                                                                              R, ldr, M, N, kbytes, st);
  if constexpr (ACT != ACT_SILU_MUL)
    return launch_skinny_cfg<ACT, F32, FP8, MT, 1, 8>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R, ldr, M, N, kbytes,
                                                       st);
  return -2;
}

template <int ACT, bool F32, bool FP8>
static int launch_skinny(const void* A, int lda_b, const float* sa, const void* W, int ldw_b, const float* sw,
                         void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                         hipStream_t st) {
  if (M <= 16)
    return launch_skinny_mt<ACT, F32, FP8, 1, 8>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R, ldr, M, N, kbytes, st);
  if (M <= 32)
    return launch_skinny_mt<ACT, F32, FP8, 2, 4>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R, ldr, M, N, kbytes, st);
  return launch_skinny_mt<ACT, F32, FP8, 4, 4>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R, ldr, M, N, kbytes, st);
}

// bf16: K % 32 == 0 (64-B chunks), M <= 64.  fp8: K (bytes) % 64 == 0.
extern "C" int dnn_gemm_skinny(const void* A, int lda, const float* sa, const void* W, int ldw, const float* sw,
                               void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int K,
                               int act, int out_f32, int fp8, hipStream_t st) {
  const int eb = fp8 ? 1 : 2;
  const int kbytes = K * eb;
  if (M <= 0 || M > 64 || N <= 0 || kbytes % 64 != 0) return -1;
  if (act == ACT_SILU_MUL && N % 32 != 0) return -1;  // packed gate|up groups of 32
  if (fp8 && (sa == nullptr || sw == nullptr)) return -1;
  const int la = lda * eb, lw = ldw * eb;
#define SKD(a)                                                                                              \
  if (act == a) {                                                                                           \
    if (fp8) {                                                                                              \
      return out_f32 ? launch_skinny<a, true, true>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st)  \
                     : launch_skinny<a, false, true>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st); \
    }                                                                                                       \
    return out_f32 ? launch_skinny<a, true, false>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st)   \
                   : launch_skinny<a, false, false>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st);  \
  }
  SKD(ACT_NONE)
  SKD(ACT_RELU)
  SKD(ACT_GELU)
  SKD(ACT_SILU_MUL)
#undef SKD
  return -2;
}
