// FP8 (OCP e4m3fn) GEMM on the CDNA4 block-scaled MFMA, plus the per-token
// activation quantizer. North-star config 5 (GPT-2 XL, fp8 weights).
//
//   C[M,N] = act( (Aq[M,K] . Wq[N,K]^T) * sa[m] * sw[n] + bias[n] ) (+ R[M,N])
//
// Aq: per-row (per-token) scaled e4m3; Wq: per-output-channel scaled e4m3
// (quantised once at load, ops/fp8.py). v_mfma_scale_f32_16x16x128_f8f6f4 with
// unit E8M0 block scales (0x7F) runs at 2x the bf16 MFMA rate (guide §3); the
// real scales are applied in the fp32 epilogue. gfx950 fp8 is OCP e4m3fn, not
// MI300's fnuz (guide §4) — the converter below is the hardware OCP one.
//
// Tiling mirrors gemm_bf16: 128x128 tiles, BK = 128 bytes of K per stage (so the
// LDS image is byte-identical to the bf16 BK=64 one: 128-B rows, chunk XOR
// (row>>1)&7 swizzle on the glds source), 4 waves 2x2, 4x4 16x16 tiles/wave.
#include "api.h"
#include "common.h"

namespace dnn {

typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int F8_BM = 128, F8_BN = 128, F8_BK = 128;  // BK in elements (= bytes)
constexpr int F8_TILE = F8_BM * F8_BK;                 // 16 KiB

__device__ __forceinline__ int f8_swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void f8_stage(const uint8_t* __restrict__ src, int ld, int r0, int nrows, int k0, char* dst,
                                         int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int rl = piece * 8 + (lane >> 3);
    const int cs = (lane & 7) ^ f8_swz(rl);
    int r = r0 + rl;
    r = r < nrows ? r : nrows - 1;
    glds16(src + (size_t)r * ld + k0 + cs * 16, dst + piece * 1024);
  }
}

__device__ __forceinline__ i32x8 f8_frag(const char* tile, int row, int grp) {
  const int c0 = (2 * grp) ^ f8_swz(row), c1 = (2 * grp + 1) ^ f8_swz(row);
  const i32x4 a = *reinterpret_cast<const i32x4*>(tile + row * 128 + (c0 << 4));
  const i32x4 b = *reinterpret_cast<const i32x4*>(tile + row * 128 + (c1 << 4));
  i32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

template <int ACT>
__global__ __launch_bounds__(256, 2) void gemm_fp8_kernel(const uint8_t* __restrict__ A, const float* __restrict__ sa,
                                                          const uint8_t* __restrict__ W, const float* __restrict__ sw,
                                                          bf16_t* __restrict__ C, int ldc, const float* __restrict__ bias,
                                                          const bf16_t* __restrict__ R, int ldr, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[4 * F8_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + F8_BN - 1) / F8_BN, ntm = (M + F8_BM - 1) / F8_BM;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * F8_BM, n0 = (tile % ntn) * F8_BN;
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / F8_BK;
  f8_stage(A, K, m0, M, 0, smem, wave, lane);
  f8_stage(W, K, n0, N, 0, smem + F8_TILE, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    char* a_s = smem + cur * 2 * F8_TILE;
    char* b_s = a_s + F8_TILE;
    if (t + 1 < nk) {
      char* na = smem + (cur ^ 1) * 2 * F8_TILE;
      f8_stage(A, K, m0, M, (t + 1) * F8_BK, na, wave, lane);
      f8_stage(W, K, n0, N, (t + 1) * F8_BK, na + F8_TILE, wave, lane);
    }
    const int grp = lane >> 4;
    i32x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = f8_frag(a_s, wm * 64 + i * 16 + (lane & 15), grp);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = f8_frag(b_s, wn * 64 + j * 16 + (lane & 15), grp);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                     0x7f7f7f7f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    const float swn = n < N ? sw[n] : 0.f;
    const float b = (bias != nullptr && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if constexpr (ACT == 3) {
          // SwiGLU on the packed gate|up weight (ops/gemm.py pack_gate_up): in each
          // 16-column tile lanes (l & 15) < 8 hold gate, the lane ^ 8 partner its up
          const float v = m < M ? acc[i][j][r] * sa[m] * swn + b : 0.f;
          const float u = __shfl_xor(v, 8, 64);
          if ((lane & 8) == 0 && m < M && n < N)
            C[(size_t)m * ldc + (n0 + wn * 64 + j * 16) / 2 + (lane & 7)] = f2bf(silu(v) * u);
        } else if (m < M && n < N) {
          float v = acc[i][j][r] * sa[m] * swn + b;
          if (ACT == 1) v = fmaxf(v, 0.f);
          if (ACT == 2) v = gelu_erf(v);
          if (R != nullptr) v += bf2f(R[(size_t)m * ldr + n]);
          C[(size_t)m * ldc + n] = f2bf(v);
        }
      }
  }
}

// Per-row absmax quantisation bf16 -> e4m3 (scale = amax / 448). One wave per row.
// SPLIT: rows of 2 kpad bytes, the residual plane after the kpad bytes of hi.
template <bool SPLIT>
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, int ldx, uint8_t* __restrict__ q,
                                                             float* __restrict__ scale, int M, int K, int kpad) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (size_t)row * ldx;
  float amax = 0.f;
  for (int c = lane * 8; c < K; c += 512) {
    const bf16x8 p = *reinterpret_cast<const bf16x8*>(xr + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f_s(p[j])));
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[row] = s;
  uint8_t* qr = q + (size_t)row * kpad * (SPLIT ? 2 : 1);
  for (int c = lane * 8; c < kpad; c += 512) {
    bf16x8 p = {0, 0, 0, 0, 0, 0, 0, 0};  // zero K-padding (K -> multiple of 128)
    if (c < K) p = *reinterpret_cast<const bf16x8*>(xr + c);
    if constexpr (SPLIT) {
      float y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = bf2f_s(p[j]) * inv;
      int h0, h1, l0, l1;
      q8_split8(y, h0, h1, l0, l1);
      *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)h0, (uint32_t)h1);
      *reinterpret_cast<uint2*>(qr + kpad + c) = make_uint2((uint32_t)l0, (uint32_t)l1);
      continue;
    }
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f_s(p[0]) * inv, bf2f_s(p[1]) * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f_s(p[2]) * inv, bf2f_s(p[3]) * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f_s(p[4]) * inv, bf2f_s(p[5]) * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f_s(p[6]) * inv, bf2f_s(p[7]) * inv, hi, true);
    *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
  }
}

// MX quantisation bf16 -> e4m3 (common.h mx_index): one e8m0 scale per (row,
// 128-column block), one wave per row, one pass — the 16 lanes of a block
// take its amax with 4 xor-shuffles, so no row amax and no second read.
// Columns K..kpad-1 are written as zeros (scale of an all-zero block: 2^-126).
__global__ __launch_bounds__(256) void quant_fp8_mx_kernel(const bf16_t* __restrict__ x, int ldx,
                                                           uint8_t* __restrict__ q, int ldq, uint8_t* __restrict__ sx,
                                                           int M, int K, int kpad) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (size_t)row * ldx;
  uint8_t* qr = q + (size_t)row * ldq;
  const int mpad = mx_mpad(M);
  for (int c0 = 0; c0 < kpad; c0 += 512) {  // wave-uniform: every lane joins the shuffles
    const int c = c0 + lane * 8;
    bf16x8 p = {0, 0, 0, 0, 0, 0, 0, 0};
    if (c < K) p = *reinterpret_cast<const bf16x8*>(xr + c);
    float v[8], amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = bf2f_s(p[j]);
      amax = fmaxf(amax, fabsf(v[j]));
    }
    amax = group_max<16>(amax);
    float inv;
    const uint32_t e = e8m0_of(amax, inv);
    if (c < kpad) {
      int lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
      *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
      if ((lane & 15) == 0) sx[mx_index(row, c >> 7, mpad)] = (uint8_t)e;
    }
  }
}

}  // namespace dnn

using namespace dnn;

// MX-scaled e4m3 rows (the W8A8 prefill's activations, gemm_fp8_256 MXA):
// q [M][ldq bytes] (ldq >= kpad), sx = mx_mpad(M) * kpad / 128 scale bytes.
extern "C" int dnn_quant_fp8_mx(const void* x, int ldx, void* q, int ldq, void* sx, int M, int K, int kpad,
                                hipStream_t st) {
  if (K % 8 != 0 || kpad % 128 != 0 || kpad < K || ldq < kpad || (ldq & 7) != 0 || M <= 0) return M <= 0 ? 0 : -1;
  hipLaunchKernelGGL(quant_fp8_mx_kernel, dim3((M + 3) / 4), dim3(256), 0, st, (const bf16_t*)x, ldx, (uint8_t*)q,
                     ldq, (uint8_t*)sx, M, K, kpad);
  return (int)hipGetLastError();
}

// 0 = auto, 128 / 256 force a tile (A/B benchmarking, tests)
static int g_fp8_tile = 0;
extern "C" int dnn_gemm_fp8_set_tile(int tile) {
  if (tile != 0 && tile != 128 && tile != 256) return -1;
  g_fp8_tile = tile;
  return 0;
}

extern "C" int dnn_gemm_fp8(const void* A, const float* sa, const void* W, const float* sw, void* C, int ldc,
                            const float* bias, const void* R, int ldr, int M, int N, int K, int act, hipStream_t st) {
  if (K % F8_BK != 0) return -1;
  if (act == 3 && N % 16 != 0) return -1;  // packed gate|up groups of 8+8
  const int tiles = ((M + F8_BM - 1) / F8_BM) * ((N + F8_BN - 1) / F8_BN);
  // large GEMMs: the 256^2 4-phase fp8 kernel (gemm_bf16.hip) when its tiles
  // still fill the chip (same wave-quantisation rule as the bf16 dispatch)
  const int tiles256 = ((M + 255) / 256) * ((N + 255) / 256);
  auto fill = [](int t, int slots) {
    const int w = (t + slots - 1) / slots;
    return (double)t / ((double)w * slots);
  };
  if (g_fp8_tile != 128 && M >= 256 && N >= 256 &&
      (g_fp8_tile == 256 || 1.4 * fill(tiles256, 256) > fill(tiles, 512)))
    return dnn_gemm_fp8_256(A, sa, W, sw, C, ldc, bias, R, ldr, M, N, K, act, st);
#define F8(a)                                                                                                        \
  if (act == a) {                                                                                                    \
    hipLaunchKernelGGL((gemm_fp8_kernel<a>), dim3(tiles), dim3(256), 0, st, (const uint8_t*)A, sa, (const uint8_t*)W, \
                       sw, (bf16_t*)C, ldc, bias, (const bf16_t*)R, ldr, M, N, K);                                   \
    return (int)hipGetLastError();                                                                                   \
  }
  F8(0) F8(1) F8(2) F8(3)
#undef F8
  return -2;
}

extern "C" int dnn_quant_fp8_rows(const void* x, int ldx, void* q, float* scale, int M, int K, int kpad,
                                  hipStream_t st, int split) {
  if (K % 8 != 0 || kpad % 8 != 0 || kpad < K) return -1;
  if (split)
    hipLaunchKernelGGL(quant_fp8_rows_kernel<true>, dim3((M + 3) / 4), dim3(256), 0, st, (const bf16_t*)x, ldx,
                       (uint8_t*)q, scale, M, K, kpad);
  else
    hipLaunchKernelGGL(quant_fp8_rows_kernel<false>, dim3((M + 3) / 4), dim3(256), 0, st, (const bf16_t*)x, ldx,
                       (uint8_t*)q, scale, M, K, kpad);
  return (int)hipGetLastError();
}
