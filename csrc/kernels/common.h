// Shared helpers for the gfx950 (CDNA4, MI355X) kernels.
// Wave = 64 lanes. All bf16 data is handled as raw 16-bit patterns and widened
// with shifts; narrowing uses the compiler's v_cvt_pk_bf16_f32 (RNE, NaN-safe).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace dnn {

typedef uint16_t bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));  // operand of v_dot2_f32_bf16

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float bf2f_s(short v) { return __uint_as_float(((uint32_t)(uint16_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// NaN-propagating max (llvm.maximum -> v_maximum3_f32 on gfx950).  In IEEE
// mode fmaxf first quiets every operand the compiler cannot prove canonical
// (MFMA results, selects) with a v_max_f32 x, x of its own unless the file is
// built with -fno-honor-nans (ops/build.py PER_FILE_FLAGS); this form needs no
// quieting under any flags.
__device__ __forceinline__ float fmax_nan(float a, float b) { return __builtin_elementwise_maximum(a, b); }

// Exact-erf GELU (nanoGPT's nn.GELU()) without the branchy libm erff: with
// z = |x|/sqrt2, erf(z) = 1 - t*P(t)*exp(-z^2), t = 1/(1 + p z) (Abramowitz &
// Stegun 7.1.26, |error| <= 1.5e-7), so
//   gelu(x) = x - q  (x >= 0),   q  (x < 0),   q = 0.5 x t P(t) exp(-x^2/2).
// Straight-line: 1 v_rcp + 1 v_exp + ~10 FMA/MUL, no divergence in an epilogue.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);
  const float q = 0.5f * x * (p * t) * e;
  return x >= 0.f ? x - q : q;
}
// Two GELUs at once on packed fp32 math: the polynomial, the squares and the
// products go through v_pk_fma_f32 / v_pk_mul_f32 (two lanes' worth per
// instruction), only the reciprocal, the exponential, |x| and the sign select
// stay per element — a GEMM epilogue applies it to 128 outputs per thread.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 z = f32x2{fabsf(x[0]), fabsf(x[1])} * 0.70710678118654752f;
  const f32x2 d = z * 0.3275911f + 1.0f;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const f32x2 a = (z * z) * -1.44269504088896341f;
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])};
  const f32x2 q = (x * 0.5f) * (p * t) * e;
  return f32x2{x[0] >= 0.f ? x[0] - q[0] : q[0], x[1] >= 0.f ? x[1] - q[1] : q[1]};
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// DPP lane moves (VALU, no LDS round trip — __shfl_xor lowers to
// ds_bpermute_b32 on gfx950): quad_perm xor1 / xor2, row_half_mirror (lane i
// <-> 7-i within 8), row_mirror (i <-> 15-i within 16).  For a reduction any
// pairing of the two halves works, so these four steps reduce a 16-lane row.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum / max over aligned groups of L lanes (L = 1..64); every lane of the group
// gets the result.
template <int L>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (L >= 2) v += dpp_f<0xB1>(v);
  if constexpr (L >= 4) v += dpp_f<0x4E>(v);
  if constexpr (L >= 8) v += dpp_f<0x141>(v);
  if constexpr (L >= 16) v += dpp_f<0x140>(v);
  if constexpr (L >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (L >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
template <int L>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (L >= 2) v = fmaxf(v, dpp_f<0xB1>(v));
  if constexpr (L >= 4) v = fmaxf(v, dpp_f<0x4E>(v));
  if constexpr (L >= 8) v = fmaxf(v, dpp_f<0x141>(v));
  if constexpr (L >= 16) v = fmaxf(v, dpp_f<0x140>(v));
  if constexpr (L >= 32) v = fmaxf(v, __shfl_xor(v, 16, 64));
  if constexpr (L >= 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }
__device__ __forceinline__ float wave_max(float v) { return group_max<64>(v); }

// 16-byte async global->LDS copy. `lds_wave_base` must be wave-uniform: lane i
// lands at lds_wave_base + 16*i (glds semantics, cdna_hip_programming.md §5).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_wave_base, 16, 0, 0);
}

// Split ("x2") activations for the W8A8 prefill: the e4m3 hi byte of y and
// the e4m3 rounding of its residual (y - hi) * 16, written as a second K plane
// (row bytes kpad..2 kpad-1).  Against [W | W / 16] along K the fp8 GEMM then
// sums hi.W + lo.W/16 = y.W to ~2^-8 relative per activation instead of the
// 2^-4 of one e4m3 byte (GPT-2 XL 2 blocks: logits 5.7 % -> 0.13 % from the
// fp32 golden, emulated; measured on the device by tests/test_transformer_gpu.py).
__device__ __forceinline__ void q8_split8(const float (&y)[8], int& h0, int& h1, int& l0, int& l1) {
  h0 = __builtin_amdgcn_cvt_pk_fp8_f32(y[0], y[1], 0, false);
  h0 = __builtin_amdgcn_cvt_pk_fp8_f32(y[2], y[3], h0, true);
  h1 = __builtin_amdgcn_cvt_pk_fp8_f32(y[4], y[5], 0, false);
  h1 = __builtin_amdgcn_cvt_pk_fp8_f32(y[6], y[7], h1, true);
  const float d[8] = {__builtin_amdgcn_cvt_f32_fp8(h0, 0), __builtin_amdgcn_cvt_f32_fp8(h0, 1),
                      __builtin_amdgcn_cvt_f32_fp8(h0, 2), __builtin_amdgcn_cvt_f32_fp8(h0, 3),
                      __builtin_amdgcn_cvt_f32_fp8(h1, 0), __builtin_amdgcn_cvt_f32_fp8(h1, 1),
                      __builtin_amdgcn_cvt_f32_fp8(h1, 2), __builtin_amdgcn_cvt_f32_fp8(h1, 3)};
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (y[j] - d[j]) * 16.f;
  l0 = __builtin_amdgcn_cvt_pk_fp8_f32(r[0], r[1], 0, false);
  l0 = __builtin_amdgcn_cvt_pk_fp8_f32(r[2], r[3], l0, true);
  l1 = __builtin_amdgcn_cvt_pk_fp8_f32(r[4], r[5], 0, false);
  l1 = __builtin_amdgcn_cvt_pk_fp8_f32(r[6], r[7], l1, true);
}

// MX (block-scaled) fp8 activations for the W8A8 prefill GEMM: one e8m0
// scale per (row, 128-column K-tile), applied by the scaled MFMA itself
// (v_mfma_scale_f32_16x16x128_f8f6f4's per-lane B scale), so every
// quantiser — a row pass or a GEMM epilogue — decides its scales from the
// 128 columns it holds, with no whole-row amax.  Byte of (row m, K-tile t) in
// a buffer of Mpad = ceil(M / 64) * 64 rows per K-tile: within a 64-row block
// the 4 bytes of rows r, r + 16, r + 32, r + 48 are one dword, so the GEMM's
// lane (row r of each of its 4 16-row fragments) loads them with one load and
// selects byte i with the MFMA's op_sel.
__host__ __device__ __forceinline__ size_t mx_index(int m, int t, int mpad) {
  return ((size_t)t * (mpad >> 6) + (m >> 6)) * 64 + (m & 15) * 4 + ((m >> 4) & 3);
}
__host__ __device__ __forceinline__ int mx_mpad(int M) { return (M + 63) & ~63; }

// e8m0 block scale: the power of two 2^e >= amax / 448 as its biased exponent
// byte (fp32 and e8m0 share the bias 127) and its reciprocal; clamped to
// [2^-126, 2^126] (never the NaN code 255, never a subnormal reciprocal).
__device__ __forceinline__ uint32_t e8m0_of(float amax, float& inv) {
  const uint32_t b = __float_as_uint(amax * (1.f / 448.f));
  uint32_t e = ((b >> 23) & 0xffu) + ((b & 0x7fffffu) != 0u ? 1u : 0u);
  e = e < 1u ? 1u : (e > 253u ? 253u : e);
  inv = __uint_as_float((254u - e) << 23);  // 2^(127 - e)
  return e;
}

// Bijective XCD-aware block remap: blocks that the dispatcher places on the same
// XCD (b % 8 equal) get a contiguous range of logical tile ids (guide §5, T1).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, idx = bid / 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace dnn
