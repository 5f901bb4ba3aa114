// Shared GEMM epilogues for the MFMA kernels (gemm_bf16.hip, gemm_skinny.hip,
// gemm_fp8.hip).  All kernels issue their MFMAs as W.A^T ("transposed
// accumulators"), so after a 16x16 MFMA lane l holds output row m = .. + (l&15)
// and the 4 consecutive columns n = .. + 4*(l>>4) + r, r = 0..3.
#pragma once
#include "common.h"

namespace dnn {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SILU_MUL = 3 };

// Vector epilogue stores need 4-column-aligned rows and 16-B aligned bases.
__device__ __forceinline__ bool epi_vec_ok(const void* C, int ldc, const float* bias, const bf16_t* R, int ldr) {
  const uintptr_t p = (uintptr_t)C | (uintptr_t)bias | (uintptr_t)R;
  return ((ldc | (R != nullptr ? ldr : 0)) & 3) == 0 && (p & 15) == 0;
}

//
// Optional dequant scales (fp8 kernels): v *= rowscale * colscale[n..n+3].
template <int ACT, bool OUT_F32>
__device__ __forceinline__ void epi_t4(f32x4 v, int m, int n, int M, int N, void* __restrict__ Cv, int ldc,
                                       const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr,
                                       bool vec, const float* __restrict__ colscale = nullptr,
                                       float rowscale = 1.f) {
  if (m >= M) return;
  if (vec && n + 3 < N) {
    if (colscale != nullptr) v *= *reinterpret_cast<const f32x4*>(colscale + n) * rowscale;
    if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (ACT == ACT_RELU) v[r] = fmaxf(v[r], 0.f);
      if (ACT == ACT_GELU) v[r] = gelu_erf(v[r]);
    }
    if (R != nullptr) {
      const bf16x4 rr = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bf2f((bf16_t)rr[r]);
    }
    if (OUT_F32) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + (size_t)m * ldc + n) = v;
    } else {
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(Cv) + (size_t)m * ldc + n) = pk;
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int nn = n + r;
    if (nn < N) {
      float x = colscale != nullptr ? v[r] * colscale[nn] * rowscale : v[r];
      x += bias != nullptr ? bias[nn] : 0.f;
      if (ACT == ACT_RELU) x = fmaxf(x, 0.f);
      if (ACT == ACT_GELU) x = gelu_erf(x);
      if (R != nullptr) x += bf2f(R[(size_t)m * ldr + nn]);
      if (OUT_F32) reinterpret_cast<float*>(Cv)[(size_t)m * ldc + nn] = x;
      else reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + nn] = f2bf(x);
    }
  }
}

// SwiGLU epilogue on a transposed accumulator tile of the packed gate|up
// weight (ops/gemm.py pack_gate_up: 8 gate rows, then the 8 matching up rows):
// lanes 0-31 hold gate columns, lanes 32-63 the up columns of the same outputs,
// so one xor-32 shuffle pairs them; lanes 0-31 write output columns
// ncol0 + 4*(lane>>4) .. +3 of the [M, N/2] result.  Every lane must call this
// (the shuffle), whatever its row.
template <bool OUT_F32>
__device__ __forceinline__ void epi_silu_t4(const f32x4& acc, int m, int ncol0, int M, int NO, void* __restrict__ Cv,
                                            int ldc, bool vec, int lane) {
  f32x4 other;
#pragma unroll
  for (int r = 0; r < 4; ++r) other[r] = __shfl_xor(acc[r], 32, 64);
  if (lane >= 32 || m >= M) return;
  const int ncol = ncol0 + (lane >> 4) * 4;
  f32x4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = silu(acc[r]) * other[r];
  if (vec && ncol + 3 < NO) {
    if (OUT_F32) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + (size_t)m * ldc + ncol) = v;
    } else {
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(Cv) + (size_t)m * ldc + ncol) = pk;
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (ncol + r < NO) {
      if (OUT_F32) reinterpret_cast<float*>(Cv)[(size_t)m * ldc + ncol + r] = v[r];
      else reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + ncol + r] = f2bf(v[r]);
    }
}

}  // namespace dnn
