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

// Folded pre-norm on an accumulator (prefill GEMMs after ops/gemm.py
// fold_norm): v = rstd[m] * v - mean[m] rstd[m] * colsum[n..n+3], rowstat[m] =
// {rstd, -mean * rstd} (RMSNorm: shift 0, no colsum) from row_stats_kernel.
__device__ __forceinline__ f32x4 epi_norm4(f32x4 v, int m, int n, int M, int N, const float2* __restrict__ rowstat,
                                           const float* __restrict__ colsum) {
  const float2 st = rowstat[m < M ? m : M - 1];
  v *= st.x;
  if (colsum != nullptr) {
    f32x4 cs;
    if (n + 3 < N) {
      cs = *reinterpret_cast<const f32x4*>(colsum + n);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[r] = n + r < N ? colsum[n + r] : 0.f;
    }
    v += st.y * cs;
  }
  return v;
}

//
// Optional dequant scales (fp8 kernels): v *= rowscale * colscale[n..n+3].
// ``stored`` (bf16 output only): receives the values as stored (bf16-rounded;
// 0 for columns past N and rows past M), for the row-statistics producer.
template <int ACT, bool OUT_F32>
__device__ __forceinline__ void epi_t4(f32x4 v, int m, int n, int M, int N, void* __restrict__ Cv, int ldc,
                                       const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr,
                                       bool vec, const float* __restrict__ colscale = nullptr,
                                       float rowscale = 1.f, f32x4* stored = nullptr) {
  if (stored != nullptr) *stored = f32x4{0.f, 0.f, 0.f, 0.f};
  if (m >= M) return;
  if (vec && n + 3 < N) {
    if (colscale != nullptr) v *= *reinterpret_cast<const f32x4*>(colscale + n) * rowscale;
    if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + n);
    if constexpr (ACT == ACT_GELU) {
      const f32x2 g0 = gelu_erf2(f32x2{v[0], v[1]}), g1 = gelu_erf2(f32x2{v[2], v[3]});
      v = f32x4{g0[0], g0[1], g1[0], g1[1]};
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (ACT == ACT_RELU) v[r] = fmaxf(v[r], 0.f);
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
      if (stored != nullptr)
        *stored = f32x4{__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                        __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
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
      if (OUT_F32) {
        reinterpret_cast<float*>(Cv)[(size_t)m * ldc + nn] = x;
      } else {
        const bf16_t b = f2bf(x);
        reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + nn] = b;
        if (stored != nullptr) (*stored)[r] = bf2f(b);
      }
    }
  }
}

// epi_t4's vector path with the bias and residual already in registers (the
// decode one-shot GEMM issues them with its first loads, so the epilogue pays
// no memory round trip after the workgroup's reduction).  Caller: m < M,
// n + 3 < N, 16-B aligned rows (epi_vec_ok).
template <int ACT>
__device__ __forceinline__ void epi_t4_pre(f32x4 v, int m, int n, void* __restrict__ Cv, int ldc, bool has_b,
                                           const f32x4& b4, bool has_r, const bf16x4& r4, f32x4* stored = nullptr) {
  if (has_b) v += b4;
  if constexpr (ACT == ACT_GELU) {
    const f32x2 g0 = gelu_erf2(f32x2{v[0], v[1]}), g1 = gelu_erf2(f32x2{v[2], v[3]});
    v = f32x4{g0[0], g0[1], g1[0], g1[1]};
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (ACT == ACT_RELU) v[r] = fmaxf(v[r], 0.f);
  }
  if (has_r) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += bf2f((bf16_t)r4[r]);
  }
  uint2 pk;
  pk.x = pack2bf(v[0], v[1]);
  pk.y = pack2bf(v[2], v[3]);
  *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(Cv) + (size_t)m * ldc + n) = pk;
  if (stored != nullptr)
    *stored = f32x4{__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u), __uint_as_float(pk.y << 16),
                    __uint_as_float(pk.y & 0xffff0000u)};
}

// Row-statistics partial of one 16-column output tile, produced in the
// epilogue of a residual-writing decode GEMM so that the
// next pre-norm projection merges ~N/16 partials per row instead of
// re-deriving the statistics from its activations in every column-tile
// workgroup.  Transposed-accumulator layout: lane (fr = l & 15, fg = l >> 4)
// holds row m's columns n0 + 4 fg .. + 3 (``x``: the stored bf16 values, 0
// past N).  Writes {mean, sum of squared deviations} of the tile's valid
// columns (two-pass over registers: no cancellation whatever the row mean)
// to rs[m * ld + n0 / 16] from lane group 0.  Every lane must call it.
__device__ __forceinline__ void epi_rowstat16(const f32x4& x, int m, int n0, int M, int N, float2* __restrict__ rs,
                                              int ld, int lane) {
  if (n0 >= N) return;  // a surplus tile past the row (uniform: n0 is the tile's): no partial, no write
  const int nt = min(16, N - n0);  // >= 1: the tile starts inside the row
  const int nv = min(4, max(0, N - n0 - 4 * (lane >> 4)));
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) s += r < nv ? x[r] : 0.f;
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mean = s / (float)nt;
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float d = r < nv ? x[r] - mean : 0.f;
    q = fmaf(d, d, q);
  }
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  if (lane < 16 && m < M) rs[(size_t)m * ld + (n0 >> 4)] = make_float2(mean, q);
}

// Consumer side: (mean, rstd) of row ``row`` of a K-wide activation from its
// ceil(K/16) tile partials rs[row * ld + i] = {mean_i, M2_i} (epi_rowstat16),
// merged by TPR adjacent lanes, each holding up to SPT partials (``p`` =
// partials sub, sub + TPR, ...; ``p0`` = partial 0).  Shifted by partial 0's
// mean c:  mean = c + S1 / K,  M2 = sum M2_i + S2 - S1^2 / K  with
// S1 = sum n_i (mean_i - c), S2 = sum n_i (mean_i - c)^2 — robust for any
// |mean| / std.  RMS (NORM 1): c = 0 and E[x^2] = (sum M2_i + S2) / K.
template <int NORM, int TPR, int SPT>
__device__ __forceinline__ float2 rowstat_merge(const float2 (&p)[SPT], float2 p0, int sub, int K, float eps) {
  const int np = (K + 15) >> 4;
  const float c = NORM == 2 ? p0.x : 0.f;
  float s1 = 0.f, s2 = 0.f, sm = 0.f;
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int idx = sub + i * TPR;
    if (idx < np) {
      const float ni = (float)min(16, K - 16 * idx);
      const float d = p[i].x - c;
      s1 = fmaf(ni, d, s1);
      s2 = fmaf(ni * d, d, s2);
      sm += p[i].y;
    }
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
    sm += __shfl_xor(sm, o, 64);
  }
  const float invk = 1.f / (float)K;
  const float var = NORM == 2 ? fmaxf((sm + s2 - s1 * s1 * invk) * invk, 0.f) : (sm + s2) * invk;
  return make_float2(NORM == 2 ? c + s1 * invk : 0.f, rsqrtf(var + eps));
}

// Widened bf16 store for two horizontally adjacent 16x16 transposed tiles
// (columns nb..nb+15 in a0, nb+16..nb+31 in a1; lane row q = lane>>4 holds
// columns 4q..4q+3 of each).  One v_permlane16_swap per dword pairs lane row
// 0 with 1 and 2 with 3, after which every lane owns 8 contiguous columns:
//   q=0: nb+0..7   q=1: nb+16..23   q=2: nb+8..15   q=3: nb+24..31
// so the tile pair leaves as ONE 16-B store per lane instead of two 8-B
// stores (guide T21: the epilogue tail is store-issue bound).  Preconditions
// (wave-uniform, checked by the caller): nb + 31 < N, 16-B aligned C/ldc and
// bias, 8-B aligned R rows.  Every lane must call it (cross-lane swap).
// The residual rows of a pair, loaded ahead of the epilogue math (RES_PRE):
// lane row q's 4 columns of each tile of the pair.
__device__ __forceinline__ void epi_pair_res_load(int m, int nb, int M, const bf16_t* __restrict__ R, int ldr,
                                                  int lane, bf16x4& r0, bf16x4& r1) {
  const int n0 = nb + (lane >> 4) * 4;
  const int mm = m < M ? m : M - 1;  // rows past M load a valid row (never stored)
  r0 = *reinterpret_cast<const bf16x4*>(R + (size_t)mm * ldr + n0);
  r1 = *reinterpret_cast<const bf16x4*>(R + (size_t)mm * ldr + n0 + 16);
}

// Residual tile of a 256-row GEMM tile by LDS-DMA into the dead operand LDS
// (TN columns, whole rows: one wave-instruction = 1 KB = 1024 / (2 TN) rows),
// 16-B chunk p of row r holding logical chunk p ^ (r & (TN/8 - 1)) (the global
// address is permuted, the LDS write stays lane-linear), so the epilogue's
// 8-B reads of 16 rows x one chunk hit distinct banks.  Rows past M read row
// M - 1 (never stored).  Replaces 32 per-lane 8-B gathers at row stride per
// lane (bench/probes/gemm_anatomy.py --residual: the residual read was ~11 us
// of a 40 us fp8 tile round).
template <int TN>
__device__ __forceinline__ void res_tile_dma(const bf16_t* __restrict__ R, int ldr, int m0, int n0, int M,
                                             char* lds, int wave, int lane) {
  constexpr int CPR = TN / 8, RPI = 1024 / (TN * 2), IPW = 256 / 8 / RPI;
#pragma unroll
  for (int k = 0; k < IPW; ++k) {
    const int rl = (wave * IPW + k) * RPI + lane / CPR;
    const int c = (lane % CPR) ^ (rl & (CPR - 1));
    glds16(R + (size_t)min(m0 + rl, M - 1) * ldr + n0 + c * 8, lds + (wave * IPW + k) * 1024);
  }
}
// the 4 residual values of row rl, tile columns cl..cl+3 (cl % 4 == 0)
template <int TN>
__device__ __forceinline__ bf16x4 res_tile_read(const char* lds, int rl, int cl) {
  constexpr int CPR = TN / 8;
  return *reinterpret_cast<const bf16x4*>(lds + rl * (TN * 2) + (((cl >> 3) ^ (rl & (CPR - 1))) << 4) + (cl & 4) * 2);
}

template <int ACT, bool RES_PRE = false>
__device__ __forceinline__ void epi_pair_bf16(f32x4 a0, f32x4 a1, int m, int nb, int M, bf16_t* __restrict__ C,
                                              int ldc, const float* __restrict__ bias,
                                              const bf16_t* __restrict__ R, int ldr, int lane,
                                              bf16x4 rp0 = bf16x4{}, bf16x4 rp1 = bf16x4{}) {
  const int q = lane >> 4;
  const int n0 = nb + q * 4, n1 = n0 + 16;
  if (bias != nullptr) {
    a0 += *reinterpret_cast<const f32x4*>(bias + n0);
    a1 += *reinterpret_cast<const f32x4*>(bias + n1);
  }
  if constexpr (ACT == ACT_GELU) {
    const f32x2 g0 = gelu_erf2(f32x2{a0[0], a0[1]}), g1 = gelu_erf2(f32x2{a0[2], a0[3]});
    const f32x2 g2 = gelu_erf2(f32x2{a1[0], a1[1]}), g3 = gelu_erf2(f32x2{a1[2], a1[3]});
    a0 = f32x4{g0[0], g0[1], g1[0], g1[1]};
    a1 = f32x4{g2[0], g2[1], g3[0], g3[1]};
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (ACT == ACT_RELU) {
      a0[r] = fmaxf(a0[r], 0.f);
      a1[r] = fmaxf(a1[r], 0.f);
    }
  }
  if (RES_PRE || (R != nullptr && m < M)) {
    bf16x4 r0 = rp0, r1 = rp1;
    if constexpr (!RES_PRE) {
      r0 = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n0);
      r1 = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      a0[r] += bf2f((bf16_t)r0[r]);
      a1[r] += bf2f((bf16_t)r1[r]);
    }
  }
  uint32_t x0 = pack2bf(a0[0], a0[1]), x1 = pack2bf(a0[2], a0[3]);
  uint32_t y0 = pack2bf(a1[0], a1[1]), y1 = pack2bf(a1[2], a1[3]);
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  if (m >= M) return;
  const int c = nb + ((q & 1) << 4) + ((q >> 1) << 3);
  *reinterpret_cast<uint4*>(C + (size_t)m * ldc + c) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

__device__ __forceinline__ bool epi_pair_ok(const void* C, int ldc, const float* bias, const bf16_t* R, int ldr) {
  return ((uintptr_t)C & 15) == 0 && (ldc & 7) == 0 && ((uintptr_t)bias & 15) == 0 &&
         ((uintptr_t)R & 7) == 0 && (R == nullptr || (ldr & 3) == 0);
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

// SwiGLU epilogue of two adjacent 16-column tiles j, j+1 at full lane use: one
// v_permlane32_swap per dword hands lanes 0-31 tile j's (gate, up) and lanes
// 32-63 tile j+1's (epi_silu_t4 exchanged with ds_bpermute and left half the
// lanes idle), and silu is x * rcp(1 + 2^(-x log2 e)) instead of an IEEE
// divide.  Every lane writes output columns ncol0 + 4*(lane>>4) .. +3 of row m
// (ncol0 = tile j's first output column).
template <bool OUT_F32>
__device__ __forceinline__ void epi_silu_pair(const f32x4& a0, const f32x4& a1, int m, int ncol0, int M, int NO,
                                              void* __restrict__ Cv, int ldc, bool vec, int lane) {
  f32x4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0[r]), __float_as_uint(a1[r]), false, false);
    const float g = __uint_as_float(s[0]), u = __uint_as_float(s[1]);
    v[r] = g * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g * -1.4426950408889634f)) * u;
  }
  if (m >= M) return;
  const int ncol = ncol0 + (lane >> 4) * 4;
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
