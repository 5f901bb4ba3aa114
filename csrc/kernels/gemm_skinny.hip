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
// Fused pre-norm (NORM = NORM_RMS / NORM_LN, bf16 only): the producing
// LayerNorm/RMSNorm is folded into the weights on the host (ops/gemm.py
// fold_norm: W' = W diag(gamma), bias' = W beta + bias, colsum[n] = sum_k W'[n,k])
// and the row statistics are accumulated from the A fragments this kernel
// streams anyway, so the norm kernel and its activation round trip disappear:
//   y = rstd[m] * (A W'^T - mean[m] colsum) + bias'   (LN; RMS: no mean term).
//
// bf16: one v_mfma_f32_16x16x32_bf16 per 16-B chunk.  fp8 (OCP e4m3fn weights
// and per-token-quantised activations, ops/fp8.py): two
// v_mfma_f32_16x16x32_fp8_fp8 per chunk (the k order inside a chunk is the same
// permutation for A and W, so the dot product is unchanged); the weight bytes
// and so the step time halve.  KS is chosen on the host so that N/16 x KS waves
// cover the CUs.
#include <algorithm>
#include "gemm_epilogue.h"
#include "gemm_head.h"
#include "gemm_oneshot.h"
#include "gemm_stream.h"

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

enum SkNorm { NORM_NONE = 0, NORM_RMS = 1, NORM_LN = 2 };

typedef float f32x2 __attribute__((ext_vector_type(2)));

// 16 OCP e4m3 weight bytes -> 16 bf16 (exact: every e4m3 value is a bf16
// value).  gfx950's v_cvt_scalef32_pk_bf16_fp8 (scale 1.0) turns two bytes into
// a packed bf16 pair in one op: 8 VALU per 16 B instead of 8 fp32 converts + 8
// repacks — the decode weight stream is VALU-paced at batch 1.
__device__ __forceinline__ void w8_to_bf16(const i32x4& w, bf16x8& lo, bf16x8& hi) {
  bf16x2v o[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[i], 1.0f, false);
    o[2 * i + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[i], 1.0f, true);
  }
  __builtin_memcpy(&lo, &o[0], 16);
  __builtin_memcpy(&hi, &o[4], 16);
}

// Shifted sum and sum of squares of the 8 bf16 of one A fragment: x - c with
// c = the row's first element, so var = E[(x-c)^2] - E[x-c]^2 does not cancel
// catastrophically when |mean| >> std (the unshifted E[x^2] - mean^2 loses
// every bit of the variance once mean^2 / var ~ 2^24).
template <int NORM>
__device__ __forceinline__ void sk_stats(const i32x4& a, float c, float& s1, float& s2) {
  if constexpr (NORM == NORM_RMS) {  // sum of squares only: one v_dot2 per bf16 pair (products exact in fp32)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x2v v = __builtin_bit_cast(bf16x2v, (uint32_t)a[i]);
      s2 = __builtin_amdgcn_fdot2_f32_bf16(v, v, s2, false);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float((uint32_t)a[i] << 16) - c;
    const float hi = __uint_as_float((uint32_t)a[i] & 0xffff0000u) - c;
    s1 += lo + hi;
    s2 = fmaf(lo, lo, fmaf(hi, hi, s2));
  }
}

template <int ACT, bool OUT_F32, int MT, int NT, bool FP8, int U, bool PIPE = false, int NORM = NORM_NONE,
          bool W8 = false, bool MS = false>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const uint8_t* __restrict__ A, int lda_b,
                                                           const float* __restrict__ sa, const uint8_t* __restrict__ W,
                                                           int ldw_b, const float* __restrict__ sw,
                                                           void* __restrict__ Cv, int ldc,
                                                           const float* __restrict__ bias,
                                                           const bf16_t* __restrict__ R, int ldr, int M, int N,
                                                           int kbytes, const float* __restrict__ colsum = nullptr,
                                                           float eps = 0.f, const uint8_t* __restrict__ Wsh = nullptr,
                                                           float2* __restrict__ rs_out = nullptr, int rs_ld = 0,
                                                           int epi_pre = 1) {
  static_assert(NORM == NORM_NONE || !FP8, "fused norm needs bf16 activations");
  static_assert(!(FP8 && W8), "W8 = fp8 weights with bf16 activations; FP8 = both fp8");
  constexpr int AU = W8 ? 2 : 1;        // 16-B A loads per chunk per M tile (W8: a chunk is 64 k = 128 B of A)
  constexpr int ACH = W8 ? 128 : 64;    // A bytes per row per chunk
  extern __shared__ __attribute__((aligned(16))) f32x4 sk_red[];  // [KS][NT*MT][64], then [KS][MT][16] x2 stats
  // wave index via readfirstlane: the K-slice bounds and the surplus-chunk tests
  // below are then scalar (s_cbranch), not exec-masked VALU branches
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), KS = blockDim.x >> 6;
  // MS (M split): one workgroup per (column tile, 16-row M tile), so M = 32..64
  // runs 2-4x the workgroups (narrow N, e.g. GPT-2's 768-wide projections, has
  // too few column tiles to fill 256 CUs otherwise).  The M tiles of a column
  // tile are consecutive logical ids on one XCD, so its weight slice is read
  // from HBM once and re-read from that XCD's L2.
  int n0;
  if constexpr (MS) {
    static_assert(MT == 1, "MS: one M tile per workgroup");
    const int mtiles = (M + 15) >> 4;
    const int lgc = xcd_remap(blockIdx.x, gridDim.x);
    const int mo = (lgc % mtiles) * 16;
    n0 = (lgc / mtiles) * (16 * NT);
    A += (size_t)mo * lda_b;
    if (sa != nullptr) sa += mo;
    Cv = reinterpret_cast<char*>(Cv) + (size_t)mo * ldc * (OUT_F32 ? 4 : 2);
    if (R != nullptr) R += (size_t)mo * ldr;
    if (rs_out != nullptr) rs_out += (size_t)mo * rs_ld;
    M = min(16, M - mo);
  } else {
    n0 = blockIdx.x * (16 * NT);
  }
  const int lg = (lane >> 4) * 16;  // byte offset of this lane group inside a 64-B chunk

  // Wsh != nullptr: W pre-shuffled into MFMA fragment order (ops/gemm.py
  // shuffle_weight): the 16 rows x 64 B of (column tile, chunk) are one
  // contiguous 1 KiB block, lane l's 16 B at l*16, the blocks of one column tile
  // consecutive along K — every wave load is a contiguous 1 KiB and a batch of U
  // chunks one U KiB stream (row-major W: 16 rows x 64 B, 16 DRAM pages per
  // load).  Llama-3 8B at M = 32: -9..-19 % per projection
  // (profiles/archive/r1_skinny_sweep_shuf.jsonl).
  const uint8_t* wp[NT];
  const int wstep = Wsh != nullptr ? 1024 : 64;  // bytes between consecutive chunks of one lane
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    if (Wsh != nullptr) {
      const int ntile = (N + 15) >> 4;
      int tcol = (n0 >> 4) + j;
      tcol = tcol < ntile ? tcol : ntile - 1;
      wp[j] = Wsh + ((size_t)tcol * (size_t)(kbytes >> 6) * 64 + lane) * 16;
    } else {
      int n = n0 + j * 16 + (lane & 15);
      n = n < N ? n : N - 1;
      wp[j] = W + (size_t)n * ldw_b + lg;
    }
  }
  const uint8_t* ap[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    int m = t * 16 + (lane & 15);
    m = m < M ? m : M - 1;
    ap[t] = A + (size_t)m * lda_b + lg * AU;
  }
  // epilogue operands first of all (as gemm_oneshot.h): wave t < MT finishes M
  // tile t after the cross-wave reduction, so it issues that tile's channel
  // scales, column sums, bias and residual now — they land under the main loop
  // and the epilogue pays no memory round trip after the barrier.  Uniform.
  // (14 VGPRs per column tile: only configs with room — the software-pipelined
  // and the wide ones spilled with it)
  constexpr bool PRE = NT <= 2 && MT * NT * U <= 8 && !PIPE && !OUT_F32 && !FP8 && ACT != ACT_SILU_MUL;
  constexpr int NP = PRE ? NT : 1;
  // (MT <= waves: wave t owns M tile t alone in the epilogue loop below, so its
  // prefetched operands are that tile's)
  const bool pre = PRE && epi_pre && wave < MT && MT * 64 <= (int)blockDim.x && (N & 3) == 0 &&
                   epi_vec_ok(Cv, ldc, bias, R, ldr) &&
                   ((reinterpret_cast<uintptr_t>(sw) | reinterpret_cast<uintptr_t>(colsum)) & 15) == 0;
  // unconditional loads (dummy address for absent operands; ``pre`` and
  // has_b / has_r decide use): a load under a branch is waited for at the merge
  f32x4 pre_sw[NP], pre_cs[NP], pre_b[NP];
  bf16x4 pre_r[NP];
  if constexpr (PRE) {
    const float* dummy = reinterpret_cast<const float*>(A);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int nn = min(n0 + j * 16 + (lane >> 4) * 4, N - 4);
      const int mm = min(min(wave, MT - 1) * 16 + (lane & 15), M - 1);
      if constexpr (W8) pre_sw[j] = *reinterpret_cast<const f32x4*>(sw + nn);
      if constexpr (NORM == NORM_LN)
        pre_cs[j] = *reinterpret_cast<const f32x4*>(colsum != nullptr ? colsum + nn : dummy);
      pre_b[j] = *reinterpret_cast<const f32x4*>(bias != nullptr ? bias + nn : dummy);
      pre_r[j] = *reinterpret_cast<const bf16x4*>(R != nullptr ? R + (size_t)mm * ldr + nn
                                                              : reinterpret_cast<const bf16_t*>(dummy));
    }
  }
  f32x4 acc[NT][MT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float st1[MT], st2[MT], shift[MT];  // shifted row statistics of this lane's A fragments (NORM)
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    st1[t] = st2[t] = 0.f;
    shift[t] = 0.f;
    if constexpr (NORM == NORM_LN) {  // RMS has no subtraction to protect: c = 0
      int m = t * 16 + (lane & 15);
      m = m < M ? m : M - 1;
      shift[t] = __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(A + (size_t)m * lda_b)) << 16);
    }
  }

  const int nch = kbytes >> 6;
  const int per = (nch + KS - 1) / KS;
  const int c0 = wave * per, c1 = min(nch, c0 + per);
  // Batches of U chunks; the last batch of a wave is partial: its loads are
  // clamped in-bounds and the surplus chunks' weights zeroed, so every batch
  // (including short K slices) issues all of its loads at once.
  auto load = [&](int cc, i32x4(&wv)[NT][U], i32x4(&av)[MT][U * AU]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ci = min(cc + u, c1 - 1);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const i32x4* src = reinterpret_cast<const i32x4*>(wp[j] + (size_t)ci * wstep);
        // each weight byte is read by exactly one wave of one workgroup (no M
        // split): stream it non-temporally so it does not evict the activations
        // and the next kernel's operands from L2 (guide: nt-weights, 5-10 % per
        // decode layer); with the M split the slice is re-read from L2 by the
        // other M tiles, so keep the default policy there
        wv[j][u] = MS ? *src : __builtin_nontemporal_load(src);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ci = min(cc + u, c1 - 1);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int h = 0; h < AU; ++h)
          av[t][u * AU + h] = *reinterpret_cast<const i32x4*>(ap[t] + (size_t)ci * ACH + 16 * h);
    }
    // keep every load of the batch ahead of the MFMAs that follow (the scheduler
    // would otherwise interleave them and wait vmcnt(0) per chunk)
    __builtin_amdgcn_sched_barrier(0);
  };
  auto comp = [&](int cc, i32x4(&wv)[NT][U], const i32x4(&av)[MT][U * AU]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (cc + u >= c1) {
#pragma unroll
        for (int j = 0; j < NT; ++j) wv[j][u] = i32x4{0, 0, 0, 0};
      } else if constexpr (NORM != NORM_NONE) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int h = 0; h < AU; ++h) sk_stats<NORM>(av[t][u * AU + h], shift[t], st1[t], st2[t]);
      }
      if constexpr (W8) {
        // the lane's 16 weight bytes are k = 16g..16g+15 of the chunk; its two A
        // pieces hold the same k, so MFMA #h pairs W bytes 8h..8h+7 with A piece h
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 wlo, whi;
          w8_to_bf16(wv[j][u], wlo, whi);
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            bf16x8 a0, a1;
            __builtin_memcpy(&a0, &av[t][2 * u], 16);
            __builtin_memcpy(&a1, &av[t][2 * u + 1], 16);
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo, a0, acc[j][t], 0, 0, 0);
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi, a1, acc[j][t], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[j][t] = sk_mma<FP8>(wv[j][u], av[t][u], acc[j][t]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  const int nb = c1 > c0 ? (c1 - c0 + U - 1) / U : 0;
  int c = c0;
  if constexpr (PIPE) {
    // software pipeline: the next batch is in flight while this one computes
    if (nb > 0) {
      i32x4 w0[NT][U], a0[MT][U * AU], w1[NT][U], a1[MT][U * AU];
      load(c, w0, a0);
      int b = 0;
      for (; b + 2 <= nb; b += 2) {
        load(c + U, w1, a1);
        comp(c, w0, a0);
        if (b + 2 < nb) load(c + 2 * U, w0, a0);
        comp(c + U, w1, a1);
        c += 2 * U;
      }
      if (b < nb) comp(c, w0, a0);
    }
  } else {
    for (int b = 0; b < nb; ++b, c += U) {
      i32x4 wv[NT][U], av[MT][U * AU];
      load(c, wv, av);
      comp(c, wv, av);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) sk_red[(wave * NT * MT + j * MT + t) * 64 + lane] = acc[j][t];
  float* sk_st = reinterpret_cast<float*>(sk_red + KS * NT * MT * 64);  // [KS][MT][2][16]
  if constexpr (NORM != NORM_NONE) {
    // the 4 lane groups hold disjoint 16-B pieces of the same 16 rows
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float a = st1[t], q = st2[t];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        sk_st[((wave * MT + t) * 2 + 0) * 16 + lane] = a;
        sk_st[((wave * MT + t) * 2 + 1) * 16 + lane] = q;
      }
    }
  }
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
    // the prefetched residual rows are tile min(wave, MT - 1)'s: only tile t == wave
    // uses them (the column operands pre_sw / pre_cs / pre_b fit every tile)
    const bool pre_t = pre && t == wave;
    if constexpr (W8) {  // per-output-channel weight scale, before the norm terms (colsum is of the dequantised W)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + j * 16 + (lane >> 4) * 4;
        if (pre) {
          s[j] *= n < N ? pre_sw[j % NP] : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) s[j][r] *= n + r < N ? sw[n + r] : 0.f;
        }
      }
    }
    if constexpr (NORM != NORM_NONE) {
      float a = 0.f, q = 0.f;
      for (int w = 0; w < KS; ++w) {
        a += sk_st[((w * MT + t) * 2 + 0) * 16 + (lane & 15)];
        q += sk_st[((w * MT + t) * 2 + 1) * 16 + (lane & 15)];
      }
      const float invk = 1.f / (float)(W8 ? kbytes : kbytes >> 1);
      const float d = a * invk;  // E[x - c]
      // LN: var = E[(x-c)^2] - E[x-c]^2, mean = c + E[x-c]; RMS (c = 0): E[x^2]
      const float mean = NORM == NORM_LN ? shift[t] + d : 0.f;
      const float var = NORM == NORM_LN ? fmaxf(q * invk - d * d, 0.f) : q * invk;
      const float rstd = rsqrtf(var + eps);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (NORM == NORM_LN) {
          const int n = n0 + j * 16 + (lane >> 4) * 4;
          if (pre) {
            s[j] = rstd * (s[j] - mean * (n < N ? pre_cs[j % NP] : f32x4{0.f, 0.f, 0.f, 0.f}));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) s[j][r] = rstd * (s[j][r] - mean * (n + r < N ? colsum[n + r] : 0.f));
          }
        } else {
          s[j] *= rstd;
        }
      }
    }
    if constexpr (ACT == ACT_SILU_MUL) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (FP8) {
          const int n = n0 + j * 16 + (lane >> 4) * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) s[j][r] *= rs * (n + r < N ? sw[n + r] : 0.f);
        }
        epi_silu_t4<OUT_F32>(s[j], m, (n0 + j * 16) / 2, M, N / 2, Cv, ldc, vec, lane);
      }
    } else if (!OUT_F32 && !FP8 && (pre_t || rs_out != nullptr)) {  // uniform
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + j * 16 + (lane >> 4) * 4;
        f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
        if (pre_t && n0 + j * 16 + 15 < N) {  // wave-uniform: the whole 16-column tile
          if (m < M)
            epi_t4_pre<ACT>(s[j], m, n, Cv, ldc, bias != nullptr, pre_b[j % NP], R != nullptr, pre_r[j % NP], &x);
        } else {
          epi_t4<ACT, OUT_F32>(s[j], m, n, M, N, Cv, ldc, bias, R, ldr, vec, nullptr, rs, &x);
        }
        // row-statistics partials of the stored tile
        if (rs_out != nullptr) epi_rowstat16(x, m, n0 + j * 16, M, N, rs_out, rs_ld, lane);
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

constexpr int SKINNY_MAX_M = 256;  // M > 64 only through the M split (medium-batch decode)

// Producer-side row statistics (gemm_epilogue.h
// epi_rowstat16 / rowstat_merge): dnn_gemm_rowstats() arms the NEXT decode
// GEMM call of this thread — ``out`` (float2 [M][ld], ld >= ceil(N/16)): the
// call's kernel writes per-16-column-tile partials of its bf16 output rows;
// ``in``: the partials of the call's input rows, merged instead of deriving
// the pre-norm statistics from the activations.  The request is consumed by
// that call whatever runs; dnn_gemm_rowstats_written() reports whether its
// kernel wrote ``out`` (the one-shot and skinny kernels do; the stream /
// split-K paths do not, and their consumer then derives its own).
struct RowStatReq {
  float2* out = nullptr;
  int out_ld = 0;
  const float2* in = nullptr;
  int in_ld = 0;
};
static thread_local RowStatReq g_rs_req, g_rs_cur;
// decode epilogue operands issued with the first loads (gemm_oneshot.h /
// gemm_skinny_kernel "pre"); 0 = after the reduction, as before (A/B)
static int g_epi_pre = 1;
extern "C" int dnn_gemm_set_epi_prefetch(int on) {
  g_epi_pre = on ? 1 : 0;
  return 0;
}
static thread_local int g_rs_written = 0;

extern "C" int dnn_gemm_rowstats(void* out, int out_ld, const void* in, int in_ld) {
  g_rs_req.out = reinterpret_cast<float2*>(out);
  g_rs_req.out_ld = out_ld;
  g_rs_req.in = reinterpret_cast<const float2*>(in);
  g_rs_req.in_ld = in_ld;
  g_rs_written = 0;
  return 0;
}

// Whether the armed call's kernel wrote the partials; also drops a request no
// decode GEMM consumed (a call that took the prefill path).
extern "C" int dnn_gemm_rowstats_written() {
  g_rs_req = RowStatReq{};
  return g_rs_written;
}

// ---- stream kernel dispatch (gemm_stream.h): 17..64 rows, fragment-order
// weights of >= g_stream_min_bytes; narrow N splits K across workgroups into
// the caller's workspace (no workspace: one slice).
static int g_stream_on = 1;  // 0 off, 1 where it measured faster, 2 forced (tests)
static int g_stream_fold = 0;  // 1: split-K combine inside the launch (last arriver); measured 4.08 -> 4.20 ms (profiles/r3_fold_decode_ab.jsonl)
static constexpr long long STREAM_CNT_BYTES = 4096;  // tile tickets at the end of the workspace (zeroed once)
static long long g_stream_min_bytes = 8ll << 20;

// K-split plan: ntiles x splitk workgroups, cps chunks per slice.  Returns
// false where the stream kernel measured slower than gemm_skinny
// (profiles/r3_stream_ab_*.jsonl, in-pipeline profiles/r3_llama8b_b32_decode_*):
// fewer than 192 workgroups (most CUs idle), fewer than 6 K-steps per slice
// (the prologue latency and the split's reduce launch not amortised), or an
// unsplit K of fewer than 12 steps (small-K wide-N heads: the skinny kernel's
// K-split waves ramp faster).  Measured wins: Llama-3 8B gate|up (no split,
// 224 workgroups x 16 steps) and down (8 slices x 7 steps).
static constexpr int STREAM_NT = 2, STREAM_MIN_STEPS = 6, STREAM_MIN_WGS = 192, STREAM_MAX_SPLIT = 16;

template <bool W8>
static bool stream_plan(int MP, int N, int kbytes, bool have_ws, long long ws_bytes, int& splitk, int& cps) {
  constexpr int BN = 64 * STREAM_NT, CS = StrCfg<W8>::CS;
  const int ntiles = (N + BN - 1) / BN, nch = kbytes / 64, steps = (nch + CS - 1) / CS;
  splitk = 1;
  if (ntiles < STREAM_MIN_WGS && have_ws) {
    const int by_steps = g_stream_on == 2 ? steps : max(1, steps / STREAM_MIN_STEPS);  // forced: split anything
    splitk = min(min((256 + ntiles - 1) / ntiles, STREAM_MAX_SPLIT), by_steps);
    if (g_stream_on == 2) {  // forced (A/B probes): DNN_STREAM_SPLITK pins the split count
      const char* e = getenv("DNN_STREAM_SPLITK");
      if (e != nullptr && atoi(e) > 0) splitk = min(atoi(e), steps);
    }
    auto need = [&](int sk) {
      return (long long)sk * MP * ntiles * BN * 4 + (long long)ntiles * sk * MP * 2 * 4 + STREAM_CNT_BYTES;
    };
    while (splitk > 1 && need(splitk) > ws_bytes) --splitk;
  }
  cps = (steps + splitk - 1) / splitk * CS;
  splitk = (nch + cps - 1) / cps;
  if (g_stream_on == 2) return splitk <= STREAM_MAX_SPLIT;  // forced (tests): every eligible shape
  if (ntiles * splitk < STREAM_MIN_WGS || cps / CS < STREAM_MIN_STEPS) return false;
  return splitk > 1 || steps >= 2 * STREAM_MIN_STEPS;
}

template <int ACT, int NORM, bool W8, int MT>
static int launch_stream_mt(const void* A, int lda_b, const void* Wsh, const float* sw, void* C, int ldc,
                            const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                            const float* colsum, float eps, hipStream_t st, void* ws, long long ws_bytes, int splitk,
                            int cps) {
  constexpr int NT = STREAM_NT, BN = 64 * NT, MP = MT * 16;
  const int ntiles = (N + BN - 1) / BN, nch = kbytes / 64;
  const int kelems = W8 ? kbytes : kbytes / 2;
  const dim3 grid(ntiles * splitk), block(256);
  if (splitk == 1) {
    hipLaunchKernelGGL((gemm_stream_kernel<MT, NT, W8, NORM, ACT, false>), grid, block, 0, st, (const uint8_t*)A,
                       lda_b, (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, nch, cps, colsum,
                       eps, kelems, (float*)nullptr, (unsigned*)nullptr);
    return (int)hipGetLastError();
  }
  if (g_stream_fold) {
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + ws_bytes - STREAM_CNT_BYTES);
    hipLaunchKernelGGL((gemm_stream_kernel<MT, NT, W8, NORM, ACT, true, true>), grid, block, 0, st, (const uint8_t*)A,
                       lda_b, (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, nch, cps, colsum,
                       eps, kelems, (float*)ws, cnt);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_stream_kernel<MT, NT, W8, NORM, ACT, true>), grid, block, 0, st, (const uint8_t*)A, lda_b,
                     (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, nch, cps, colsum, eps, kelems,
                     (float*)ws, (unsigned*)nullptr);
  const int NO = ACT == ACT_SILU_MUL ? N / 2 : N;
  const long long threads = (long long)M * ((NO + 3) / 4);
  hipLaunchKernelGGL((gemm_stream_reduce<ACT, NORM, W8>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     (const float*)ws, splitk, MP, ntiles * BN, (const uint8_t*)A, lda_b, sw, colsum, eps, kelems, C,
                     ldc, bias, (const bf16_t*)R, ldr, M, N, g_epi_pre);
  return (int)hipGetLastError();
}

// ---- one-shot kernel dispatch (gemm_oneshot.h): 17..64 rows, fragment-order
// weights.  A config is (MT rows/16 per workgroup, NTW column tiles, STEPS
// LDS steps per wave, split-K); the plan below is fitted to
// bench/oneshot_sweep.py, and dnn_gemm_set_oneshot can pin a config (A/B).
static int g_os_on = 1;                             // 0 off, 1 planned shapes, 2 every eligible shape (tests)
// LDS floor of a one-shot launch (bytes; 0 = the kernel's own size, so two
// workgroups may share a CU).  Rounds 5-6 kept it above half the CU's 160 KB
// (one workgroup per CU) against a rare few-ulp error seen only with two
// workgroups per CU; that error was the SLP vectoriser's packed subtract
// (gemm_oneshot.h "The race of rounds 5-6", the library now builds this file
// with -fno-slp-vectorize), and the floor measured neutral both ways
// (GPT-2 decode 0.5662 vs 0.5674 ms, XL fp8 3.8187 vs 3.8196 ms,
// profiles/r6_oneshot_race_root_cause.md), so it is off.
static int g_os_lds_floor = 0;
extern "C" int dnn_gemm_set_oneshot_lds_floor(int bytes) {
  g_os_lds_floor = bytes < 0 ? 0 : bytes;
  return 0;
}
static int g_os_pin[4] = {0, 0, 0, 0};              // mt, ntw, steps, splitk (0 = planned)
// race probe (bench/probes/oneshot_race_probe.py): non-null = the instrumented
// ABL 256 variant of the forced LN + GELU shapes (MT 2, STEPS 1, bf16) writes
// one OS_PROBE_WORDS record per workgroup here
static int* g_os_probe = nullptr;
static int g_os_probe_abl = 0;  // 256 detector, 512 entry barrier, 1024 double image sync (gemm_oneshot.h)
extern "C" int dnn_gemm_set_oneshot_probe(void* rec, int abl) {
  g_os_probe = static_cast<int*>(rec);
  g_os_probe_abl = abl;
  return 0;
}

struct OsCfg {
  int mt = 0, ntw = 0, steps = 0, splitk = 1;
};

template <bool W8>
constexpr bool os_fits(int ntw, int steps) {
  return ntw * steps * (W8 ? 4 : 8) <= 32;
}

static long long os_ws_need(const OsCfg& c, int M, int N) {
  if (c.splitk <= 1) return 0;
  const int MP = 16 * c.mt, mgroups = (M + MP - 1) / MP, BN = 16 * c.ntw;
  const long long Ns = (long long)((N + BN - 1) / BN) * BN, MPT = (long long)mgroups * MP;
  return (long long)c.splitk * MPT * Ns * 4 + (long long)c.splitk * MPT * 2 * 4;
}

// The plan (profiles/r4_oneshot_sweep*.jsonl): returns false where gemm_skinny /
// gemm_stream stay.
template <bool W8>
static bool os_plan(int M, int N, int kbytes, bool have_ws, long long ws_bytes, OsCfg& c) {
  const int nch = kbytes / 64, CS = W8 ? 4 : 8;
  if (g_os_pin[0] > 0) {
    c.mt = g_os_pin[0];
    c.ntw = g_os_pin[1];
    c.steps = g_os_pin[2];
    c.splitk = max(1, g_os_pin[3]);
  } else {
    if (g_os_on == 0) return false;
    if (g_os_on == 1) {
      // measured wins (profiles/r4_oneshot_sweep.jsonl, isolated graph-timed
      // launches, weights rotated past the MALL): 33..64 rows, the whole K in
      // one slice — GPT-2 (bf16, K 768): QKV 5.39 -> 4.76, O 3.66 -> 3.10,
      // c_fc 5.46 -> 4.80 us; GPT-2 XL (W8, K 1600): QKV 9.69 -> 8.35, O
      // 5.79 -> 5.00, c_fc 9.70 -> 8.71 us.  Split-K shapes (c_proj K 3072 /
      // 6400, every Llama-3 8B projection at 32 rows) measured slower: they
      // keep gemm_skinny / gemm_stream.
      // the 50304-wide heads measured slower (GPT-2 26.2 -> 36.3 us, XL W8
      // 38.3 -> 47.2 us, profiles/r4_oneshot_heads.jsonl): wide N stays skinny
      if (M <= 32 || N >= 16384 || nch > 4 * (W8 ? 2 : 1) * CS) return false;
      c.splitk = 1;
      c.steps = W8 ? 2 : 1;
      const bool narrow = N <= (W8 ? 2048 : 1024);
      c.mt = narrow ? 1 : 2;
      c.ntw = narrow ? (W8 ? 2 : 1) : (W8 ? 4 : 2);
      return os_fits<W8>(c.ntw, c.steps);
    }
    c.mt = 2;
    const int ntile16 = (N + 15) / 16;
    // chunks per workgroup slice: 4 waves x STEPS x CS
    c.steps = nch <= 4 * CS ? 1 : 2;
    c.splitk = (nch + 4 * c.steps * CS - 1) / (4 * c.steps * CS);
    const int mgroups = (M + 16 * c.mt - 1) / (16 * c.mt);
    c.ntw = 1;
    for (int ntw : {4, 2}) {
      if (os_fits<W8>(ntw, c.steps) && (ntile16 + ntw - 1) / ntw * mgroups * c.splitk >= 256) {
        c.ntw = ntw;
        break;
      }
    }
  }
  if (c.mt != 1 && c.mt != 2 && c.mt != 4) return false;
  if (c.ntw != 1 && c.ntw != 2 && c.ntw != 4) return false;
  if (c.steps != 1 && c.steps != 2) return false;
  if (c.mt == 4 && c.steps == 2) return false;  // 256 KB of LDS
  if (!os_fits<W8>(c.ntw, c.steps)) return false;  // weight registers would spill
  const int per = 4 * c.steps * CS;
  const int cps = (nch + c.splitk - 1) / c.splitk;
  if (cps > per) return false;
  if (c.splitk > 1 && (!have_ws || os_ws_need(c, M, N) > ws_bytes || c.splitk > STR_MAX_SPLIT)) return false;
  return true;
}

template <int MT, int NTW, int STEPS, int ACT, int NORM, bool W8, int ABL = 0>
static int launch_os_cfg(const void* A, int lda_b, const void* Wsh, const float* sw, void* C, int ldc,
                         const float* bias, const void* R, int ldr, int M, int N, int kbytes, const float* colsum,
                         float eps, hipStream_t st, void* ws, int splitk) {
  constexpr int MP = MT * 16, BN = 16 * NTW;
  const int nch = kbytes / 64;
  const int cps = (nch + splitk - 1) / splitk;
  splitk = (nch + cps - 1) / cps;
  const int ntiles = (N + BN - 1) / BN, mgroups = (M + MP - 1) / MP;
  const int kelems = W8 ? kbytes : kbytes / 2;
  const dim3 grid(ntiles * mgroups * splitk), block(256);
  const size_t smem = std::max<size_t>(os_lds_bytes<MT, STEPS>(), (size_t)g_os_lds_floor);
  if (splitk == 1) {
    // row statistics: partials of the output (not for the half-width SwiGLU
    // output); merged partials of the input when they fit OS_RS_SPT per thread
    float2* rso = ACT != ACT_SILU_MUL ? g_rs_cur.out : nullptr;
    const float2* rsi = (NORM != 0 && (kelems + 15) / 16 <= OS_RS_SPT * (256 / MP)) ? g_rs_cur.in : nullptr;
    if constexpr (ABL == 0 && MT == 2 && STEPS == 1 && !W8 && NORM == 2 && ACT == ACT_GELU && NTW <= 2) {
      if (g_os_probe_abl != 0 && rsi == nullptr) {
#define OSP(B)                                                                                                    \
  if (g_os_probe_abl == B) {                                                                                      \
    hipLaunchKernelGGL((gemm_oneshot_kernel<MT, NTW, W8, NORM, ACT, false, STEPS, B>), grid, block, smem, st,      \
                       (const uint8_t*)A, lda_b, (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, \
                       nch, cps, colsum, eps, kelems, (float*)g_os_probe, ntiles, mgroups, nullptr, 0, nullptr, 0,   \
                       g_epi_pre);                                                                                \
    return (int)hipGetLastError();                                                                                \
  }
        OSP(256) OSP(2048) OSP(16384) OSP(32768) OSP(65536)
#undef OSP
        return -2;
      }
    }
    hipLaunchKernelGGL((gemm_oneshot_kernel<MT, NTW, W8, NORM, ACT, false, STEPS, ABL>), grid, block, smem, st,
                       (const uint8_t*)A, lda_b, (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N,
                       nch, cps, colsum, eps, kelems, (float*)nullptr, ntiles, mgroups, rso, g_rs_cur.out_ld, rsi,
                       g_rs_cur.in_ld, g_epi_pre);
    if (rso != nullptr) g_rs_written = 1;
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_oneshot_kernel<MT, NTW, W8, NORM, ACT, true, STEPS>), grid, block, smem, st,
                     (const uint8_t*)A, lda_b, (const uint8_t*)Wsh, sw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, nch,
                     cps, colsum, eps, kelems, (float*)ws, ntiles, mgroups);
  const int NO = ACT == ACT_SILU_MUL ? N / 2 : N;
  const long long threads = (long long)M * ((NO + 3) / 4);
  hipLaunchKernelGGL((gemm_stream_reduce<ACT, NORM, W8>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     (const float*)ws, splitk, mgroups * MP, ntiles * BN, (const uint8_t*)A, lda_b, sw, colsum, eps,
                     kelems, C, ldc, bias, (const bf16_t*)R, ldr, M, N, g_epi_pre);
  return (int)hipGetLastError();
}

template <int ACT, int NORM, bool W8>
static int launch_os(const OsCfg& c, const void* A, int lda_b, const void* Wsh, const float* sw, void* C, int ldc,
                     const float* bias, const void* R, int ldr, int M, int N, int kbytes, const float* colsum,
                     float eps, hipStream_t st, void* ws) {
  // configs whose weight registers (NTW x STEPS x CS x 4 VGPRs) pass 128 spill
  // at the 256-VGPR cap of 2 workgroups per CU: not instantiated
#define OSC(MTV, NTV, SV)                                                                                        \
  if (c.mt == MTV && c.ntw == NTV && c.steps == SV) {                                                          \
    if constexpr (os_fits<W8>(NTV, SV))                                                                         \
      return launch_os_cfg<MTV, NTV, SV, ACT, NORM, W8>(A, lda_b, Wsh, sw, C, ldc, bias, R, ldr, M, N, kbytes,   \
                                                        colsum, eps, st, ws, c.splitk);                         \
    return -3;                                                                                                  \
  }
  OSC(1, 1, 1) OSC(1, 2, 1) OSC(1, 4, 1) OSC(1, 1, 2) OSC(1, 2, 2) OSC(1, 4, 2)
  OSC(2, 1, 1) OSC(2, 2, 1) OSC(2, 4, 1) OSC(2, 1, 2) OSC(2, 2, 2) OSC(2, 4, 2)
  OSC(4, 1, 1) OSC(4, 2, 1) OSC(4, 4, 1)
#undef OSC
  return -3;
}

template <int ACT, int NORM, bool W8>
static bool os_eligible(const void* A, int lda_b, const void* Wsh, int M, int kbytes) {
  if (Wsh == nullptr || M < 17 || M > 64 || kbytes % 64 != 0) return false;
  return ((uintptr_t)A & 15) == 0 && (lda_b & 15) == 0;
}

extern "C" int dnn_gemm_set_oneshot(int on, int mt, int ntw, int steps, int splitk) {
  g_os_on = on;
  g_os_pin[0] = mt;
  g_os_pin[1] = ntw;
  g_os_pin[2] = steps;
  g_os_pin[3] = splitk;
  return 0;
}

// Sweep / A-B entry (bench/oneshot_sweep.py): plain product (no epilogue), an
// explicit config; returns -1 when the config does not apply to the shape.
extern "C" int dnn_gemm_oneshot_sweep(const void* A, int lda, const void* Wsh, const float* sw, void* C, int ldc, int M,
                                      int N, int K, int mt, int ntw, int steps, int splitk, int w8, void* ws,
                                      long long ws_bytes, hipStream_t st) {
  const int kbytes = w8 ? K : K * 2;
  if (!os_eligible<ACT_NONE, 0, false>(A, lda * 2, Wsh, M, kbytes) || (w8 && sw == nullptr)) return -1;
  const int saved[4] = {g_os_pin[0], g_os_pin[1], g_os_pin[2], g_os_pin[3]};
  g_os_pin[0] = mt;
  g_os_pin[1] = ntw;
  g_os_pin[2] = steps;
  g_os_pin[3] = splitk;
  OsCfg c;
  const bool ok = w8 ? os_plan<true>(M, N, kbytes, ws != nullptr, ws_bytes, c)
                     : os_plan<false>(M, N, kbytes, ws != nullptr, ws_bytes, c);
  for (int i = 0; i < 4; ++i) g_os_pin[i] = saved[i];
  if (!ok) return -1;
  return w8 ? launch_os<ACT_NONE, 0, true>(c, A, lda * 2, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N, kbytes, nullptr,
                                           0.f, st, ws)
            : launch_os<ACT_NONE, 0, false>(c, A, lda * 2, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N, kbytes, nullptr,
                                            0.f, st, ws);
}

// Anatomy probe (bench/probes/oneshot_anatomy.py): the planned one-shot
// launch with parts removed (gemm_oneshot_kernel ABL); cfg 0 = 2/4/2 W8 (GPT-2
// XL c_attn, c_fc), 1 = 1/2/2 W8 (XL O), 2 = 2/2/1 bf16 (GPT-2 c_attn, c_fc).
extern "C" int dnn_gemm_oneshot_ablate(const void* A, int lda, const void* Wsh, const float* sw, void* C, int ldc,
                                       int M, int N, int K, int cfg, int abl, hipStream_t st) {
  const bool w8 = cfg != 2;
  const int kbytes = w8 ? K : K * 2, lb = lda * (w8 ? 2 : 2);
  if (!os_eligible<ACT_NONE, 0, false>(A, lb, Wsh, M, kbytes) || (w8 && sw == nullptr)) return -1;
#define ABLC(CFG, MTV, NTV, SV, W8V)                                                                                   \
  if (cfg == CFG) {                                                                                                    \
    switch (abl) {                                                                                                     \
      case 0: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 0>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 1: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 1>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 2: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 2>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 3: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 3>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 4: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 4>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 8: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 8>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 7: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 7>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, N,  \
                                                                     kbytes, nullptr, 0.f, st, nullptr, 1);           \
      case 32: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 32>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, \
                                                                       N, kbytes, nullptr, 0.f, st, nullptr, 1);      \
      case 64: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 64>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, \
                                                                       N, kbytes, nullptr, 0.f, st, nullptr, 1);      \
      case 67: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 67>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, M, \
                                                                       N, kbytes, nullptr, 0.f, st, nullptr, 1);      \
      case 128: return launch_os_cfg<MTV, NTV, SV, ACT_NONE, 0, W8V, 128>(A, lb, Wsh, sw, C, ldc, nullptr, nullptr, 0, \
                                                                         M, N, kbytes, nullptr, 0.f, st, nullptr, 1); \
      default: return -2;                                                                                              \
    }                                                                                                                  \
  }
  ABLC(0, 2, 4, 2, true) ABLC(1, 1, 2, 2, true) ABLC(2, 2, 2, 1, false)
#undef ABLC
  return -2;
}

template <int ACT, int NORM, bool W8>
static bool stream_eligible(const void* A, int lda_b, const void* Wsh, int M, int N, int kbytes) {
  if (!g_stream_on || Wsh == nullptr || M < 17 || M > 64 || kbytes % 64 != 0) return false;
  if (((uintptr_t)A & 15) != 0 || (lda_b & 15) != 0) return false;
  return (long long)((N + 15) / 16 * 16) * kbytes >= g_stream_min_bytes;
}

extern "C" int dnn_gemm_set_stream(int on, long long min_bytes, int fold) {
  g_stream_on = on;
  if (fold >= 0) g_stream_fold = fold;
  if (min_bytes > 0) g_stream_min_bytes = min_bytes;
  return 0;
}

// Per chunk a wave issues NT weight loads and MT activation loads (L2) for
// NT x MT MFMAs.  The configuration table below is fitted to
// bench/skinny_sweep.py on MI355X (profiles/archive/r1_skinny_sweep.jsonl, weights
// rotated past the 256 MB MALL):
//   M <= 8     : 1 tile, 4 chunks in flight, 8 waves/WG (within 3% of the best
//                row-major config on every Llama-3 / GPT-2 XL shape); with the
//                fragment-order copy (Wsh) the per-class rules below
//   M <= 16    : wide N (>= 16K): 4 tiles x 2 chunks, 2 waves; else 2 tiles x 2
//                chunks pipelined, 4 waves
//   M <= 64    : by N class (wide >= 16K / mid / narrow <= 4K): 4 / 2 / 1 column
//                tiles x 2 chunks, 4 waves (activation re-reads dominate as M
//                grows, so narrow N keeps one column tile for more workgroups)
// A/B pin of the M 17..64 bf16 fragment-order configuration (bench/probes/decode_ab.py
// --switch skinny_pin): one of the table's template configurations with any wave
// count, for the calls of width N (0: every width); id 0 = the table below.
// A pinned shape also bypasses the one-shot and stream plans (k: its K in
// elements, 0 = any).
struct SkinnyPin {
  int id = 0, ks = 4, n = 0, k = 0;
};
static SkinnyPin g_skinny_pin;
extern "C" int dnn_gemm_set_skinny_pin(int id, int ks, int n, int k) {
  if (id < 0 || id > 6 || ks < 1 || ks > 8) return -1;
  g_skinny_pin = SkinnyPin{id, ks, n, k};
  return 0;
}

template <int ACT, bool F32, bool FP8, int MT, int NT, int U, bool PIPE, int NORM, bool W8, bool MS = false>
static int launch_skinny_cfg(const void* A, int lda_b, const float* sa, const void* W, int ldw_b, const float* sw,
                             void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                             int ks, const float* colsum, float eps, hipStream_t st, const void* Wsh) {
  const int groups = (N + 16 * NT - 1) / (16 * NT) * (MS ? (M + 15) / 16 : 1);
  while (ks > 1 && kbytes / 64 < ks) ks >>= 1;
  size_t smem = (size_t)ks * NT * MT * 64 * sizeof(f32x4);
  if (NORM != NORM_NONE) smem += (size_t)ks * MT * 2 * 16 * sizeof(float);
  float2* rso = (!F32 && !FP8 && ACT != ACT_SILU_MUL) ? g_rs_cur.out : nullptr;
  hipLaunchKernelGGL((gemm_skinny_kernel<ACT, F32, MT, NT, FP8, U, PIPE, NORM, W8, MS>), dim3(groups), dim3(64 * ks), smem,
                     st, (const uint8_t*)A, lda_b, sa, (const uint8_t*)W, ldw_b, sw, C, ldc, bias, (const bf16_t*)R,
                     ldr, M, N, kbytes, colsum, eps, (const uint8_t*)Wsh, rso, g_rs_cur.out_ld, g_epi_pre);
  if (rso != nullptr) g_rs_written = 1;
  return (int)hipGetLastError();
}

template <int ACT, bool F32, bool FP8, int NORM = NORM_NONE, bool W8 = false>
static int launch_skinny(const void* A, int lda_b, const float* sa, const void* W, int ldw_b, const float* sw,
                         void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int kbytes,
                         hipStream_t st, const float* colsum = nullptr, float eps = 0.f,
                         const void* Wsh = nullptr, void* ws = nullptr, long long ws_bytes = 0) {
  // this call consumes the row-statistics request (dnn_gemm_rowstats); it is
  // in effect for this call's launch only
  struct Scope {
    ~Scope() { g_rs_cur = RowStatReq{}; }
  } scope;
  g_rs_cur = g_rs_req;
  g_rs_req = RowStatReq{};
  g_rs_written = 0;
  const bool pin_any = g_skinny_pin.id != 0 && (g_skinny_pin.n == 0 || g_skinny_pin.n == N) &&
                       (g_skinny_pin.k == 0 || g_skinny_pin.k * 2 == kbytes);
  if constexpr (!F32 && !FP8 && ACT != ACT_RELU) if (!pin_any) {
    OsCfg oc;
    if (os_eligible<ACT, NORM, W8>(A, lda_b, Wsh, M, kbytes) && os_plan<W8>(M, N, kbytes, ws != nullptr, ws_bytes, oc))
      return launch_os<ACT, NORM, W8>(oc, A, lda_b, Wsh, sw, C, ldc, bias, R, ldr, M, N, kbytes, colsum, eps, st, ws);
    int splitk = 1, cps = 0;
    if (stream_eligible<ACT, NORM, W8>(A, lda_b, Wsh, M, N, kbytes) &&
        stream_plan<W8>(M <= 32 ? 32 : 64, N, kbytes, ws != nullptr, ws_bytes, splitk, cps)) {
      if (M <= 32)
        return launch_stream_mt<ACT, NORM, W8, 2>(A, lda_b, Wsh, sw, C, ldc, bias, R, ldr, M, N, kbytes, colsum, eps,
                                                  st, ws, ws_bytes, splitk, cps);
      return launch_stream_mt<ACT, NORM, W8, 4>(A, lda_b, Wsh, sw, C, ldc, bias, R, ldr, M, N, kbytes, colsum, eps,
                                                st, ws, ws_bytes, splitk, cps);
    }
  }
  const bool wide = N >= 16384;
#define CFG(MTV, NTV, UV, PV, KSV)                                                                                   \
  return launch_skinny_cfg<ACT, F32, FP8, MTV, NTV, UV, PV, NORM, W8>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, R,   \
                                                                       ldr, M, N, kbytes, KSV, colsum, eps, st, Wsh)
#define CFG_MS(NTV, UV, PV, KSV)                                                                                 \
  return launch_skinny_cfg<ACT, F32, FP8, 1, NTV, UV, PV, NORM, W8, true>(A, lda_b, sa, W, ldw_b, sw, C, ldc, bias, \
                                                                           R, ldr, M, N, kbytes, KSV, colsum, eps, st, \
                                                                           Wsh)
  const bool pinned = g_skinny_pin.id != 0 && !FP8 && !W8 && Wsh != nullptr && M > 16 && M <= 64 &&
                      (g_skinny_pin.n == 0 || g_skinny_pin.n == N) &&
                      (g_skinny_pin.k == 0 || g_skinny_pin.k * 2 == kbytes);
  if (pinned) {
    const int pk = g_skinny_pin.ks;
    switch (g_skinny_pin.id) {  // (MT, NT, U, PIPE) / M-split (NT, U, PIPE) of the table
      case 1: CFG(2, 1, 2, false, pk);
      case 2: CFG(2, 1, 8, false, pk);
      case 3: CFG(2, 2, 2, true, pk);
      case 4: CFG(2, 4, 2, false, pk);
      case 5: CFG_MS(2, 4, false, pk);
      case 6: CFG_MS(1, 4, false, pk);
      default: break;
    }
  }
  // medium M (64, 256], decode of larger batches: always the M split, one
  // 16-row tile per workgroup; the weight slice of a column tile is re-read
  // from its XCD's L2 by the M tiles (the 128^2 GEMM would launch only a
  // handful of tiles at these shapes)
  if (M > 64) {
    if (N <= 1024) CFG_MS(1, 4, false, 4);
    CFG_MS(2, 2, false, 4);
  }
  if (M <= 8) {
    // batch 1-8: the fragment-order copy (Wsh) is streamed whenever the layer
    // attached one; per shape class: QKV-sized N 1 tile x 4 chunks on 4 waves
    // (Llama-3 8B fp8 decode graph 12.25 -> 10.33 us), the rest below
    if (!FP8 && Wsh != nullptr && N > 4096 && N < 16384 && kbytes <= 8192) CFG(1, 1, 4, false, 4);
    // fp8 vocabulary head (128K x 4K, fragment order): 2 column tiles per wave
    // 83.3 -> 75.8 us, 6.9 TB/s (profiles/archive/r2_skinny_sweep_w8_m1.jsonl)
    if (W8 && Wsh != nullptr && N >= 65536) CFG(1, 2, 4, false, 8);
    // fp8 gate|up (28K x 4K) with the fused RMSNorm: 2 column tiles x 2 chunks
    // on 2 waves 23.3 -> 21.3 us (profiles/archive/r2_w8_decode_projections.jsonl)
    if (W8 && Wsh != nullptr && N >= 16384) CFG(1, 2, 2, false, 2);
    CFG(1, 1, 4, false, 8);
  }
  if (M <= 16) {
    if (wide) CFG(1, 4, 2, false, 2);
    CFG(1, 2, 2, true, 4);
  }
  // M in (16, 64]: profiles/archive/r1_skinny_sweep.jsonl + r1_skinny_sweep_m32_m64.jsonl
  // (bf16 and W8 on the GPT-2 / GPT-2 XL / Llama-3 shapes), checked in the decode
  // pipeline: wide N streams 4 column tiles on 2 waves, deep K (bf16 >= 8K) 1 tile
  // x 8 chunks on 2 waves, narrow N one column tile on 4 waves (more workgroups)
  // M split (one 16-row tile per workgroup) where the column tiles alone are
  // too few for 256 CUs: graph-timed sweep profiles/archive/r1_skinny_sweep_ms.jsonl —
  // GPT-2 N=768: 5.8 -> 3.8 us (K=768), 15.9 -> 8.3 us (K=3072) at M=64;
  // GPT-2 XL W8 N=1600: 9.8 -> 7.0 / 28.5 -> 16.0 us; Llama W8 N=4096 at M=32.
  if (!FP8 && Wsh != nullptr) {
    // fragment-order weights (M 17..64): graph-timed sweep profiles/archive/r1_skinny_sweep_shuf_fit.jsonl,
    // every rule within 1.0-1.1x of the best config of its shapes (Llama-3 8B at M = 32,
    // GPT-2 at M = 64, GPT-2 XL W8 at M = 64)
    if (wide) {
      if (M <= 32) CFG(2, 4, 2, false, 2);
      CFG(4, 4, 2, false, 2);
    }
    if (N <= 1024) CFG_MS(1, 4, false, 4);
    // (8-wave variants of the Llama-3 8B B=32 QKV / O rules below measured within
    // noise in one process, decode_ab.py --switch skinny_pin, profiles/r6_skinny_pin_ab.jsonl)
    if (!W8 && N > 4096 && M <= 32) CFG(2, 2, 2, true, 4);  // Llama QKV (6144)
    if (W8 && N > 4096) CFG_MS(4, 2, false, 4);
    if (kbytes >= 8192) CFG_MS(2, 4, false, 4);
    CFG_MS(2, 2, false, 4);
  }
  if (!FP8) {
    if (N <= 1024) CFG_MS(1, 2, true, 4);
    if (N <= 2048 || (W8 && N <= 4096)) CFG_MS(2, 2, true, 4);
  }
#undef CFG_MS
  const bool deep = kbytes >= 16384;
  const bool narrow = N <= 4096;
  if (M <= 32) {
    if (wide) CFG(2, 4, 2, false, 2);
    if (deep) CFG(2, 1, 8, false, 2);
    if (narrow) CFG(2, 1, 2, false, 4);
    CFG(2, 2, 2, true, 4);
  }
  if (wide) CFG(4, 4, 2, false, 2);
  if (deep) CFG(4, 1, 8, false, 2);
  if (narrow) CFG(4, 1, 2, false, 4);
  CFG(4, 2, 2, false, 4);
#undef CFG
}

// bf16: K % 32 == 0 (64-B chunks), M <= SKINNY_MAX_M (M > 64: M split).  fp8: K (bytes) % 64 == 0, M <= 64.
extern "C" int dnn_gemm_skinny(const void* A, int lda, const float* sa, const void* W, int ldw, const float* sw,
                               void* C, int ldc, const float* bias, const void* R, int ldr, int M, int N, int K,
                               int act, int out_f32, int fp8, hipStream_t st, const void* Wsh, void* ws,
                               long long ws_bytes) {
  const int eb = fp8 ? 1 : 2;
  const int kbytes = K * eb;
  if (M <= 0 || M > (fp8 ? 64 : SKINNY_MAX_M) || N <= 0 || kbytes % 64 != 0) return -1;
  if (act == ACT_SILU_MUL && N % 16 != 0) return -1;  // packed gate|up groups of 8+8
  if (fp8 && (sa == nullptr || sw == nullptr)) return -1;
  const int la = lda * eb, lw = ldw * eb;
#define SKD(a)                                                                                              \
  if (act == a) {                                                                                           \
    if (fp8) {                                                                                              \
      return out_f32 ? launch_skinny<a, true, true>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st,  \
                                                    nullptr, 0.f, Wsh)                                        \
                     : launch_skinny<a, false, true>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st, \
                                                     nullptr, 0.f, Wsh);                                      \
    }                                                                                                       \
    return out_f32 ? launch_skinny<a, true, false>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st,   \
                                                   nullptr, 0.f, Wsh)                                         \
                   : launch_skinny<a, false, false>(A, la, sa, W, lw, sw, C, ldc, bias, R, ldr, M, N, kbytes, st,  \
                                                    nullptr, 0.f, Wsh, ws, ws_bytes);                         \
  }
  SKD(ACT_NONE)
  SKD(ACT_RELU)
  SKD(ACT_GELU)
  SKD(ACT_SILU_MUL)
#undef SKD
  return -2;
}

// Pre-norm fused skinny GEMM (bf16): y = act(rstd (A W'^T - mean colsum) + bias) (+ R),
// norm = 1 RMSNorm, 2 LayerNorm (colsum required); W', bias', colsum from
// ops/gemm.py fold_norm.  act: NONE / GELU / SILU_MUL.
extern "C" int dnn_gemm_skinny_norm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                                    const void* R, int ldr, int M, int N, int K, int act, int norm,
                                    const float* colsum, float eps, hipStream_t st, const void* Wsh, void* ws,
                                    long long ws_bytes) {
  const int kbytes = K * 2;
  if (M <= 0 || M > SKINNY_MAX_M || N <= 0 || kbytes % 64 != 0) return -1;
  if (act == ACT_SILU_MUL && N % 16 != 0) return -1;
  if (norm == NORM_LN && colsum == nullptr) return -1;
  const int la = lda * 2, lw = ldw * 2;
#define SKN(a, nm)                                                                                                   \
  if (act == a && norm == nm)                                                                                        \
    return launch_skinny<a, false, false, nm>(A, la, nullptr, W, lw, nullptr, C, ldc, bias, R, ldr, M, N, kbytes, st, \
                                              colsum, eps, Wsh, ws, ws_bytes);
  SKN(ACT_NONE, NORM_RMS)
  SKN(ACT_SILU_MUL, NORM_RMS)
  SKN(ACT_NONE, NORM_LN)
  SKN(ACT_GELU, NORM_LN)
#undef SKN
  return -2;
}

// Weight-only fp8 (W8A16) skinny GEMM: W OCP e4m3 [N, ldw bytes] with per-channel
// scales sw, A bf16, bf16 MFMA on the exactly-converted weights; half the
// weight bytes of bf16 with the bf16 pipeline's epilogues and fused pre-norm
// (norm 0 = none).  K % 64 == 0 (logical K; the weight rows may be padded).
extern "C" int dnn_gemm_skinny_w8(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc,
                                  const float* bias, const void* R, int ldr, int M, int N, int K, int act, int norm,
                                  const float* colsum, float eps, hipStream_t st, const void* Wsh, void* ws,
                                  long long ws_bytes) {
  if (M <= 0 || M > SKINNY_MAX_M || N <= 0 || K % 64 != 0 || ldw < K || sw == nullptr) return -1;
  if (act == ACT_SILU_MUL && N % 16 != 0) return -1;
  if (norm == NORM_LN && colsum == nullptr) return -1;
  const int la = lda * 2;
#define SKW(a, nm)                                                                                                    \
  if (act == a && norm == nm)                                                                                         \
    return launch_skinny<a, false, false, nm, true>(A, la, nullptr, W, ldw, sw, C, ldc, bias, R, ldr, M, N, K, st,     \
                                                    colsum, eps, Wsh, ws, ws_bytes);
  SKW(ACT_NONE, NORM_NONE)
  SKW(ACT_NONE, NORM_RMS)
  SKW(ACT_SILU_MUL, NORM_RMS)
  SKW(ACT_NONE, NORM_LN)
  SKW(ACT_GELU, NORM_LN)
#undef SKW
  return -2;
}

// Configuration sweep for bench/skinny_sweep.py (no epilogue ops): nt in
// {1,2,4}, u in {2,4,8}, pipe in {0,1}; ks = waves per workgroup; w8 = fp8
// weights (W8A16, sw = channel scales) instead of bf16.
template <int MT, int NT, int U, bool PIPE, bool W8, bool MS = false, bool SHUF = false>
static int skinny_sweep_launch(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc,
                               int M, int N, int K, int ks, hipStream_t st) {
  // SHUF: W points at the pre-shuffled copy
  const int groups = (N + 16 * NT - 1) / (16 * NT) * (MS ? (M + 15) / 16 : 1);
  const size_t smem = (size_t)ks * NT * MT * 64 * sizeof(f32x4);
  hipLaunchKernelGGL((gemm_skinny_kernel<ACT_NONE, false, MT, NT, false, U, PIPE, NORM_NONE, W8, MS>),
                     dim3(groups),
                     dim3(64 * ks), smem, st, (const uint8_t*)A, lda * 2, nullptr, (const uint8_t*)W,
                     W8 ? ldw : ldw * 2, sw, C, ldc, nullptr, nullptr, 0, M, N, W8 ? K : K * 2, nullptr, 0.f,
                     SHUF ? (const uint8_t*)W : nullptr);
  return (int)hipGetLastError();
}

template <int MT, bool W8, bool SHUF = false>
static int skinny_sweep_mt(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc, int M,
                           int N, int K, int nt, int u, int ks, int pipe, hipStream_t st) {
#define SW(NTV, UV)                                                                                                  \
  if (nt == NTV && u == UV)                                                                                          \
    return pipe ? skinny_sweep_launch<MT, NTV, UV, true, W8, false, SHUF>(A, lda, W, ldw, sw, C, ldc, M, N, K, ks, st) \
                : skinny_sweep_launch<MT, NTV, UV, false, W8, false, SHUF>(A, lda, W, ldw, sw, C, ldc, M, N, K, ks, st);
  SW(1, 2) SW(1, 4) SW(1, 8) SW(2, 2) SW(2, 4) SW(2, 8) SW(4, 2) SW(4, 4)
#undef SW
  return -2;
}

template <bool W8, bool SHUF = false>
static int skinny_sweep_ms(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc, int M,
                           int N, int K, int nt, int u, int ks, int pipe, hipStream_t st) {
#define SW(NTV, UV)                                                                                                  \
  if (nt == NTV && u == UV)                                                                                          \
    return pipe ? skinny_sweep_launch<1, NTV, UV, true, W8, true, SHUF>(A, lda, W, ldw, sw, C, ldc, M, N, K, ks, st) \
                : skinny_sweep_launch<1, NTV, UV, false, W8, true, SHUF>(A, lda, W, ldw, sw, C, ldc, M, N, K, ks, st);
  SW(1, 2) SW(1, 4) SW(1, 8) SW(2, 2) SW(2, 4) SW(2, 8) SW(4, 2) SW(4, 4)
#undef SW
  return -2;
}

// pipe bit 0: software pipeline; bit 1: M split (MS); bit 2: pre-shuffled W (SHUF)
extern "C" int dnn_gemm_skinny_sweep(const void* A, int lda, const void* W, int ldw, const float* sw, void* C,
                                     int ldc, int M, int N, int K, int nt, int u, int ks, int pipe, int w8,
                                     hipStream_t st) {
  if (M <= 0 || M > 64 || K % 64 != 0 || ks < 1 || ks > 8 || (w8 && sw == nullptr)) return -1;
  if ((pipe & 6) == 6) {  // pre-shuffled weights + M split
    pipe &= 1;
    return w8 ? skinny_sweep_ms<true, true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st)
              : skinny_sweep_ms<false, true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st);
  }
  if (pipe & 4) {  // pre-shuffled weights (no M split)
    pipe &= 1;
#define SWS(MTV)                                                                                                 \
  return w8 ? skinny_sweep_mt<MTV, true, true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st)        \
            : skinny_sweep_mt<MTV, false, true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st);
    if (M <= 16) SWS(1)
    if (M <= 32) SWS(2)
    SWS(4)
#undef SWS
  }
  if (pipe & 2) {  // M split: one 16-row tile per workgroup
    pipe &= 1;
    return w8 ? skinny_sweep_ms<true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st)
              : skinny_sweep_ms<false>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st);
  }
#define SWM(MTV)                                                                                  \
  return w8 ? skinny_sweep_mt<MTV, true>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st) \
            : skinny_sweep_mt<MTV, false>(A, lda, W, ldw, sw, C, ldc, M, N, K, nt, u, ks, pipe, st);
  if (M <= 16) SWM(1)
  if (M <= 32) SWM(2)
  SWM(4)
#undef SWM
}

namespace dnn {

// ---- decode vocabulary head (gemm_head.h): logits + per-workgroup argmax partials
static int g_head_on = 1;

extern "C" int dnn_gemm_set_head(int on) {
  g_head_on = on;
  return 0;
}

static int head_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cus[dev] = v;
  }
  return cus[dev];
}

template <bool W8, int NORM, int NCH, int CPP, int GS>
static int launch_head_cfg(const void* A, int lda_b, const void* Wsh, const float* sw, const float* colsum,
                           const float* bias, float eps, void* C, int ldc, int M, int N, int K, int grid, void* part,
                           hipStream_t st) {
  constexpr size_t smem = head_lds_bytes<W8, NCH, CPP, GS>();
  hipLaunchKernelGGL((gemm_head_kernel<W8, NORM, NCH, CPP, GS>), dim3(grid), dim3(512), smem, st, (const uint8_t*)A, lda_b, (const uint8_t*)Wsh, sw, colsum,
                     bias, eps, (bf16_t*)C, ldc, M, N, K, (int2*)part);
  return (int)hipGetLastError();
}

template <int NORM>
static int launch_head(bool w8, int nch, const void* A, int lda_b, const void* Wsh, const float* sw,
                       const float* colsum, const float* bias, float eps, void* C, int ldc, int M, int N, int K,
                       int grid, void* part, hipStream_t st) {
  // (weight chunks, chunks per K pass, chunks per load group): the LDS image is
  // 64 rows x CPP chunks of activations (<= 128 KiB); GPT-2 family widths
#define HEADC(W8V, NCHV, CPPV, GSV)                                                                             \
  if (w8 == W8V && nch == NCHV)                                                                                 \
    return launch_head_cfg<W8V, NORM, NCHV, CPPV, GSV>(A, lda_b, Wsh, sw, colsum, bias, eps, C, ldc, M, N, K, grid, \
                                                      part, st);
  HEADC(false, 8, 8, 8)     // gpt2-tiny (d 256)
  HEADC(false, 24, 24, 12)  // gpt2 (d 768)
  HEADC(false, 32, 32, 8)   // gpt2-medium (d 1024)
  HEADC(false, 40, 20, 10)  // gpt2-large (d 1280), 2 K passes
  HEADC(false, 50, 28, 7)   // gpt2-xl bf16 (d 1600), 2 K passes
  HEADC(true, 4, 4, 4)      // gpt2-tiny fp8
  HEADC(true, 12, 12, 4)    // gpt2 fp8
  HEADC(true, 16, 16, 4)    // gpt2-medium fp8
  HEADC(true, 20, 10, 5)    // gpt2-large fp8, 2 K passes
  HEADC(true, 25, 14, 5)    // gpt2-xl fp8 (d 1600), 2 K passes
#undef HEADC
  return -3;
}

// Returns the number of partials per row (the grid, > 0), or < 0 when the
// shape is not covered (the caller runs the GEMM + argmax_rows instead).
// part: >= M x part_cap int2; C: bf16 [M, ldc], ldc % 4 == 0.
extern "C" int dnn_gemm_head(const void* A, int lda, const void* Wsh, const float* sw, const float* colsum,
                             const float* bias, float eps, int norm, void* C, int ldc, int M, int N, int K, int w8,
                             void* part, int part_cap, hipStream_t st) {
  if (!g_head_on || M < 1 || M > 64 || N < 16 || Wsh == nullptr || part == nullptr || C == nullptr) return -1;
  if ((w8 && sw == nullptr) || (norm == NORM_LN && colsum == nullptr) || norm < 0 || norm > 2) return -1;
  if (((uintptr_t)A & 15) != 0 || ((lda * 2) & 15) != 0 || ((uintptr_t)C & 7) != 0 || (ldc & 3) != 0 || ldc < N)
    return -1;
  if (K <= 0 || K % (w8 ? 64 : 32) != 0) return -1;
  const int nch = w8 ? K / 64 : K / 32;
  const int ntile16 = (N + 15) / 16;
  const int cus = head_cus();
  if (cus <= 0) return -1;
  int grid = (ntile16 + 7) / 8;
  grid = grid < cus ? grid : cus;
  if ((long long)grid * 16 < ntile16 || grid > part_cap) return -1;  // at most two column tiles per wave
  int rc;
  if (norm == NORM_LN)
    rc = launch_head<NORM_LN>(w8 != 0, nch, A, lda * 2, Wsh, sw, colsum, bias, eps, C, ldc, M, N, K, grid, part, st);
  else if (norm == NORM_RMS)
    rc = launch_head<NORM_RMS>(w8 != 0, nch, A, lda * 2, Wsh, sw, colsum, bias, eps, C, ldc, M, N, K, grid, part, st);
  else
    rc = launch_head<NORM_NONE>(w8 != 0, nch, A, lda * 2, Wsh, sw, colsum, bias, eps, C, ldc, M, N, K, grid, part,
                                st);
  if (rc == -3) return -1;
  return rc != 0 ? -2 : grid;
}

}  // namespace dnn
