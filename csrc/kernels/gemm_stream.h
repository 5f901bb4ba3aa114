// Weight-streaming decode GEMM for 17..64 rows with large weights ("stream"
// kernel): C[M,N] = epi(A[M,K] . W[N,K]^T), W in the skinny kernel's fragment
// order (ops/gemm.py shuffle_weight), bf16 or OCP e4m3 (W8A16).
//
// Why a second decode GEMM: gemm_skinny splits K over the waves of a workgroup,
// so every wave loads its own A fragments (16 rows x 64 B per instruction)
// straight to VGPRs, and with the M split each weight slice is re-read by 2-4
// workgroups.  At 32-64 rows that puts 3-6x the weight bytes through each CU's
// load path (guide §5, "x operand through LDS in full lines": fragment-shaped
// x +18..45 %), and Llama-3 8B B=32 projections stream at 3-4.8 TB/s.
// Here:
//   * a workgroup owns BN = 64 NT output columns (4 waves x NT 16-column
//     tiles) and ONE K range; the waves share the A rows of that range, staged
//     through LDS in full 512-B row segments (global_load_dwordx4 -> ds_write),
//     so A crosses the load path once per workgroup: A : W bytes = M : BN;
//   * each wave streams its own weight tiles straight to VGPRs (guide: GEMV
//     row — no LDS round trip), non-temporally (read once), two K-steps of
//     weights in flight (16 KiB per wave);
//   * narrow N is split over K across workgroups (SPLIT): fp32 partial slabs
//     [splitk][Mp][Ns] in a caller workspace, summed by gemm_stream_reduce with
//     the epilogue (bias / act / residual / fused norm / fp8 channel scale).
//
// LDS image of one A step: Mp rows x 512 B, 16-B slot j of row r stored at
// j ^ (r & 15): conflict-free for the 4 ds_read_b128 lane groups of every
// fragment read (bf16: slot 4c+g, W8: 8c+2g+h) and for the ds_write_b128 of
// the staging pass (checked exhaustively offline).
//
// Fused pre-norm (NORM_RMS / NORM_LN, weights folded on the host, gemm_skinny
// header): row statistics are accumulated from the A fragments, by wave t for
// M tile t; LN statistics are shifted by the row's first element (the same
// shift in every K slice, so slices add).
#pragma once
#include <type_traits>

#include "gemm_epilogue.h"

namespace dnn {

constexpr int STR_SB = 512;  // A bytes per row per K-step (bf16: 8 chunks of 32 k; W8: 4 chunks of 64 k)

template <bool W8>
struct StrCfg {
  static constexpr int ACH = W8 ? 128 : 64;  // A bytes per row per 64-B weight chunk
  static constexpr int CS = STR_SB / ACH;    // weight chunks per K-step
  static constexpr int AU = W8 ? 2 : 1;      // 16-B A pieces per chunk per lane
};

template <int NORM>
__device__ __forceinline__ void str_stats(const bf16x8& a, float c, float& s1, float& s2) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = bf2f_s(a[i]) - c;
    if constexpr (NORM == 2) s1 += x;
    s2 = fmaf(x, x, s2);
  }
}

// Write-through (sc1) stores and L1-bypassing (sc1) loads of split-K partials:
// relaxed agent-scope 8-byte atomics on global (addrspace 1) pointers lower to
// global_store_dwordx2 sc1 / global_load_dwordx2 sc1 (MI355X_MICROARCH.md,
// visibility: the forms that need no release / acquire fence).
typedef GLB_AS unsigned long long gu64_t;
__device__ __forceinline__ void str_store_sc1(float* p, const f32x4& v) {
  gu64_t* q = (gu64_t*)(p);  // C-style: an address-space cast (flat -> global)
  __hip_atomic_store(q, __builtin_bit_cast(unsigned long long, f32x2{v[0], v[1]}), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, __builtin_bit_cast(unsigned long long, f32x2{v[2], v[3]}), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void str_store_sc1_2(float* p, float a, float b) {
  __hip_atomic_store((gu64_t*)(p),
                     __builtin_bit_cast(unsigned long long, f32x2{a, b}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SC1>
__device__ __forceinline__ f32x2 str_load2(const float* p) {
  if constexpr (SC1) {
    const unsigned long long x = __hip_atomic_load((gu64_t*)(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_bit_cast(f32x2, x);
  } else {
    return *reinterpret_cast<const f32x2*>(p);
  }
}

constexpr int STR_MAX_SPLIT = 16;

// Row statistics (mean, rstd) of row m from the per-slice partial sums of
// (tile `tile`'s copy in) the statistics region.
template <int NORM, bool SC1>
__device__ __forceinline__ void str_row_norm(const float* st, int splitk, int MP, int tile, int m,
                                             const uint8_t* __restrict__ A, int lda_b, int kelems, float eps,
                                             float& mean, float& rstd) {
  float a = 0.f, q = 0.f;
  for (int s = 0; s < splitk; ++s) {
    const f32x2 v = str_load2<SC1>(st + (((size_t)tile * splitk + s) * MP + m) * 2);
    a += v[0];
    q += v[1];
  }
  const float invk = 1.f / (float)kelems, d = a * invk;
  const float sh = NORM == 2 ? bf2f(*reinterpret_cast<const bf16_t*>(A + (size_t)m * lda_b)) : 0.f;
  mean = NORM == 2 ? sh + d : 0.f;
  const float var = NORM == 2 ? fmaxf(q * invk - d * d, 0.f) : q * invk;
  rstd = rsqrtf(var + eps);
}

// Sum of the splitk partials of outputs (m, n..n+3): every slice's partial is
// loaded before the first add (surplus loads clamped to the last slice and
// weighted 0): one memory round trip, not splitk dependent ones.  Then the fp8
// channel scale and the folded norm.
template <int NORM, bool W8, bool SC1>
__device__ __forceinline__ f32x4 str_combine4(const float* slab, int splitk, int MP, int Ns, int m, int n, int N,
                                              const float* __restrict__ sw, const float* __restrict__ colsum,
                                              float mean, float rstd) {
  f32x2 part[STR_MAX_SPLIT][2];
#pragma unroll
  for (int s = 0; s < STR_MAX_SPLIT; ++s) {
    const float* p = slab + ((size_t)min(s, splitk - 1) * MP + m) * Ns + n;
    part[s][0] = str_load2<SC1>(p);
    part[s][1] = str_load2<SC1>(p + 2);
  }
  f32x4 v = f32x4{part[0][0][0], part[0][0][1], part[0][1][0], part[0][1][1]};
#pragma unroll
  for (int s = 1; s < STR_MAX_SPLIT; ++s) {
    const float w = s < splitk ? 1.f : 0.f;
    v += f32x4{part[s][0][0], part[s][0][1], part[s][1][0], part[s][1][1]} * w;
  }
  if (n + 3 < N && ((reinterpret_cast<uintptr_t>(sw) | reinterpret_cast<uintptr_t>(colsum)) & 15) == 0) {
    if constexpr (W8) v *= *reinterpret_cast<const f32x4*>(sw + n);
    if constexpr (NORM == 2) v = rstd * (v - mean * *reinterpret_cast<const f32x4*>(colsum + n));
    if constexpr (NORM == 1) v *= rstd;
    return v;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool ok = n + r < N;
    if constexpr (W8) v[r] *= ok ? sw[n + r] : 0.f;
    if constexpr (NORM == 2) v[r] = rstd * (v[r] - mean * (ok ? colsum[n + r] : 0.f));
    if constexpr (NORM == 1) v[r] *= rstd;
  }
  return v;
}

// Combine + epilogue of output items (row m, 4 output columns o): packed
// gate|up (SiLU-mul) pairs gate columns 16g+w.. with up columns 16g+8+w.
template <int ACT, int NORM, bool W8, bool SC1>
__device__ __forceinline__ void str_combine_item(const float* slab, int splitk, int MP, int Ns, int tile, int m, int o,
                                                 const uint8_t* __restrict__ A, int lda_b,
                                                 const float* __restrict__ sw, const float* __restrict__ colsum,
                                                 float eps, int kelems, void* __restrict__ Cv, int ldc,
                                                 const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr,
                                                 int M, int N, bool pre = true) {
  float mean = 0.f, rstd = 1.f;
  if constexpr (NORM != 0)
    str_row_norm<NORM, SC1>(slab + (size_t)splitk * MP * Ns, splitk, MP, tile, m, A, lda_b, kelems, eps, mean, rstd);
  if constexpr (ACT == ACT_SILU_MUL) {
    const int NO = N / 2;
    if (o >= NO) return;
    const int g = o >> 3, w = o & 7;
    const f32x4 gt = str_combine4<NORM, W8, SC1>(slab, splitk, MP, Ns, m, g * 16 + w, N, sw, colsum, mean, rstd);
    const f32x4 up = str_combine4<NORM, W8, SC1>(slab, splitk, MP, Ns, m, g * 16 + 8 + w, N, sw, colsum, mean, rstd);
    bf16_t* C = reinterpret_cast<bf16_t*>(Cv) + (size_t)m * ldc + o;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (o + r < NO) C[r] = f2bf(silu(gt[r]) * up[r]);
  } else {
    if (o >= N) return;
    const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
    if (pre && vec && o + 3 < N && m < M) {
      // bias and residual issued with the partials: one memory round trip for
      // the item instead of two (Llama-3 down projection + residual)
      f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x4 r4 = bf16x4{0, 0, 0, 0};
      if (bias != nullptr) b4 = *reinterpret_cast<const f32x4*>(bias + o);
      if (R != nullptr) r4 = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + o);
      epi_t4_pre<ACT>(str_combine4<NORM, W8, SC1>(slab, splitk, MP, Ns, m, o, N, sw, colsum, mean, rstd), m, o, Cv,
                      ldc, bias != nullptr, b4, R != nullptr, r4);
      return;
    }
    epi_t4<ACT, false>(str_combine4<NORM, W8, SC1>(slab, splitk, MP, Ns, m, o, N, sw, colsum, mean, rstd), m, o, M,
                       N, Cv, ldc, bias, R, ldr, vec);
  }
}

// The last-arriving workgroup of tile `tile` combines its MP x BN outputs.
template <int ACT, int NORM, bool W8, bool SC1>
__device__ __forceinline__ void str_combine_tile(const float* slab, int splitk, int MP, int Ns, int tile, int BN,
                                                 const uint8_t* __restrict__ A, int lda_b,
                                                 const float* __restrict__ sw, const float* __restrict__ colsum,
                                                 float eps, int kelems, void* __restrict__ Cv, int ldc,
                                                 const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr,
                                                 int M, int N, int tid) {
  const int per_row = (ACT == ACT_SILU_MUL ? BN / 2 : BN) / 4;
  const int o0 = (ACT == ACT_SILU_MUL ? tile * BN / 2 : tile * BN);
  for (int i = tid; i < MP * per_row; i += 256) {
    const int m = i / per_row, o = o0 + (i - m * per_row) * 4;
    if (m < M)
      str_combine_item<ACT, NORM, W8, SC1>(slab, splitk, MP, Ns, tile, m, o, A, lda_b, sw, colsum, eps, kelems, Cv, ldc,
                                           bias, R, ldr, M, N);
  }
}

template <int MT, int NT, bool W8, int NORM, int ACT, bool SPLIT, bool FOLD = false>
__global__ __launch_bounds__(256, 1) void gemm_stream_kernel(const uint8_t* __restrict__ A, int lda_b,
                                                             const uint8_t* __restrict__ Wsh,
                                                             const float* __restrict__ sw, void* __restrict__ Cv,
                                                             int ldc, const float* __restrict__ bias,
                                                             const bf16_t* __restrict__ R, int ldr, int M, int N,
                                                             int nch, int cps, const float* __restrict__ colsum,
                                                             float eps, int kelems, float* __restrict__ slab,
                                                             unsigned* __restrict__ cnt = nullptr) {
  using Cfg = StrCfg<W8>;
  constexpr int ACH = Cfg::ACH, CS = Cfg::CS, AU = Cfg::AU;
  constexpr int MP = MT * 16;
  constexpr int BN = 64 * NT;
  constexpr int APASS = MP * STR_SB / 4096;  // 16-B staging loads per thread per step
  __shared__ __attribute__((aligned(1024))) char lds[2 * MP * STR_SB + 4 * 16 * 2 * 4];
  float* st_lds = reinterpret_cast<float*>(lds + 2 * MP * STR_SB);  // [MT][2][16] row statistics (no SPLIT)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = (N + BN - 1) / BN;
  const int splitk = gridDim.x / ntiles;
  const int lg = xcd_remap(blockIdx.x, gridDim.x);
  // slice-major: the workgroups of one XCD mostly share a K slice, so its A
  // rows are fetched into that XCD's L2 once
  const int slice = lg / ntiles, tile = lg - slice * ntiles;
  const int c0 = slice * cps, c1 = min(nch, c0 + cps);
  const int nsteps = (c1 - c0 + CS - 1) / CS;
  const int ntile16 = (N + 15) >> 4;

  const uint8_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int ct = tile * (4 * NT) + wave * NT + j;
    ct = ct < ntile16 ? ct : ntile16 - 1;
    wp[j] = Wsh + ((size_t)ct * nch + c0) * 1024 + lane * 16;
  }
  // staging pass p: flat byte p*4096 + tid*16 of the step's [MP][512] A image
  const uint8_t* ap[APASS];
  int aoff[APASS], aslot[APASS];
#pragma unroll
  for (int p = 0; p < APASS; ++p) {
    const int flat = p * 4096 + tid * 16, row = flat >> 9, slot = (flat & 511) >> 4;
    ap[p] = A + (size_t)min(row, M - 1) * lda_b;
    aslot[p] = slot * 16;
    aoff[p] = row * STR_SB + ((slot ^ (row & 15)) << 4);
  }
  const int a_last = c1 * ACH - 16;  // last valid 16 B of this slice's A rows (surplus chunks clamp here)
  // fragment read offsets (bytes inside a step image) for M tile t, chunk cc, piece h
  const int fr = lane & 15, fg = lane >> 4;
  auto frag_off = [&](int t, int cc, int h) {
    const int row = 16 * t + fr;
    const int slot = (cc * ACH + fg * (ACH / 4) + 16 * h) >> 4;
    return row * STR_SB + ((slot ^ (row & 15)) << 4);
  };

  float shift = 0.f, s1 = 0.f, s2 = 0.f;  // statistics of row 16*wave + fr (waves < MT)
  if constexpr (NORM == 2) {
    const int row = min(16 * wave + fr, M - 1);
    shift = bf2f(*reinterpret_cast<const bf16_t*>(A + (size_t)row * lda_b));
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  i32x4 wa[NT][CS], wb[NT][CS], as[APASS];
  auto load_w = [&](i32x4(&w)[NT][CS], int s) {
#pragma unroll
    for (int cc = 0; cc < CS; ++cc) {
      const int c = min(s * CS + cc, c1 - c0 - 1);  // surplus chunks of the last step: clamped, zeroed at use
#pragma unroll
      for (int j = 0; j < NT; ++j)
        w[j][cc] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp[j] + (size_t)c * 1024));
    }
  };
  auto load_a = [&](int s) {
#pragma unroll
    for (int p = 0; p < APASS; ++p)
      as[p] = *reinterpret_cast<const i32x4*>(ap[p] + min((c0 + s * CS) * ACH + aslot[p], a_last));
  };
  auto store_a = [&](int buf) {
    char* base = lds + buf * (MP * STR_SB);
#pragma unroll
    for (int p = 0; p < APASS; ++p) *reinterpret_cast<i32x4*>(base + aoff[p]) = as[p];
  };
  auto compute = [&](i32x4(&w)[NT][CS], int buf, int s) {
    const char* base = lds + buf * (MP * STR_SB);
#pragma unroll
    for (int cc = 0; cc < CS; ++cc) {
      const bool valid = c0 + s * CS + cc < c1;  // wave-uniform
      if (!valid) {
#pragma unroll
        for (int j = 0; j < NT; ++j) w[j][cc] = i32x4{0, 0, 0, 0};
      }
      bf16x8 af[MT][AU];
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int h = 0; h < AU; ++h) af[t][h] = *reinterpret_cast<const bf16x8*>(base + frag_off(t, cc, h));
      if constexpr (NORM != 0) {
        if (valid) {
#pragma unroll
          for (int t = 0; t < MT; ++t)
            if (t == wave) {
#pragma unroll
              for (int h = 0; h < AU; ++h) str_stats<NORM>(af[t][h], shift, s1, s2);
            }
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (W8) {
          bf16x8 wlo, whi;
          bf16x2v o[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            o[2 * i] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[j][cc][i], 1.0f, false);
            o[2 * i + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[j][cc][i], 1.0f, true);
          }
          __builtin_memcpy(&wlo, &o[0], 16);
          __builtin_memcpy(&whi, &o[4], 16);
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo, af[t][0], acc[j][t], 0, 0, 0);
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi, af[t][AU - 1], acc[j][t], 0, 0, 0);
          }
        } else {
          bf16x8 wf;
          __builtin_memcpy(&wf, &w[j][cc], 16);
#pragma unroll
          for (int t = 0; t < MT; ++t)
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af[t][0], acc[j][t], 0, 0, 0);
        }
      }
    }
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // One K-step s on weight set `cur` (A image in buffer s & 1): the next A
  // rows go to registers before the MFMAs, the weights of step s + 2 are
  // issued into `cur` right after them, and the step ends waiting only for
  // the A rows and the weights of step s + 1.  MORE_A / MORE_W are compile-
  // time, so no load sits behind a runtime branch (hipcc would otherwise
  // count conservatively and drain the weight stream at every step).
  auto step = [&](auto more_a_t, auto more_w_t, i32x4(&cur)[NT][CS], int s) {
    constexpr bool MORE_A = decltype(more_a_t)::value, MORE_W = decltype(more_w_t)::value;
    if constexpr (MORE_A) load_a(s + 1);
    compute(cur, s & 1, s);
    if constexpr (MORE_W) {
      load_w(cur, s + 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NT * CS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (MORE_A) store_a((s + 1) & 1);
    barrier();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  if (nsteps > 0) {
    load_w(wa, 0);
    load_a(0);
    if (nsteps > 1) {
      load_w(wb, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NT * CS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    store_a(0);
    barrier();
    int s = 0;
    for (; s + 3 < nsteps; s += 2) {  // both steps of a pair have more A rows and weights to issue
      step(T_{}, T_{}, wa, s);
      step(T_{}, T_{}, wb, s + 1);
    }
    const int r = nsteps - s;  // 1..3 steps left
    if (r == 3) {
      step(T_{}, T_{}, wa, s);
      step(T_{}, F_{}, wb, s + 1);
      step(F_{}, F_{}, wa, s + 2);
    } else if (r == 2) {
      step(T_{}, F_{}, wa, s);
      step(F_{}, F_{}, wb, s + 1);
    } else {
      step(F_{}, F_{}, wa, s);
    }
  }

  // ---- statistics of this wave's M tile: the 4 lane groups hold disjoint k
  if constexpr (NORM != 0) {
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
  }

  if constexpr (SPLIT) {
    // fp32 partials of this K slice: slab[slice][m][n] (Ns = ntiles * BN
    // columns), then the row statistics per (tile, slice): [ntiles][splitk][MP][2]
    const int Ns = ntiles * BN;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = tile * BN + (wave * NT + j) * 16 + fg * 4;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + fr;
        float* dst = slab + ((size_t)slice * MP + m) * Ns + n;
        if constexpr (FOLD) {
          str_store_sc1(dst, acc[j][t]);
        } else {
          *reinterpret_cast<f32x4*>(dst) = acc[j][t];
        }
      }
    }
    if constexpr (NORM != 0) {
      if (wave < MT && lane < 16) {
        float* st = slab + (size_t)splitk * MP * Ns + (((size_t)tile * splitk + slice) * MP + 16 * wave + lane) * 2;
        if constexpr (FOLD) {
          str_store_sc1_2(st, s1, s2);
        } else {
          st[0] = s1;
          st[1] = s2;
        }
      }
    }
    if constexpr (FOLD) {
      // In-launch split-K combine (guide §5 'Projection GEMM at M = 256' item
      // 2, write-through form; MI355X_MICROARCH.md visibility table row 1):
      // partials stored sc1 and drained by every storing wave, a workgroup
      // barrier, ONE lane's relaxed agent-scope ticket add; the workgroup that
      // draws splitk - 1 combines the tile, reading every partial with sc1
      // loads only (no acquire fence), and re-arms the ticket for the next call
      // (the counters start zeroed: ops/gemm.py decode_workspace).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      unsigned* last_flag = reinterpret_cast<unsigned*>(st_lds);
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = old == (unsigned)splitk - 1;
        if (last) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag[0] = last ? 1u : 0u;
      }
      __syncthreads();
      if (last_flag[0] == 0) return;
      str_combine_tile<ACT, NORM, W8, true>(slab, splitk, MP, Ns, tile, BN, A, lda_b, sw, colsum, eps, kelems, Cv, ldc,
                                            bias, R, ldr, M, N, tid);
    }
    return;
  } else {
    float mean[MT], rstd[MT];
    if constexpr (NORM != 0) {
      if (wave < MT && lane < 16) {
        st_lds[(wave * 2 + 0) * 16 + lane] = s1;
        st_lds[(wave * 2 + 1) * 16 + lane] = s2;
      }
      __syncthreads();
      const float invk = 1.f / (float)kelems;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const float a = st_lds[(t * 2 + 0) * 16 + fr], q = st_lds[(t * 2 + 1) * 16 + fr];
        const float d = a * invk;
        const float sh = NORM == 2 ? bf2f(*reinterpret_cast<const bf16_t*>(A + (size_t)min(16 * t + fr, M - 1) *
                                                                               lda_b))
                                   : 0.f;
        mean[t] = NORM == 2 ? sh + d : 0.f;
        const float var = NORM == 2 ? fmaxf(q * invk - d * d, 0.f) : q * invk;
        rstd[t] = rsqrtf(var + eps);
      }
    }
    const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int nb = tile * BN + (wave * NT + j) * 16;
      const int n = nb + fg * 4;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        f32x4 v = acc[j][t];
        const int m = 16 * t + fr;
        const bool v4 = n + 3 < N &&
                        ((reinterpret_cast<uintptr_t>(sw) | reinterpret_cast<uintptr_t>(colsum)) & 15) == 0;
        if constexpr (W8) {
          if (v4) {
            v *= *reinterpret_cast<const f32x4*>(sw + n);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] *= n + r < N ? sw[n + r] : 0.f;
          }
        }
        if constexpr (NORM == 2) {
          if (v4) {
            v = rstd[t] * (v - mean[t] * *reinterpret_cast<const f32x4*>(colsum + n));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rstd[t] * (v[r] - mean[t] * (n + r < N ? colsum[n + r] : 0.f));
          }
        } else if constexpr (NORM == 1) {
          v *= rstd[t];
        }
        if constexpr (ACT == ACT_SILU_MUL) {
          epi_silu_t4<false>(v, m, nb / 2, M, N / 2, Cv, ldc, vec, lane);
        } else {
          epi_t4<ACT, false>(v, m, n, M, N, Cv, ldc, bias, R, ldr, vec);
        }
      }
    }
  }
}

// Split-K combine + epilogue as its own launch (no workspace counters, or the
// fold switched off): one thread per (row, 4 output columns).
template <int ACT, int NORM, bool W8>
__global__ __launch_bounds__(256) void gemm_stream_reduce(const float* __restrict__ slab, int splitk, int MP, int Ns,
                                                          const uint8_t* __restrict__ A, int lda_b,
                                                          const float* __restrict__ sw,
                                                          const float* __restrict__ colsum, float eps, int kelems,
                                                          void* __restrict__ Cv, int ldc,
                                                          const float* __restrict__ bias,
                                                          const bf16_t* __restrict__ R, int ldr, int M, int N,
                                                          int epi_pre = 1) {
  const int NO = ACT == ACT_SILU_MUL ? N / 2 : N;
  const int per_row = (NO + 3) / 4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int m = idx / per_row, o = (idx - m * per_row) * 4;
  if (m >= M) return;
  str_combine_item<ACT, NORM, W8, false>(slab, splitk, MP, Ns, 0, m, o, A, lda_b, sw, colsum, eps, kelems, Cv, ldc,
                                         bias, R, ldr, M, N, epi_pre != 0);
}

}  // namespace dnn
