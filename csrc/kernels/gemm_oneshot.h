// One-shot decode GEMM for 17..64 rows ("oneshot" kernel):
//   C[M,N] = epi(A[M,K] . W[N,K]^T), W in fragment order (ops/gemm.py
//   shuffle_weight), bf16 or OCP e4m3 (W8A16), bf16 activations.
//
// Why a third decode GEMM.  At 32-64 rows the mid-size projections (GPT-2 /
// GPT-2 XL, Llama-3 QKV / O) are neither compute- nor HBM-bound: a 2.5-10 MB
// weight matrix is a few microseconds of HBM, but gemm_skinny streams each
// wave's K slice in batches of U chunks, each batch a dependent memory round
// trip (3-7 per wave, ~1-2 us each under load), with the activations loaded
// fragment-shaped (16 rows x 64 B per instruction: twice the TA work of a
// full-line load, guide §5 "x operand through LDS in full lines"); the sweep
// (profiles/archive/r1_skinny_sweep_shuf_fit.jsonl) puts every configuration at
// 0.4-0.9 TB/s on those shapes.  gemm_stream fixes the A path but pipelines
// K-steps, which only pays for >= 8 MB weights with >= 6 steps per slice.
//
// Here a workgroup issues EVERY load of its work at once and waits once:
//   * tile = MP = 16 MT rows x BN = 16 NTW columns x one K slice; the 4 waves
//     split the slice into contiguous quarters (no cross-wave operand sharing,
//     so no barrier before the MFMAs);
//   * each wave copies its A rows [MP][its quarter] into a private LDS image
//     by LDS-DMA (global_load_lds_dwordx4, full 128-B lines: an instruction
//     moves 2 rows x 512 B), in steps of 512 B per row with 16-B slot j of row
//     r at j ^ (r & 15) — the stream kernel's image, conflict-free for every
//     ds_read_b128 fragment read — the swizzle applied on the source address
//     (LDS-DMA writes lane-linear);
//   * each wave loads its quarter of the NTW weight tiles straight to VGPRs,
//     non-temporally (read once), all chunks in flight;
//   * the A rows are issued first, then the weights step-major; the folded
//     norm's row statistics are taken from the image once every load has
//     landed and the workgroup has synchronised ("Retiring the image"
//     below; the round-4 version took them under the weight flight, measured
//     neutral against taking them from the MFMA fragments,
//     profiles/r4_oneshot_norm_ab*.jsonl);
//   * MFMAs from LDS fragments x register weights; the 4
//     partial sums meet in LDS (each wave reuses its own image region), and
//     the epilogue runs in the workgroup (bias / GELU / residual / packed
//     SwiGLU / fp8 channel scale / folded pre-norm from row statistics
//     accumulated off the A fragments), or
//   * SPLIT: fp32 partials of the slice in gemm_stream's slab layout
//     [slice][MPT][Ns] (+ row statistics [tile][slice][MPT][2]), summed with
//     the epilogue by gemm_stream_reduce.
// The M split (MT < 4 at M = 64) puts the m-groups of one (tile, slice)
// on consecutive logical ids of one XCD, so the weight slice comes from HBM
// once and the other m-groups re-read it from that XCD's L2.
#pragma once
#include "gemm_stream.h"

namespace dnn {

constexpr int OS_SB = 512;  // A bytes per row per LDS step (bf16: 8 chunks of 32 k; W8: 4 chunks of 64 k)
constexpr int OS_RS_SPT = 16;  // producer row-statistics partials per thread (consumer merge)

template <int MT, int STEPS>
constexpr int os_lds_bytes() {
  return 4 * STEPS * MT * 16 * OS_SB + 4 * MT * 2 * 16 * 4;  // 4 wave images + row statistics
}

// ABL (probe only, bench/probes/oneshot_anatomy.py; 0 in every product launch):
// bit 1 no weight loads, 2 no activation image, 4 no MFMAs, 8 no epilogue
// stores, 32 return at once (the launch alone), 64 no cross-wave reduction
// (each wave's own partial goes to the epilogue), 128 the round-4/5 counted
// image wait (racy, below) — what each part costs.
//
// Retiring the image.  The image is read only after composable_kernel's
// direct-load sequence (block_sync_lds_direct_load: vmcnt(0), lgkmcnt(0),
// s_barrier), not after a count of the weights issued behind it: an LDS-DMA is
// not ordered with the plain loads that follow it.  The round-4/5 counted wait
// stays as the probe bit ABL 128; the sync costs nothing measurable
// (oneshot_anatomy.py counted_wait arm within +-0.13 us,
// profiles/r5_oneshot_anatomy_imagesync.jsonl).  Plain loads issued before
// the image (row-statistics partials, epilogue operands) are retired by
// counted waits: plain loads complete in order among themselves.
// tests/test_isa_lds_dma_order.py checks the sequence in the product ISA.
//
// The "race" of rounds 5-6 was not in the image.  A rare few-ulp error in one
// workgroup's second 16-row tile, only with two workgroups on a CU
// (profiles/r5_oneshot_race_screen_*.jsonl), survived every image-side change
// (a second barrier, CK / ck_tile wait forms, an s_sleep, register-staged
// images, LDS floors 0 / 72 KB; profiles/r6_oneshot_race_root_cause.md).  The
// epilogue-input dump (probe bit 32768) pinned it: in the failing wave exactly
// ONE element of the t = 1 row statistics was summed as x instead of x - shift,
// in lanes 48-63 only, for all 16 rows (delta s1 == shift exactly, delta s2 ==
// 2 x shift - shift^2 for an element of the wave's own range).  Those elements
// are the low halves of the SLP vectoriser's packed subtracts
// (v_pk_add_f32 dst, src, shift op_sel:[0,1] neg_lo:[0,1] neg_hi:[0,1]) whose
// low result a later 32-bit VALU op reads: under co-residency that read
// returned the register's pre-subtract value.  Built with -fno-slp-vectorize
// (ops/build.py PER_FILE_FLAGS; no cross-half packed FP32 in the kernel) the
// same launches ran 10000 calls at two workgroups per CU with 0 mismatches,
// against 100 mismatches of the SLP build in the same session
// (profiles/r6_oneshot_race_root_cause.jsonl, r6h).  The LDS floor
// (g_os_lds_floor) is a measured performance choice again.
constexpr int OS_PROBE_WORDS = 1024;  // race-probe record per workgroup (int32 words)

__device__ __forceinline__ uint32_t os_hash16(const bf16x8& v) {  // race probe: a 16-B read's fingerprint
  uint32_t w[4];
  __builtin_memcpy(w, &v, 16);
  return (w[0] * 0x9E3779B1u) ^ (w[1] * 0x85EBCA77u) ^ (w[2] * 0xC2B2AE3Du) ^ (w[3] * 0x27D4EB2Fu) ^ 0x5bd1e995u;
}

__device__ __forceinline__ void os_image_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
// race-probe variants of the image sync (ABL 2048 / 4096 / 8192 / 16384):
// composable_kernel's separate vmcnt(0) then lgkmcnt(0); vmcnt(0) alone
// (ck_tile); the wait plus a short s_sleep (a pure delay); the wait and two
// barriers (profiles/r6_oneshot_race_root_cause.jsonl)
template <int ABL>
__device__ __forceinline__ void os_image_sync_v() {
  if constexpr ((ABL & 2048) != 0) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else if constexpr ((ABL & 4096) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else if constexpr ((ABL & 8192) != 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_sleep 1" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else if constexpr ((ABL & 16384) != 0) {
    os_image_sync();
    __builtin_amdgcn_s_barrier();
  } else {
    os_image_sync();
  }
}

template <int MT, int NTW, bool W8, int NORM, int ACT, bool SPLIT, int STEPS, int ABL = 0>
__global__ __launch_bounds__(256, 2) void gemm_oneshot_kernel(const uint8_t* __restrict__ A, int lda_b,
                                                              const uint8_t* __restrict__ Wsh,
                                                              const float* __restrict__ sw, void* __restrict__ Cv,
                                                              int ldc, const float* __restrict__ bias,
                                                              const bf16_t* __restrict__ R, int ldr, int M, int N,
                                                              int nch, int cps, const float* __restrict__ colsum,
                                                              float eps, int kelems, float* __restrict__ slab,
                                                              int ntiles, int mgroups,
                                                              float2* __restrict__ rs_out = nullptr, int rs_ld = 0,
                                                              const float2* __restrict__ rs_in = nullptr,
                                                              int rs_ld_in = 0, int epi_pre = 1) {
  if constexpr ((ABL & 32) != 0) return;
  using Cfg = StrCfg<W8>;
  // Race-probe bits (bench/probes/oneshot_race_probe.py; never in a product
  // launch).  ``slab`` is then a per-workgroup int32 record (OS_PROBE_WORDS):
  //   256  detector: every 16-B image read of the row-statistics pass is
  //        hashed and read again after the MFMAs; lane l's record word is the
  //        mask of its (chunk, row tile) reads whose bytes changed in between;
  //   512  one workgroup barrier at entry (and nothing else);
  //   1024 the image sync twice before the statistics pass.
  static_assert((ABL & 256) == 0 || (!W8 && STEPS == 1 && !SPLIT), "race detector: bf16 one-step images only");
  if constexpr ((ABL & 512) != 0) __syncthreads();
  constexpr int ACH = Cfg::ACH, CS = Cfg::CS, AU = Cfg::AU;
  constexpr int MP = MT * 16;
  constexpr int BN = 16 * NTW;
  constexpr int CPW = STEPS * CS;                  // max chunks per wave
  constexpr int IMG = STEPS * MP * OS_SB;          // one wave's A image
  constexpr int GPS = MP * OS_SB / 1024;           // LDS-DMA instructions per step
  extern __shared__ __attribute__((aligned(1024))) char os_lds[];
  float* st_lds = reinterpret_cast<float*>(os_lds + 4 * IMG);  // [4 waves][MT][2][16]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = xcd_remap(blockIdx.x, gridDim.x);
  // tile-major inside a slice, m-group fastest: one (tile, slice)'s m-groups
  // are consecutive logical ids (one XCD: its weight slice is fetched once)
  const int mg = lg % mgroups;
  const int rest = lg / mgroups;
  const int tile = rest % ntiles, slice = rest / ntiles;
  const int m0 = mg * MP;
  const int ntile16 = (N + 15) >> 4;

  // this wave's chunk range [w0, w1) inside the slice
  const int s0 = slice * cps, s1 = min(nch, s0 + cps);
  const int cpw = (cps + 3) >> 2;
  const int w0 = min(s1, s0 + wave * cpw), w1 = min(s1, w0 + cpw);
  const int nvalid = w1 - w0;  // 0..CPW, wave-uniform

  char* img = os_lds + wave * IMG;
  const int fr = lane & 15, fg = lane >> 4;
  // producer-side row statistics (rs_in, no SPLIT; host: ceil(K/16) <= OS_RS_SPT
  // x TPR): the partials of the workgroup's rows are loaded first of all, so
  // the explicit vmcnt waits below (which count only the weights) cover them
  constexpr int TPR = 256 / MP, SPT = OS_RS_SPT;
  const bool rsi = NORM != 0 && !SPLIT && rs_in != nullptr;  // uniform
  float2 rsp[SPT], rs0 = make_float2(0.f, 0.f);
  if (rsi) {
    const float2* p = rs_in + (size_t)min(m0 + tid / TPR, M - 1) * rs_ld_in;
    const int np = (kelems + 15) >> 4, sub = tid % TPR;
    rs0 = p[0];
#pragma unroll
    for (int i = 0; i < SPT; ++i) rsp[i] = p[min(sub + i * TPR, np - 1)];
  }
  // ---- epilogue operands first of all (as the row-statistics partials): the
  // channel scales, column sums, bias and residual of the wave's output tiles
  // land with the image, so the epilogue after the cross-wave reduction pays
  // no memory round trip.  Uniform: vector-aligned operands, N % 4 == 0.
  constexpr int QPW = (NTW * MT + 3) / 4;  // epilogue tiles per wave
  // (14 VGPRs per tile: up to 2 tiles per wave; the 64 x 64 tiles spilled with 4)
  constexpr bool PRE = QPW <= 2 && !SPLIT && ACT != ACT_SILU_MUL;
  const bool pre = PRE && epi_pre && (N & 3) == 0 && epi_vec_ok(Cv, ldc, bias, R, ldr) &&
                   ((reinterpret_cast<uintptr_t>(sw) | reinterpret_cast<uintptr_t>(colsum)) & 15) == 0;
  // Unconditional, branch-free loads (absent operands read a valid dummy
  // address, and ``pre`` / has_b / has_r decide what is used): a load under a
  // branch made the compiler wait for it at the merge, before the image was
  // even issued.
  f32x4 pre_sw[QPW], pre_cs[QPW], pre_b[QPW];
  bf16x4 pre_r[QPW];
  if constexpr (PRE) {
    const float* dummy = reinterpret_cast<const float*>(A);
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int q = min(wave + 4 * k, NTW * MT - 1);
      const int nn = min((tile * NTW + q / MT) * 16 + fg * 4, N - 4);
      const int mm = min(m0 + 16 * (q % MT) + fr, M - 1);
      if constexpr (W8) pre_sw[k] = *reinterpret_cast<const f32x4*>(sw + nn);
      if constexpr (NORM == 2) pre_cs[k] = *reinterpret_cast<const f32x4*>(colsum != nullptr ? colsum + nn : dummy);
      pre_b[k] = *reinterpret_cast<const f32x4*>(bias != nullptr ? bias + nn : dummy);
      pre_r[k] = *reinterpret_cast<const bf16x4*>(R != nullptr ? R + (size_t)mm * ldr + nn
                                                              : reinterpret_cast<const bf16_t*>(dummy));
    }
  }
  float shift[MT], s1s[MT], s2s[MT];
  [[maybe_unused]] uint32_t prb_h[CPW][MT];  // ABL 256: hashes of the statistics pass's image reads
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    shift[t] = 0.f;
    s1s[t] = s2s[t] = 0.f;
    if constexpr (NORM == 2) {
      if (!rsi) {
        const int row = min(m0 + 16 * t + fr, M - 1);
        shift[t] = bf2f(*reinterpret_cast<const bf16_t*>(A + (size_t)row * lda_b));
      }
    }
  }
  // the loads above (row-statistics partials, epilogue operands, shifts) stay
  // ahead of the image and the weights: the counted vmcnt waits below retire
  // the image by counting only the weights issued after it, so nothing may be
  // scheduled in between (a prefetch load sunk past the LDS-DMA let the image
  // be read before it landed)
  __builtin_amdgcn_sched_barrier(0);
  // ---- issue: every A row segment of the wave's range by LDS-DMA (full
  // lines), then every weight chunk, step-major (all in flight at once; the
  // image is read after os_image_sync)
  const int kb0 = w0 * ACH;  // first A byte of the wave's range in a row
  // last valid 16 B of the range (surplus slots clamp here; their weights are zeroed)
  const int kb_last = min(max(w1, w0 + 1), nch) * ACH - 16;
  i32x4 wv[NTW][CPW];
#pragma unroll
  for (int s = 0; s < (ABL & 2 ? 0 : STEPS); ++s) {
#pragma unroll
    for (int p = 0; p < GPS; ++p) {
      const int r = 2 * p + (lane >> 5);  // row inside the step image
      const int j = lane & 31;            // LDS slot of this lane
      const int g = j ^ (r & 15);         // global slot it holds
      const int row = min(m0 + r, M - 1);
      const int kb = min(kb0 + s * OS_SB + g * 16, kb_last);
      glds16(A + (size_t)row * lda_b + kb, img + s * MP * OS_SB + p * 1024);
    }
  }
#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      int ct = tile * NTW + j;
      ct = ct < ntile16 ? ct : ntile16 - 1;
      const uint8_t* wp = Wsh + ((size_t)ct * nch) * 1024 + lane * 16;
#pragma unroll
      for (int c = s * CS; c < (s + 1) * CS; ++c) {
        const int cc = min(min(w0 + c, max(w1, w0 + 1) - 1), nch - 1);
        if constexpr (ABL & 1)
          wv[j][c] = i32x4{cc, j, 0, 0};
        else
          wv[j][c] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp + (size_t)cc * 1024));
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);

  // ---- row statistics of this wave's K range from its image (the 4 lane
  // groups hold disjoint k)
  if (rsi) {
    // merge the producer's partials instead (plain loads issued before the
    // weights: the counted wait retires them): mean / rstd of row tid / TPR
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEPS * NTW * CS) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    const float2 mr = rowstat_merge<NORM, TPR, SPT>(rsp, rs0, tid % TPR, kelems, eps);
    if (tid % TPR == 0) {
      st_lds[(tid / TPR) * 2 + 0] = mr.x;
      st_lds[(tid / TPR) * 2 + 1] = mr.y;
    }
    __builtin_amdgcn_sched_barrier(0);
  } else if constexpr (NORM != 0) {
    if constexpr ((ABL & 128) != 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEPS * NTW * CS) : "memory");  // racy (probe only)
    else
      os_image_sync_v<ABL>();  // the image (see "Retiring the image")
    if constexpr ((ABL & 1024) != 0) os_image_sync();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int s = c / CS, cc = c % CS;
      if (c < nvalid) {  // wave-uniform
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int h = 0; h < AU; ++h) {
            const int row = 16 * t + fr;
            const int slot = (cc * ACH + fg * (ACH / 4) + 16 * h) >> 4;
            const bf16x8 a8 =
                *reinterpret_cast<const bf16x8*>(img + s * MP * OS_SB + row * OS_SB + ((slot ^ (row & 15)) << 4));
            if constexpr ((ABL & 256) != 0) prb_h[c][t] = os_hash16(a8);
            str_stats<NORM>(a8, shift[t], s1s[t], s2s[t]);
          }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  f32x4 acc[NTW][MT];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the image and every weight retired (ABL 128: step 1's weights, NTW x CS
  // loads issued last, still in flight — racy for the image, probe only)
  if constexpr (STEPS == 2 && (ABL & 128) != 0) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NTW * CS) : "memory");
  } else if constexpr ((ABL & 128) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    os_image_sync_v<ABL>();  // again after a statistics pass: the weights land here, the barrier is cheap
  }
  __builtin_amdgcn_sched_barrier(0);

#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const int s = c / CS, cc = c % CS;
    if (STEPS == 2 && c == CS) {  // step 1's weights
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (ABL & 4) continue;
    const bool valid = c < nvalid;  // wave-uniform
    if (!valid) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) wv[j][c] = i32x4{0, 0, 0, 0};
    }
    bf16x8 af[MT][AU];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int h = 0; h < AU; ++h) {
        const int row = 16 * t + fr;
        const int slot = (cc * ACH + fg * (ACH / 4) + 16 * h) >> 4;
        af[t][h] = *reinterpret_cast<const bf16x8*>(img + s * MP * OS_SB + row * OS_SB + ((slot ^ (row & 15)) << 4));
      }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      if constexpr (W8) {
        bf16x8 wlo, whi;
        bf16x2v o[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[2 * i] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)wv[j][c][i], 1.0f, false);
          o[2 * i + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)wv[j][c][i], 1.0f, true);
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
        __builtin_memcpy(&wf, &wv[j][c], 16);
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af[t][0], acc[j][t], 0, 0, 0);
      }
    }
  }

  // ABL 256: the statistics pass's reads again, after the MFMAs
  if constexpr ((ABL & 256) != 0 && NORM != 0) {
    uint32_t mask = 0;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int s = c / CS, cc = c % CS;
      if (c < nvalid && !rsi) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int row = 16 * t + fr;
          const int slot = (cc * ACH + fg * (ACH / 4)) >> 4;
          const bf16x8 a8 =
              *reinterpret_cast<const bf16x8*>(img + s * MP * OS_SB + row * OS_SB + ((slot ^ (row & 15)) << 4));
          if (os_hash16(a8) != prb_h[c][t]) mask |= 1u << (c * MT + t);
        }
      }
    }
    int* rec = reinterpret_cast<int*>(slab) + (size_t)lg * OS_PROBE_WORDS;
    rec[16 + wave * 64 + lane] = (int)mask;
  }

  // ---- row statistics of this wave's K range: the 4 lane groups hold disjoint k
  if (NORM != 0 && !rsi) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float a = s1s[t], q = s2s[t];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        st_lds[((wave * MT + t) * 2 + 0) * 16 + lane] = a;
        st_lds[((wave * MT + t) * 2 + 1) * 16 + lane] = q;
      }
    }
  }
  // ---- the 4 K-quarters meet in LDS: each wave parks its sums in its own
  // image (its fragment reads are complete), then every wave reads all four
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  f32x4* red = reinterpret_cast<f32x4*>(img);
  if constexpr ((ABL & 64) == 0) {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t) red[(j * MT + t) * 64 + lane] = acc[j][t];
    __syncthreads();
  }

  const int Ns = ntiles * BN;
  const int MPT = mgroups * MP;
#pragma unroll
  for (int k = 0; k < QPW; ++k) {
    const int q = wave + 4 * k;
    if (q >= NTW * MT) break;  // wave-uniform
    const int j = q / MT, t = q % MT;
    f32x4 v;
    if constexpr ((ABL & 64) != 0) {
      v = acc[j][t];
    } else {
      v = reinterpret_cast<const f32x4*>(os_lds)[(j * MT + t) * 64 + lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) v += reinterpret_cast<const f32x4*>(os_lds + w * IMG)[(j * MT + t) * 64 + lane];
    }
    const int ml = 16 * t + fr;       // row inside the m-group
    const int m = m0 + ml;
    const int nb = (tile * NTW + j) * 16;
    const int n = nb + fg * 4;
    float a = 0.f, q2 = 0.f;
    if constexpr (NORM != 0) {
      if (!rsi) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          a += st_lds[((w * MT + t) * 2 + 0) * 16 + fr];
          q2 += st_lds[((w * MT + t) * 2 + 1) * 16 + fr];
        }
      }
    }
    if constexpr (SPLIT) {
      *reinterpret_cast<f32x4*>(slab + ((size_t)slice * MPT + m) * Ns + n) = v;
      if constexpr (NORM != 0) {
        if (tile == 0 && j == 0 && lane < 16) {  // statistics once per (slice, row): tile 0 (gemm_stream_reduce reads tile 0)
          float* st = slab + (size_t)(cps > 0 ? (nch + cps - 1) / cps : 1) * MPT * Ns +
                      ((size_t)slice * MPT + m) * 2;
          st[0] = a;
          st[1] = q2;
        }
      }
      continue;
    } else {
      if constexpr (W8) {
        if (pre) {
          v *= n < N ? pre_sw[k] : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= n + r < N ? sw[n + r] : 0.f;
        }
      }
      if constexpr (NORM != 0) {
        const float invk = 1.f / (float)kelems, d = a * invk;
        float mean = NORM == 2 ? shift[t] + d : 0.f;
        const float var = NORM == 2 ? fmaxf(q2 * invk - d * d, 0.f) : q2 * invk;
        float rstd = rsqrtf(var + eps);
        if (rsi) {
          mean = st_lds[ml * 2 + 0];
          rstd = st_lds[ml * 2 + 1];
        }
        if constexpr ((ABL & 32768) != 0) {  // race probe: the epilogue's inputs of this (tile, lane)
          float* d32 = slab + ((size_t)lg * 2 + (q & 1)) * 64 * 24 + lane * 24;
          d32[0] = v[0];
          d32[1] = v[1];
          d32[2] = v[2];
          d32[3] = v[3];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            d32[4 + w] = st_lds[((w * MT + t) * 2 + 0) * 16 + fr];
            d32[8 + w] = st_lds[((w * MT + t) * 2 + 1) * 16 + fr];
          }
          d32[12] = shift[t];
          d32[13] = mean;
          d32[14] = rstd;
          d32[15] = (float)q;
          d32[16] = __int_as_float((int)__builtin_amdgcn_s_getreg((31 << 11) | 4));
          d32[17] = __int_as_float((int)__builtin_amdgcn_s_getreg((31 << 11) | 20));
          d32[18] = __int_as_float(wave);
        }
        if constexpr (NORM == 2) {
          if (pre) {
            v = rstd * (v - mean * (n < N ? pre_cs[k] : f32x4{0.f, 0.f, 0.f, 0.f}));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rstd * (v[r] - mean * (n + r < N ? colsum[n + r] : 0.f));
          }
        } else {
          v *= rstd;
        }
      }
      const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
      if constexpr (ABL & 8) {
        if (v[0] == 12345.f) reinterpret_cast<float*>(Cv)[0] = v[1];  // keep the sums live, store nothing
      } else if constexpr (ACT == ACT_SILU_MUL) {
        epi_silu_t4<false>(v, m, nb / 2, M, N / 2, Cv, ldc, vec, lane);
      } else if (pre && nb + 15 < N) {  // wave-uniform (epi_rowstat16 shuffles): the whole 16-column tile
        f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m < M) epi_t4_pre<ACT>(v, m, n, Cv, ldc, bias != nullptr, pre_b[k], R != nullptr, pre_r[k], &x);
        if (rs_out != nullptr) epi_rowstat16(x, m, nb, M, N, rs_out, rs_ld, lane);
      } else if (rs_out != nullptr) {  // uniform: row-statistics partials of the stored tile
        f32x4 x;
        epi_t4<ACT, false>(v, m, n, M, N, Cv, ldc, bias, R, ldr, vec, nullptr, 1.f, &x);
        epi_rowstat16(x, m, nb, M, N, rs_out, rs_ld, lane);
      } else {
        epi_t4<ACT, false>(v, m, n, M, N, Cv, ldc, bias, R, ldr, vec);
      }
    }
  }
  if constexpr ((ABL & 65536) != 0) __syncthreads();  // race probe: no wave leaves before the epilogue is done
  if constexpr ((ABL & 256) != 0) {
    if (tid == 0) {
      int* rec = reinterpret_cast<int*>(slab) + (size_t)lg * OS_PROBE_WORDS;
      rec[0] = (int)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID: wave/simd/cu/sh/se ids
      rec[1] = (int)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
      rec[15] = (int)blockIdx.x;
    }
  }
}

}  // namespace dnn
