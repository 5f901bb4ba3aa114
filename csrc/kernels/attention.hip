// Attention kernels for gfx950: QKV split (+RoPE, KV-cache write), causal
// flash-attention prefill on MFMA, and split-K decode attention.
//
// Replaces nanoGPT's CausalSelfAttention internals (qkv split, causal SDPA;
// Block of partitions/gpt_model_parts.py:20-21,32-33,46-47) and the Llama GQA
// attention. The reference recomputes the full prefix every call (no KV cache);
// here K/V live in a per-stage cache [B][Hkv][S][hd] (bf16, sized from the 288
// GB HBM) and positions/lengths are read from device memory so decode steps
// replay one captured HIP graph.
//
// Flash prefill structure (cdna_hip_programming.md App. B + §3 "accumulator as
// next operand"): 4 waves x 32 query rows; per 64-key block each wave computes
// S^T = K.Q^T with v_mfma_f32_32x32x16_bf16 (query on the lane, keys in the 16
// accumulator registers, so the row max/sum are in-register + one xor-32
// shuffle), then O^T += V^T . P^T with the S^T accumulators converted to bf16
// as the B operand (no LDS round trip for P) and V^T fragments fetched with
// ds_read_b64_tr_b16 (hardware transpose) from a row-padded V tile. K rows are
// XOR-swizzled so the A-fragment ds_read_b128 reads are conflict-free.
#include "common.h"

#include <cstdlib>

namespace dnn {

// Phase timestamps of decode-attention block (0,0), thread 0: only in the
// bench-only probe build (-DDNN_DEC_PROBE, bench/attn_probe.py).
#ifdef DNN_DEC_PROBE
__device__ unsigned long long dec_probe_ts[32];
#define DEC_PROBE(i, dep)                                                             \
  do {                                                                                \
    asm volatile("" ::"v"(dep));                                                      \
    if (threadIdx.x == 0 && (blockIdx.x | blockIdx.y) == 0) {                         \
      dec_probe_ts[i] = __builtin_amdgcn_s_memrealtime();                             \
      dec_probe_ts[16 + i] = __builtin_amdgcn_s_memtime();                             \
    }                                                                                 \
  } while (0)
#else
#define DEC_PROBE(i, dep) do { } while (0)
#endif

typedef short s16x4 __attribute__((ext_vector_type(4)));

// e4m3 KV cache (KV8) conversions of 8 entries: bf16 -> OCP e4m3 (RNE,
// saturated to +-448 first: the hardware convert does not clamp) and back
// (exact: v_cvt_scalef32_pk_bf16_fp8 at scale 1).
__device__ __forceinline__ uint2 kv8_pack8(const i32x4& x) {  // 8 bf16 -> 8 e4m3
  int lo = 0, hi = 0;
  float f[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = fminf(fmaxf(__uint_as_float((uint32_t)x[i] << 16), -448.f), 448.f);
    f[2 * i + 1] = fminf(fmaxf(__uint_as_float((uint32_t)x[i] & 0xffff0000u), -448.f), 448.f);
  }
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return make_uint2((uint32_t)lo, (uint32_t)hi);
}
__device__ __forceinline__ i32x4 kv8_unpack8(const uint2 w) {  // 8 e4m3 -> 8 bf16
  i32x4 r;
  r[0] = __builtin_bit_cast(int, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, false));
  r[1] = __builtin_bit_cast(int, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, true));
  r[2] = __builtin_bit_cast(int, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, false));
  r[3] = __builtin_bit_cast(int, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, true));
  return r;
}


// ---------------------------------------------------------------------------
// QKV split: qkv rows r = b*T + t, columns [q H*hd | k Hkv*hd | v Hkv*hd].
// q -> q_out[b][h][t][:] (RoPE'd when rope), k/v -> cache[b][hkv][pos[b]+t][:].
// One thread = 8 elements of the first half + the matching 8 of the second
// half of one head (rotate-half pairs).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void qkv_split_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ q,
                                                        bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int B, int T,
                                                        int H, int Hkv, int hd, int S, const int* __restrict__ pos,
                                                        const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                        int rope, int kv8) {
  const int half = hd / 2, groups = half / 8;
  const int heads = H + 2 * Hkv;
  const long total = (long)B * T * heads * groups;
  const int ld = heads * hd;
  for (long gi = blockIdx.x * (long)blockDim.x + threadIdx.x; gi < total; gi += (long)gridDim.x * blockDim.x) {
    const int g = (int)(gi % groups);
    long r = gi / groups;
    const int hh = (int)(r % heads);
    r /= heads;
    const int t = (int)(r % T), b = (int)(r / T);
    const int p = (pos != nullptr ? pos[b] : 0) + t;
    if (p >= S) continue;  // past the cache capacity: drop (never write out of bounds)
    const bf16_t* src = qkv + (size_t)(b * T + t) * ld + hh * hd;
    const int i0 = g * 8;
    const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(src + i0);
    const bf16x8 x2 = *reinterpret_cast<const bf16x8*>(src + half + i0);
    bf16x8 y1 = x1, y2 = x2;
    if (rope && hh < H + Hkv) {
      const float* cr = cosT + (size_t)p * half + i0;
      const float* sr = sinT + (size_t)p * half + i0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = bf2f_s(x1[j]), c = bf2f_s(x2[j]), co = cr[j], si = sr[j];
        y1[j] = (short)f2bf(a * co - c * si);
        y2[j] = (short)f2bf(c * co + a * si);
      }
    }
    if (kv8 && hh >= H) {  // e4m3 cache rows: 8 + 8 bytes
      uint8_t* d8 = reinterpret_cast<uint8_t*>(hh < H + Hkv ? kc : vc) +
                    (((size_t)b * Hkv + (hh < H + Hkv ? hh - H : hh - H - Hkv)) * S + p) * hd;
      *reinterpret_cast<uint2*>(d8 + i0) = kv8_pack8(__builtin_bit_cast(i32x4, y1));
      *reinterpret_cast<uint2*>(d8 + half + i0) = kv8_pack8(__builtin_bit_cast(i32x4, y2));
      continue;
    }
    bf16_t* dst;
    if (hh < H) {
      dst = q + (((size_t)b * H + hh) * T + t) * hd;
    } else if (hh < H + Hkv) {
      dst = kc + (((size_t)b * Hkv + (hh - H)) * S + p) * hd;
    } else {
      dst = vc + (((size_t)b * Hkv + (hh - H - Hkv)) * S + p) * hd;
    }
    *reinterpret_cast<bf16x8*>(dst + i0) = y1;
    *reinterpret_cast<bf16x8*>(dst + half + i0) = y2;
  }
}

// ---------------------------------------------------------------------------
// Causal flash-attention prefill (chunked: queries at absolute pos[b]+t attend
// keys 0..pos[b]+t of the cache).
// ---------------------------------------------------------------------------
constexpr int FA_QB = 128, FA_KB = 64;

template <int HD>
struct FaSmem {
  static constexpr int K_BYTES = FA_KB * HD * 2;
  static constexpr int V_STRIDE = HD * 2 + 64;  // padded row: conflict-free tr reads
  static constexpr int V_BYTES = FA_KB * V_STRIDE;
  static constexpr int TOTAL = K_BYTES + V_BYTES;
};

template <int HD>
__device__ __forceinline__ int k_swz(int key, int chunk) {
  return HD == 64 ? (chunk ^ ((key >> 1) & 7)) : (chunk ^ (key & 15));
}

// QKV: q is the c_attn output itself (rows b*T+t, row stride ldq, columns
// [q H*hd | k Hkv*hd | v Hkv*hd], no RoPE): Q and the chunk's own keys/values
// (positions >= pos[b]) are read straight from it, older keys from the cache,
// and the first query head of each kv group copies its 128-row slice of new
// K/V into the cache — the qkv_split launch and its round trip disappear.
// grid (H, B, query blocks), dispatched x fastest: every (b, h) of the last
// query block (the causal diagonal's longest key range) goes first, the
// one-block workgroups fill the tail (longest-processing-time-first).  With
// blockIdx.x = query block the heavy workgroups were spread over the whole
// dispatch and the last ones ran alone: GPT-2 B=64 T=512 0.1050 -> 0.0931 ms,
// T=2048 0.140 -> 0.089, hd 128 T=4096 1.092 -> 0.781 (profiles/r4_flash_lpt_ab.jsonl)
//
// PIPE (hd 64, opt-in: DNN_FLASH_PIPE=1): three K/V buffers and
// two score accumulators, so block j+1's S = K Q^T MFMAs are issued before
// block j's softmax and P.V — the matrix pipe works through the softmax VALU
// of the same wave instead of waiting on the S -> max -> exp -> P.V chain
// (PMC before: MFMA 0.14 busy, profiles/r4_pmc_flash_lpt.md).
// Measured slower, so off by default: GPT-2 B=64 T=512 0.0950 -> 0.1075 ms,
// B=8 T=2048 0.0851 -> 0.0986, 4-stage prefill 4.21 -> 4.13 M tok/s
// (profiles/r5_flash_pipe_ab.jsonl): the second accumulator takes the kernel
// from 144 to 212 VGPRs and three buffers to 60 KB of LDS, i.e. from 3 to 2
// workgroups per CU — the lost wave per SIMD overlapped the chain better.
template <int HD, bool QKV = false, bool KV8 = false, bool DB = false, bool PIPE = false>
__global__ __launch_bounds__(256, 2) void flash_attn_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                            const bf16_t* __restrict__ vc, bf16_t* __restrict__ o, int T,
                                                            int H, int Hkv, int S, const int* __restrict__ pos,
                                                            float scale_log2, int ldq = 0,
                                                            bf16_t* __restrict__ kc_out = nullptr,
                                                            bf16_t* __restrict__ vc_out = nullptr) {
  using SM = FaSmem<HD>;
  // DB: two K/V buffers, one barrier per block (the block after next is staged
  // into the other buffer while this one is read)
  __shared__ __attribute__((aligned(16))) char smem[SM::TOTAL * (PIPE ? 3 : DB ? 2 : 1)];
  char* ks = smem;
  char* vs = smem + SM::K_BYTES;
  constexpr int NKS = HD / 16;  // k-steps of the QK^T contraction
  constexpr int NDT = HD / 32;  // 32-wide d tiles of O
  constexpr int CH = HD / 8;    // 16-B chunks per row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int qb = (int)(gridDim.z - 1 - blockIdx.z), hh = blockIdx.x, b = blockIdx.y;
  const int kvh = hh / (H / Hkv);
  const int p0 = pos != nullptr ? pos[b] : 0;
  const int kv_len = p0 + T;
  const int qrow0 = qb * FA_QB + wave * 32;            // this wave's first query (chunk-relative)
  const int qrow = qrow0 + r32;                        // this lane's query
  const int q_abs = p0 + min(qrow, T - 1);
  const int wave_qmax = p0 + min(qrow0 + 31, T - 1);   // wave-uniform
  const int wave_qmin = p0 + min(qrow0, T - 1);
  const int blk_qmax = p0 + min(qb * FA_QB + FA_QB - 1, T - 1);
  const int kv_end = min(min(kv_len, blk_qmax + 1), S);  // never read past the cache

  const bf16_t* krow_new = nullptr;  // QKV: this sequence's new-key rows (position p0 + t = row b*T + t)
  const bf16_t* vrow_new = nullptr;
  if constexpr (QKV) {
    krow_new = q + (size_t)b * T * ldq + (size_t)(H + kvh) * HD;
    vrow_new = q + (size_t)b * T * ldq + (size_t)(H + Hkv + kvh) * HD;
    if (hh % (H / Hkv) == 0) {  // cache write of rows t in [qb*128, qb*128+128), once per kv head
      bf16_t* kd = kc_out + ((size_t)b * Hkv + kvh) * S * HD;
      bf16_t* vd = vc_out + ((size_t)b * Hkv + kvh) * S * HD;
      for (int e = tid; e < FA_QB * CH; e += 256) {
        const int t = qb * FA_QB + e / CH, c = e % CH;
        if (t < T && p0 + t < S) {
          if constexpr (KV8) {
            uint8_t* kd8 = reinterpret_cast<uint8_t*>(kc_out) + ((size_t)b * Hkv + kvh) * S * HD;
            uint8_t* vd8 = reinterpret_cast<uint8_t*>(vc_out) + ((size_t)b * Hkv + kvh) * S * HD;
            *reinterpret_cast<uint2*>(kd8 + (size_t)(p0 + t) * HD + c * 8) =
                kv8_pack8(*reinterpret_cast<const i32x4*>(krow_new + (size_t)t * ldq + c * 8));
            *reinterpret_cast<uint2*>(vd8 + (size_t)(p0 + t) * HD + c * 8) =
                kv8_pack8(*reinterpret_cast<const i32x4*>(vrow_new + (size_t)t * ldq + c * 8));
          } else {
            *reinterpret_cast<uint4*>(kd + (size_t)(p0 + t) * HD + c * 8) =
                *reinterpret_cast<const uint4*>(krow_new + (size_t)t * ldq + c * 8);
            *reinterpret_cast<uint4*>(vd + (size_t)(p0 + t) * HD + c * 8) =
                *reinterpret_cast<const uint4*>(vrow_new + (size_t)t * ldq + c * 8);
          }
        }
      }
    }
  }

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[qrow][ks*16 + 8h + j]
  bf16x8 qf[NKS];
  {
    const bf16_t* qp = QKV ? q + ((size_t)b * T + min(qrow, T - 1)) * ldq + (size_t)hh * HD + 8 * h
                           : q + (((size_t)b * H + hh) * T + min(qrow, T - 1)) * HD + 8 * h;
#pragma unroll
    for (int s = 0; s < NKS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + s * 16);
  }
  f32x16 oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) oacc[i] = f32x16{};
  float m_i = -INFINITY, l_i = 0.f;

  const bf16_t* kbase = kc + ((size_t)b * Hkv + kvh) * S * HD;
  const bf16_t* vbase = vc + ((size_t)b * Hkv + kvh) * S * HD;

  // K/V blocks are register double-buffered: block kb0+64 is fetched from
  // global memory while block kb0 is computed, then written to LDS after the
  // trailing barrier.  (Fetching two blocks ahead measured neutral at GPT-2
  // prefill, 0.1058 -> 0.1051 ms, and slower at hd 128, 1.121 -> 1.218 ms at
  // T = 4096: profiles/r3_flash_prefetch_depth.jsonl.  The PMC there: MFMA
  // pipe 11 % busy, VALU ~30 %, waves waiting the rest.)
  constexpr int NIT = (FA_KB * CH) / 256;
  i32x4 pkA[NIT], pvA[NIT];  // ext vectors: uint4 structs do not promote out of scratch
  auto fetch = [&](int kb0, i32x4(&pk)[NIT], i32x4(&pv)[NIT]) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = it * 256 + tid;
      const int key = e / CH, c = e % CH;
      const int kk = min(kb0 + key, kv_len - 1);
      if (QKV && kk >= p0) {
        pk[it] = *reinterpret_cast<const i32x4*>(krow_new + (size_t)(kk - p0) * ldq + c * 8);
        pv[it] = *reinterpret_cast<const i32x4*>(vrow_new + (size_t)(kk - p0) * ldq + c * 8);
      } else if constexpr (KV8) {
        const uint8_t* kb8 = reinterpret_cast<const uint8_t*>(kc) + ((size_t)b * Hkv + kvh) * S * HD;
        const uint8_t* vb8 = reinterpret_cast<const uint8_t*>(vc) + ((size_t)b * Hkv + kvh) * S * HD;
        pk[it] = kv8_unpack8(*reinterpret_cast<const uint2*>(kb8 + (size_t)kk * HD + c * 8));
        pv[it] = kv8_unpack8(*reinterpret_cast<const uint2*>(vb8 + (size_t)kk * HD + c * 8));
      } else {
        pk[it] = *reinterpret_cast<const i32x4*>(kbase + (size_t)kk * HD + c * 8);
        pv[it] = *reinterpret_cast<const i32x4*>(vbase + (size_t)kk * HD + c * 8);
      }
    }
  };
  auto stage = [&](i32x4(&pk)[NIT], i32x4(&pv)[NIT]) __attribute__((always_inline)) {
    // ---- stage K (swizzled) and V (padded rows) from the prefetch registers ----
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = it * 256 + tid;
      const int key = e / CH, c = e % CH;
      *reinterpret_cast<i32x4*>(ks + key * HD * 2 + (k_swz<HD>(key, c) << 4)) = pk[it];
      *reinterpret_cast<i32x4*>(vs + key * SM::V_STRIDE + c * 16) = pv[it];
    }
  };
  // ---- S^T for two 32-key tiles of the block staged at kbuf ----
  auto s_mfma = [&](const char* kbuf, f32x16(&sacc)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      sacc[kt] = f32x16{};
      const int key = kt * 32 + r32;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kbuf + key * HD * 2 + (k_swz<HD>(key, 2 * s + h) << 4));
        sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kt], 0, 0, 0);
      }
    }
  };
  auto softmax_pv = [&](int kb0, f32x16(&sacc)[2], const char* vbuf) __attribute__((always_inline)) {
    {
      // ---- mask + online softmax (lane = one query; keys in registers) ----
      // VALU is the bound at hd 64 (2 x 8 MFMAs per 64 keys vs ~5 VALU slots per
      // score), so: the mask only runs on blocks that cross this wave's diagonal
      // or the cache end; the max is taken on raw scores (scale > 0), 3-input;
      // the scale folds into the exponent's FMA; v_exp_f32 directly.
      if (kb0 + FA_KB - 1 > wave_qmin || kb0 + FA_KB > kv_len) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int key = kb0 + kt * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
            if (key > q_abs || key >= kv_len) sacc[kt][g] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int g = 0; g < 16; g += 2) mx = fmax_nan(mx, fmax_nan(sacc[kt][g], sacc[kt][g + 1]));
      mx = fmax_nan(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmax_nan(m_i, mx * scale_log2);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_i - m_use);
      // exponent arguments, row sums and the O rescale on packed fp32 math
      // (v_pk_fma / v_pk_add / v_pk_mul: two scores per instruction), only the
      // exponentials per element — the softmax VALU work bounds hd 64
      const f32x2 sl2 = f32x2{scale_log2, scale_log2}, negm = f32x2{-m_use, -m_use};
      f32x2 rs2 = f32x2{0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int g = 0; g < 16; g += 2) {
          const f32x2 arg = f32x2{sacc[kt][g], sacc[kt][g + 1]} * sl2 + negm;
          const f32x2 pv = f32x2{__builtin_amdgcn_exp2f(arg[0]), __builtin_amdgcn_exp2f(arg[1])};
          sacc[kt][g] = pv[0];
          sacc[kt][g + 1] = pv[1];
          rs2 += pv;
        }
      float rs = rs2[0] + rs2[1];
      rs += __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
      m_i = m_new;
      // hd 64 (VALU-bound): the running max rarely moves once the first blocks
      // are in, so skip the rescale when it moved for no query of the wave
      // (0.1120 -> 0.1104 ms on GPT-2 B=64 T=512); at hd 128 the branch costs
      // more than it saves (1.174 -> 1.202 ms at T=4096), the rescale stays
      // unconditional there (profiles/archive/r2_flash_packed_softmax_ab.jsonl)
      if (HD != 64 || !__all(alpha == 1.f)) {
        const f32x2 a2 = f32x2{alpha, alpha};
#pragma unroll
        for (int i = 0; i < NDT; ++i)
#pragma unroll
          for (int g = 0; g < 16; g += 2) {
            const f32x2 o = f32x2{oacc[i][g], oacc[i][g + 1]} * a2;
            oacc[i][g] = o[0];
            oacc[i][g + 1] = o[1];
          }
      }
      // ---- O^T += V^T . P^T ----
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pf;
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[j] = (short)f2bf(sacc[kt][8 * s + j]);
          const int krow = kt * 32 + 16 * s + 4 * h + ((lane & 15) >> 2);
          const int gsub = (lane >> 4) & 1;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const int dcol = dt * 32 + gsub * 16 + 4 * (lane & 3);
            const char* a0 = vbuf + krow * SM::V_STRIDE + dcol * 2;
            const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a0));
            const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a0 + 8 * SM::V_STRIDE));
            bf16x8 vf;
            vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
            vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
            oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[dt], 0, 0, 0);
          }
        }
    }
  };
  auto compute = [&](int kb0) __attribute__((always_inline)) {
    if (kb0 <= wave_qmax) {
      f32x16 sacc[2];
      s_mfma(ks, sacc);
      softmax_pv(kb0, sacc, vs);
    }
  };
  if constexpr (PIPE) {
    // blocks j and j+1 staged in buffers j % 3, (j+1) % 3; block j+2 in the
    // prefetch registers; sc = S of block j.  One barrier per block: past it
    // every wave is done with block j-1, whose buffer takes block j+2.
    auto buf = [&](int j) __attribute__((always_inline)) { return smem + (j % 3) * SM::TOTAL; };
    if (kv_end > 0) {
      fetch(0, pkA, pvA);
      ks = buf(0);
      vs = ks + SM::K_BYTES;
      stage(pkA, pvA);
      if (FA_KB < kv_end) {
        fetch(FA_KB, pkA, pvA);
        ks = buf(1);
        vs = ks + SM::K_BYTES;
        stage(pkA, pvA);
        if (2 * FA_KB < kv_end) fetch(2 * FA_KB, pkA, pvA);
      }
    }
    __syncthreads();
    f32x16 sa[2], sb[2];
    if (kv_end > 0) s_mfma(buf(0), sa);  // block 0 <= wave_qmax always (p0 >= 0)
    auto iter = [&](int j, f32x16(&sc)[2], f32x16(&sn)[2]) __attribute__((always_inline)) {
      const int kb0 = j * FA_KB;
      __syncthreads();
      if (kb0 + 2 * FA_KB < kv_end) {
        ks = buf(j + 2);
        vs = ks + SM::K_BYTES;
        stage(pkA, pvA);
        if (kb0 + 3 * FA_KB < kv_end) fetch(kb0 + 3 * FA_KB, pkA, pvA);
      }
      if (kb0 + FA_KB < kv_end && kb0 + FA_KB <= wave_qmax) s_mfma(buf(j + 1), sn);
      if (kb0 <= wave_qmax) softmax_pv(kb0, sc, buf(j) + SM::K_BYTES);
    };
    for (int j = 0; j * FA_KB < kv_end; j += 2) {
      iter(j, sa, sb);
      if ((j + 1) * FA_KB >= kv_end) break;
      iter(j + 1, sb, sa);
    }
  } else if constexpr (!DB) {
    if (kv_end > 0) fetch(0, pkA, pvA);
    for (int kb0 = 0; kb0 < kv_end; kb0 += FA_KB) {
      stage(pkA, pvA);
      __syncthreads();
      if (kb0 + FA_KB < kv_end) fetch(kb0 + FA_KB, pkA, pvA);
      compute(kb0);
      __syncthreads();
    }
  } else {
    if (kv_end > 0) {
      fetch(0, pkA, pvA);
      stage(pkA, pvA);
      if (FA_KB < kv_end) fetch(FA_KB, pkA, pvA);
    }
    int buf = 0;
    for (int kb0 = 0; kb0 < kv_end; kb0 += FA_KB) {
      // block kb0 is in buffer `buf` and every wave is done with the other one
      __syncthreads();
      ks = smem + buf * SM::TOTAL;
      vs = ks + SM::K_BYTES;
      compute(kb0);
      if (kb0 + FA_KB < kv_end) {
        ks = smem + (buf ^ 1) * SM::TOTAL;
        vs = ks + SM::K_BYTES;
        stage(pkA, pvA);
        if (kb0 + 2 * FA_KB < kv_end) fetch(kb0 + 2 * FA_KB, pkA, pvA);
      }
      buf ^= 1;
    }
  }
  // ---- normalise + store: lane = query, regs = d ----
  if (qrow < T) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    bf16_t* op = o + ((size_t)b * T + qrow) * (size_t)(H * HD) + hh * HD;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * h;
        uint2 w;
        w.x = pack2bf(oacc[dt][4 * g4 + 0] * inv, oacc[dt][4 * g4 + 1] * inv);
        w.y = pack2bf(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d) = w;
      }
  }
}

// ---------------------------------------------------------------------------
// Decode attention (one query token per sequence), split over the key axis.
// grid = (B*Hkv, NS); each workgroup handles the G = H/Hkv query heads of one
// kv head over keys [split*chunk, (split+1)*chunk) ∩ [0, lens[b]) and writes an
// unnormalised partial (o, m, l) to ws; decode_combine merges the splits.
// ---------------------------------------------------------------------------
constexpr int DEC_MAXG = 8;
constexpr int DEC_U = 8;  // key/value rows in flight per thread
static_assert(DEC_U % 2 == 0, "P.V folds key pairs");

// 8 consecutive head-dim elements [8*sub, 8*sub+8) of one head row, RoPE'd
// (rotate-half: element i pairs with i +- hd/2) when ROPE, and
// rounded to bf16 exactly as qkv_split stores them.
template <int HD, bool ROPE>
__device__ __forceinline__ void load_head8(const bf16_t* __restrict__ row, int sub, const float* __restrict__ cosT,
                                           const float* __restrict__ sinT, int p, float out[8]) {
  // branch-free (ROPE is compile-time): every load of a caller's unrolled loop
  // sits in one basic block, so the scheduler issues them all before the first
  // wait instead of one dependent round trip per head
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(row + sub * 8);
  if constexpr (!ROPE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = bf2f_s(x[j]);
  } else {
    constexpr int HALFC = HD / 16;  // 16-B chunks per half row
    const bool lo = sub < HALFC;
    const int psub = lo ? sub + HALFC : sub - HALFC;
    const bf16x8 y = *reinterpret_cast<const bf16x8*>(row + psub * 8);
    const int i0 = (lo ? sub : psub) * 8;
    const float4* cr = reinterpret_cast<const float4*>(cosT + (size_t)p * (HD / 2) + i0);
    const float4* sr = reinterpret_cast<const float4*>(sinT + (size_t)p * (HD / 2) + i0);
    const float4 c0 = cr[0], c1 = cr[1], s0 = sr[0], s1 = sr[1];
    const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // same expression as qkv_split (cache rows must match bit for bit)
      const float a = bf2f_s(x[j]), c = bf2f_s(y[j]);
      const float r = lo ? a * cv[j] - c * sv[j] : a * cv[j] + c * sv[j];
      out[j] = bf2f(f2bf(r));
    }
  }
}

// e4m3 KV cache helpers: 16 floats -> 16 OCP e4m3 bytes (round to nearest,
// saturated to +-448 first: the hardware convert does not clamp), and 16 e4m3
// bytes -> 8 packed bf16 pairs (exact; v_cvt_scalef32_pk_bf16_fp8 at scale 1).
__device__ __forceinline__ void kv8_pack(const float (&x)[16], i32x4& out) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = fminf(fmaxf(x[4 * w + j], -448.f), 448.f);
    int v = 0;
    v = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], v, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], v, true);
    out[w] = v;
  }
}
__device__ __forceinline__ void kv8_unpack(const i32x4& w, uint32_t (&p)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[2 * i] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[i], 1.0f, false));
    p[2 * i + 1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((uint32_t)w[i], 1.0f, true));
  }
}

// FUSED (decode steps): q, the new key (RoPE'd) and value are read straight
// from the QKV projection row of each sequence, the key count is pos[b] + 1,
// and the workgroup whose split holds the new position writes it into the
// cache; its own scores use the register copy, so no other split touches that
// row and there is no qkv_split launch.  Otherwise q is head-major (B,H,hd)
// and lens[b] keys are cached.
// MF: scores on MFMA.  The LDS-score layout (LPK lanes per key, a 4-step DPP
// row reduction per key and head) costs ~20 VALU ops per 4 keys and head; with
// one wave per SIMD (small grids: Llama-3 batch 1 has 8 workgroups) nothing
// hides that and the score loop, not memory, set the kernel time (~1.2 us per
// 128 keys, profiles/archive/r2_attn_decode_phase_probe.jsonl).  With MF a wave
// computes S^T for a tile of 16 keys x 16 query-head columns (G used) as
// HD/32 v_mfma_f32_16x16x32_bf16: lane l feeds key row l&15 (A, straight from
// the cache) and head l&15 (B = q^T, RoPE'd once); C lands as 4 keys x 1 head
// per lane.  Softmax, P.V and the reduction are unchanged.
// KV8: the cache holds OCP e4m3 (unit scale, range +-448; kc/vc are byte
// arrays of the same [B][Hkv][S][HD] shape): a lane's 16-B load is 16 key
// dims instead of 8, so a key row is HD/16 lanes and the K/V bytes per step
// halve; entries are converted to bf16 in registers (exact) before the same
// v_dot2 math, and the new key/value row is rounded to e4m3 once — its score
// uses the rounded copy, so the current step sees what later steps will read.
template <int HD, int G, int FM, bool NT, bool MF = false, bool KV8 = false, int RU = 0>
__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16_t* __restrict__ q, int ldq,
                                                          bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                          float* __restrict__ ws, int H, int Hkv, int S,
                                                          const int* __restrict__ lens, const float* __restrict__ cosT,
                                                          const float* __restrict__ sinT, float scale_log2,
                                                          int chunk_cap, bf16_t* __restrict__ o_direct) {
  constexpr bool FUSED = FM != 0;  // FM: 0 = q head-major + cached keys, 1 = fused QKV rows, 2 = fused + RoPE
  constexpr bool ROPE = FM == 2;
  // rows in flight per thread (RU > 0 overrides): KV8 rows are half the bytes,
  // so 10 rows keep the same bytes in flight and one batch covers 640 keys at
  // hd 64 (the 512-567-token benchmark contexts take one K and one V round
  // trip, not two).  bf16 MHA with 10 or 12 rows measured neutral (GPT-2 B=64
  // 0.585 / 0.584 / 0.590 ms, profiles/archive/r2_decode_rows_in_flight_bf16_ab.jsonl):
  // that path is bound by the K/V bytes, not by its round trips
  constexpr int DEC_U = RU > 0 ? RU : (KV8 ? 10 : dnn::DEC_U);
  static_assert(DEC_U % 2 == 0, "P.V folds key pairs");
  constexpr int ELT = KV8 ? 16 : 8;     // head dims per 16-B lane load
  constexpr int LPK = HD / ELT;         // lanes per key row (16 B each)
  constexpr int GPB = 256 / LPK;        // key groups per block
  extern __shared__ __attribute__((aligned(16))) float dsm[];   // [G][chunk_cap] scores, then reduction scratch
  const int bk = blockIdx.x, split = blockIdx.y, NS = gridDim.y;
  DEC_PROBE(0, 0);
  const int b = bk / Hkv, kvh = bk % Hkv;
  const int p_new = FUSED ? lens[b] : 0;  // FUSED: lens = positions already cached
  const int len = FUSED ? min(p_new + 1, S) : min(lens[b], S);  // never read past the cache capacity
  // splits share the *runtime* length evenly (one captured graph serves every step)
  const int chunk = (len + NS - 1) / NS;
  const int k0 = split * chunk, k1 = min(len, k0 + chunk);
  DEC_PROBE(1, k1);
  const int tid = threadIdx.x, sub = tid % LPK, grp = tid / LPK;
  float* wsp = ws + ((size_t)bk * NS + split) * G * (HD + 2);
  if (k0 >= k1) {
    for (int i = tid; i < G * (HD + 2); i += 256) {
      const int c = i % (HD + 2);
      wsp[i] = c == HD ? -INFINITY : 0.f;
    }
    return;
  }
  bf16_t* kb = kc + ((size_t)b * Hkv + kvh) * S * HD;
  bf16_t* vb = vc + ((size_t)b * Hkv + kvh) * S * HD;
  constexpr int EB = KV8 ? 1 : 2;  // cache bytes per element
  uint8_t* kb8 = reinterpret_cast<uint8_t*>(kc) + ((size_t)b * Hkv + kvh) * S * HD * EB;
  uint8_t* vb8 = reinterpret_cast<uint8_t*>(vc) + ((size_t)b * Hkv + kvh) * S * HD * EB;
  float qv[G][ELT];
  float nk[ELT] = {}, nv[ELT] = {};
  // FUSED: is the new key inside this split (and inside the cache)?
  const bool own_new = FUSED && p_new < S && p_new >= k0 && p_new < k1;
  if constexpr (FUSED) {
    const bf16_t* row = q + (size_t)b * ldq;
    const int pr = min(p_new, S - 1);  // RoPE table row (overflow is dropped, never read out of bounds)
    if constexpr (!MF) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int h8 = 0; h8 < ELT / 8; ++h8)
          load_head8<HD, ROPE>(row + (kvh * G + g) * HD, sub * (ELT / 8) + h8, cosT, sinT, pr, qv[g] + 8 * h8);
    }
    // new key / value: loaded unconditionally (used only when own_new), no branch
#pragma unroll
    for (int h8 = 0; h8 < ELT / 8; ++h8) {
      load_head8<HD, ROPE>(row + (H + kvh) * HD, sub * (ELT / 8) + h8, cosT, sinT, pr, nk + 8 * h8);
      load_head8<HD, false>(row + (H + Hkv + kvh) * HD, sub * (ELT / 8) + h8, nullptr, nullptr, 0, nv + 8 * h8);
    }
  } else if constexpr (!MF) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int h8 = 0; h8 < ELT / 8; ++h8) {
        const bf16x8 pq = *reinterpret_cast<const bf16x8*>(q + ((size_t)b * H + kvh * G + g) * HD + sub * ELT + 8 * h8);
#pragma unroll
        for (int j = 0; j < 8; ++j) qv[g][8 * h8 + j] = bf2f_s(pq[j]);
      }
  }
  const int knew = own_new ? p_new - k0 : -1;  // split-relative index of the register-held key
  // q and the new key are bf16-exact (rounded after RoPE): pack them into bf16
  // pairs so a score is 4 v_dot2_f32_bf16 per lane instead of 8 converts + 8 FMAs.
  uint32_t qp[G][ELT / 2], nkp[ELT / 2];  // bf16 pairs, reinterpreted only at the dot2 call
  if constexpr (!MF) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < ELT / 2; ++j) qp[g][j] = pack2bf(qv[g][2 * j], qv[g][2 * j + 1]);
  }
  uint32_t nvp[ELT / 2];
  i32x4 nk8 = {0, 0, 0, 0}, nv8 = {0, 0, 0, 0};  // KV8: the new row as stored (e4m3)
  if constexpr (KV8) {
    kv8_pack(nk, nk8);
    kv8_pack(nv, nv8);
    kv8_unpack(nk8, nkp);  // the register copy = what the cache will hold
    kv8_unpack(nv8, nvp);
  } else {
#pragma unroll
    for (int j = 0; j < ELT / 2; ++j) nkp[j] = pack2bf(nk[j * 2], nk[j * 2 + 1]);
#pragma unroll
    for (int j = 0; j < ELT / 2; ++j) nvp[j] = pack2bf(nv[j * 2], nv[j * 2 + 1]);
  }
  float* sc = dsm;  // [G][chunk]
  const int n = k1 - k0;
  DEC_PROBE(2, nvp[0]);
  if constexpr (MF) {
    static_assert(G <= 16, "MFMA score tile has 16 head columns");
    constexpr int NKC = HD / 32;  // k-steps of 32 dims
    constexpr int TB = 4;         // key tiles in flight per wave
    const int lane = tid & 63, wave = tid >> 6, hj = lane & 15, c4 = lane >> 4;
    bf16x8 qB[NKC], nkA[NKC];
#pragma unroll
    for (int m = 0; m < NKC; ++m) {
      float t8[8];
      const int hq = min(hj, G - 1);  // columns >= G load a valid head and are zeroed (no branch)
      if constexpr (FUSED) {
        load_head8<HD, ROPE>(q + (size_t)b * ldq + (kvh * G + hq) * HD, c4 + 4 * m, cosT, sinT, min(p_new, S - 1), t8);
      } else {
        const bf16x8 pq = *reinterpret_cast<const bf16x8*>(q + ((size_t)b * H + kvh * G + hq) * HD + (c4 + 4 * m) * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) t8[j] = bf2f_s(pq[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) qB[m][j] = hj < G ? (short)f2bf(t8[j]) : (short)0;
      if constexpr (FUSED) {  // the new key in A layout (rows of its tile come from registers)
        load_head8<HD, ROPE>(q + (size_t)b * ldq + (H + kvh) * HD, c4 + 4 * m, cosT, sinT, min(p_new, S - 1), t8);
#pragma unroll
        for (int j = 0; j < 8; ++j) nkA[m][j] = (short)f2bf(t8[j]);
        if constexpr (KV8)  // the register copy = the stored e4m3 row
          nkA[m] = __builtin_bit_cast(bf16x8, kv8_unpack8(kv8_pack8(__builtin_bit_cast(i32x4, nkA[m]))));
      }
    }
    const int ntile = (n + 15) / 16;
    for (int t0 = 0; t0 < ntile; t0 += 4 * TB) {
      bf16x8 ka[TB][NKC];
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) {
        const int kk = min((t0 + tb * 4 + wave) * 16 + hj, n - 1);
#pragma unroll
        for (int m = 0; m < NKC; ++m) {
          if constexpr (KV8) {  // 8 e4m3 entries -> the same bf16 A fragment
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const u32x2* kp8 = reinterpret_cast<const u32x2*>(kb8 + (size_t)(k0 + kk) * HD + (c4 + 4 * m) * 8);
            const u32x2 w = NT ? __builtin_nontemporal_load(kp8) : *kp8;
            ka[tb][m] = __builtin_bit_cast(bf16x8, kv8_unpack8(make_uint2(w[0], w[1])));
          } else {
            const bf16x8* kp = reinterpret_cast<const bf16x8*>(kb + (size_t)(k0 + kk) * HD + (c4 + 4 * m) * 8);
            ka[tb][m] = NT ? __builtin_nontemporal_load(kp) : *kp;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (t0 == 0) DEC_PROBE(8, ka[0][0][0]);
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) {
        const int t = t0 + tb * 4 + wave;
        if (t >= ntile) break;  // wave-uniform
        if (FUSED && t * 16 + hj == knew) {
#pragma unroll
          for (int m = 0; m < NKC; ++m) ka[tb][m] = nkA[m];
        }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < NKC; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[tb][m], qB[m], acc, 0, 0, 0);
        if (t0 == 0 && tb == 0) DEC_PROBE(9, acc[0]);
        if (hj < G) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = t * 16 + c4 * 4 + r;
            if (key < n) sc[hj * chunk_cap + key] = acc[r] * scale_log2;
          }
        }
      }
    }
  } else {
  // Scores: batches of DEC_U key rows per thread, all loads issued before the
  // first use (memory-level parallelism is the whole game in decode).
  for (int kb0 = 0; kb0 < n; kb0 += GPB * DEC_U) {
    bf16x8 kr[DEC_U];
#pragma unroll
    for (int u = 0; u < DEC_U; ++u) {
      const int kk = min(kb0 + u * GPB + grp, n - 1);
      // NT: the caches are far larger than L2 / MALL and every row is read once
      // per step, so stream them non-temporally (GPT-2 B=64: 0.658 -> 0.590 ms
      // per decode step); small caches (batch 1) stay cacheable: they live in
      // the MALL from one step to the next
      const bf16x8* kp = reinterpret_cast<const bf16x8*>(kb8 + ((size_t)(k0 + kk) * HD + sub * ELT) * EB);
      kr[u] = NT ? __builtin_nontemporal_load(kp) : *kp;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < DEC_U; ++u) {
      if (kb0 + u * GPB >= n) break;  // workgroup-uniform: the rest of the batch is past the context
      const int kk = kb0 + u * GPB + grp;
      uint32_t kp[ELT / 2];
      if constexpr (KV8) {
        kv8_unpack(__builtin_bit_cast(i32x4, kr[u]), kp);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) kp[j] = (uint32_t)(uint16_t)kr[u][2 * j] | ((uint32_t)(uint16_t)kr[u][2 * j + 1] << 16);
      }
      if (FUSED && kk == knew) {
#pragma unroll
        for (int j = 0; j < ELT / 2; ++j) kp[j] = nkp[j];
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < ELT / 2; ++j) d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, qp[g][j]), __builtin_bit_cast(bf16x2v, kp[j]), d, false);
        d = group_sum<LPK>(d);  // DPP row reduction over the LPK lanes of this key
        if (sub == 0 && kk < n) sc[g * chunk_cap + kk] = d * scale_log2;
      }
    }
  }
  }
  DEC_PROBE(10, 0);
  // first batch of value rows: requested now, in flight across the barrier and
  // the softmax (they depend only on the key range).  Issuing it before the
  // score loop instead measured slower on the e4m3 path (GPT-2 B=64 0.523 ->
  // 0.531 ms, B=256 1.053 -> 1.108: 142 VGPRs, profiles/archive/r2_kv8_v_early_ab.jsonl)
  bf16x8 vr0[DEC_U];
#pragma unroll
  for (int u = 0; u < DEC_U; ++u) {
    const int kk = min(u * GPB + grp, n - 1);
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vb8 + ((size_t)(k0 + kk) * HD + sub * ELT) * EB);
    vr0[u] = NT ? __builtin_nontemporal_load(vp) : *vp;
  }
  __syncthreads();
  DEC_PROBE(3, 0);
  // per-head max and exp (one wave per head, strided)
  __shared__ float mh[DEC_MAXG], lh[DEC_MAXG];
  const int wave = tid >> 6, lane = tid & 63;
  for (int g = wave; g < G; g += 4) {
    float mx = -INFINITY;
    for (int i = lane; i < n; i += 64) mx = fmaxf(mx, sc[g * chunk_cap + i]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float e = exp2f(sc[g * chunk_cap + i] - mx);
      sc[g * chunk_cap + i] = e;
      s += e;
    }
    s = wave_sum(s);
    if (lane == 0) { mh[g] = mx; lh[g] = s; }
  }
  __syncthreads();
  DEC_PROBE(4, 0);
  // P.V: thread owns d chunk `sub` for key group `grp`
  float acc[G][ELT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < ELT; ++j) acc[g][j] = 0.f;
  for (int kb0 = 0; kb0 < n; kb0 += GPB * DEC_U) {
    bf16x8 vr[DEC_U];
    if (kb0 == 0) {
#pragma unroll
      for (int u = 0; u < DEC_U; ++u) vr[u] = vr0[u];
    } else {
#pragma unroll
      for (int u = 0; u < DEC_U; ++u) {
        const int kk = min(kb0 + u * GPB + grp, n - 1);
        const bf16x8* vp = reinterpret_cast<const bf16x8*>(vb8 + ((size_t)(k0 + kk) * HD + sub * ELT) * EB);
        vr[u] = NT ? __builtin_nontemporal_load(vp) : *vp;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // Key pairs (u, u+1) of this thread share the d chunk: interleave their
    // value rows into bf16 pairs (v_perm) and fold both probabilities, rounded
    // to bf16 as in an MFMA P.V, into one v_dot2_f32_bf16 per element.
#pragma unroll
    for (int u = 0; u < DEC_U; u += 2) {
      if (kb0 + u * GPB >= n) break;  // workgroup-uniform, as in the score loop
      const int ka = kb0 + u * GPB + grp, kz = ka + GPB;
      uint32_t wa[ELT / 2], wz[ELT / 2];
      if constexpr (KV8) {
        kv8_unpack(__builtin_bit_cast(i32x4, vr[u]), wa);
        kv8_unpack(__builtin_bit_cast(i32x4, vr[u + 1]), wz);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wa[j] = (uint32_t)(uint16_t)vr[u][2 * j] | ((uint32_t)(uint16_t)vr[u][2 * j + 1] << 16);
          wz[j] = (uint32_t)(uint16_t)vr[u + 1][2 * j] | ((uint32_t)(uint16_t)vr[u + 1][2 * j + 1] << 16);
        }
      }
      if (FUSED && ka == knew) {
#pragma unroll
        for (int j = 0; j < ELT / 2; ++j) wa[j] = nvp[j];
      }
      if (FUSED && kz == knew) {
#pragma unroll
        for (int j = 0; j < ELT / 2; ++j) wz[j] = nvp[j];
      }
      uint32_t pr[ELT];  // element e of both rows: (row u, row u+1)
#pragma unroll
      for (int j = 0; j < ELT / 2; ++j) {
        pr[2 * j] = __builtin_amdgcn_perm(wz[j], wa[j], 0x05040100u);
        pr[2 * j + 1] = __builtin_amdgcn_perm(wz[j], wa[j], 0x07060302u);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pa = ka < n ? sc[g * chunk_cap + ka] : 0.f;
        const float pz = kz < n ? sc[g * chunk_cap + kz] : 0.f;
        const bf16x2v pp = __builtin_bit_cast(bf16x2v, pack2bf(pa, pz));
#pragma unroll
        for (int j = 0; j < ELT; ++j)
          acc[g][j] = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2v, pr[j]), acc[g][j], false);
      }
    }
  }
  DEC_PROBE(5, acc[0][0]);
  __syncthreads();  // scores no longer needed: reuse dsm as [GPB][G][HD] reduction scratch
  float* red = dsm;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < ELT; ++j) red[((size_t)grp * G + g) * HD + sub * ELT + j] = acc[g][j];
  __syncthreads();
  for (int i = tid; i < G * HD; i += 256) {
    const int g = i / HD, d = i % HD;
    float s = 0.f;
    for (int r = 0; r < GPB; ++r) s += red[((size_t)r * G + g) * HD + d];
    if (NS == 1) {  // single split: normalise and write the output directly (no combine pass)
      o_direct[(size_t)b * H * HD + (kvh * G + g) * HD + d] = f2bf(s / lh[g]);
    } else {
      wsp[g * (HD + 2) + d] = s;
    }
  }
  if (NS > 1 && tid < G) {
    wsp[tid * (HD + 2) + HD] = mh[tid];
    wsp[tid * (HD + 2) + HD + 1] = lh[tid];
  }
  // the new key / value row into the cache, last: a store issued before the
  // K/V loads would sit in front of them in this wave's vmcnt queue
  if (KV8 && FUSED && own_new && grp == 0) {
    *reinterpret_cast<i32x4*>(kb8 + (size_t)p_new * HD + sub * 16) = nk8;
    *reinterpret_cast<i32x4*>(vb8 + (size_t)p_new * HD + sub * 16) = nv8;
  } else if (FUSED && own_new && grp == 0) {
    uint4 wk, wv;
    uint32_t* pk = reinterpret_cast<uint32_t*>(&wk);
    uint32_t* pv = reinterpret_cast<uint32_t*>(&wv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pk[j] = nkp[j];
      pv[j] = nvp[j];
    }
    *reinterpret_cast<uint4*>(kb + (size_t)p_new * HD + sub * 8) = wk;
    *reinterpret_cast<uint4*>(vb + (size_t)p_new * HD + sub * 8) = wv;
  }
  DEC_PROBE(7, 0);
}

// ---------------------------------------------------------------------------
// One-pass decode attention (round 3): every key and value row of a split is
// requested before the first score is formed, so a workgroup's whole K/V
// range is in flight at once instead of one batch per round trip.
//
// attn_decode_kernel above runs K batch -> scores -> softmax pass -> V batch
// -> P.V -> V batch ...: at Llama-3 8B B=32 (B*Hkv = 256, 3 splits of ~180
// keys) that chain ran at 3.5 TB/s plus a 4.8 us combine launch, at GPT-2
// B=64 at 5.0 TB/s.  Here, for a split of at most CAP = NW*KT*16 keys:
//   1. q / new key / new value (first in the vmcnt queue), then every K tile
//      of the wave (KT x HD/32 16-B loads per lane), then the first VE value
//      rows of the thread;
//   2. scores on MFMA as K lands (16 keys x 16 head columns per tile, lane =
//      key row, B = q^T), written to LDS, and each wave's per-head max kept
//      in registers -> LDS (no separate max pass);
//   3. the remaining value rows are issued as soon as the K registers are
//      free, then one barrier;
//   4. P.V on v_dot2 (thread = 8 dims of VU rows), exponentials taken where
//      they are used, row sums carried beside the accumulators;
//   5. one LDS reduction over the row groups, output written directly (one
//      split) or as the (o, m, l) partial decode_combine_kernel merges.
// Cache rows past the runtime length are never scored: their loads are
// clamped to the last valid row (same address: coalesced).
template <int HD, int G, int FM, bool NT, int NW, int KT, int VE, int VU, bool RS = false, bool KNT = NT,
          bool KF = false>
__global__ __launch_bounds__(NW * 64) void attn_decode_1p_kernel(const bf16_t* __restrict__ q, int ldq,
                                                               bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                               float* __restrict__ ws, int H, int Hkv, int S,
                                                               const int* __restrict__ lens,
                                                               const float* __restrict__ cosT,
                                                               const float* __restrict__ sinT, float scale_log2,
                                                               bf16_t* __restrict__ o_direct) {
  // RS: scores in the row layout (thread = 8 dims of key rows grp + GPB*u, dot2
  // + DPP row sum, as the value rows) instead of MFMA key tiles; KNT: the key
  // loads non-temporal (NT: the value loads)
  constexpr bool FUSED = FM != 0, ROPE = FM == 2;
  constexpr int NTH = NW * 64;
  constexpr int LPK = HD / 8;          // lanes per value row (16 B = 8 dims each)
  constexpr int GPB = NTH / LPK;       // value row groups
  constexpr int NKC = HD / 32;         // MFMA k-steps of a key tile
  constexpr int CAP = RS ? GPB * VU : NW * KT * 16;  // keys per split (host-checked)
  constexpr int KR = RS ? VU : 1;      // key rows per thread (RS)
  static_assert(GPB * VU >= CAP, "value rows must cover the key tiles");
  static_assert(VE <= VU && VU % 2 == 0 && G <= 16, "bad shape");
  __shared__ __attribute__((aligned(16))) float sc[CAP * G];  // scaled scores, [key][head] (one LDS read per key)
  __shared__ float wmax[NW][G];        // per-wave score max per head
  extern __shared__ __attribute__((aligned(16))) float red1p[];  // [NW][G][HD] + [NW][G]

  const int bk = blockIdx.x, split = blockIdx.y, NS = gridDim.y;
  const int b = bk / Hkv, kvh = bk % Hkv;
  const int p_new = FUSED ? lens[b] : 0;
  const int len = FUSED ? min(p_new + 1, S) : min(lens[b], S);
  const int chunk = (len + NS - 1) / NS;
  const int k0 = split * chunk, k1 = min(len, k0 + chunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hj = lane & 15, c4 = lane >> 4;
  const int sub = tid % LPK, grp = tid / LPK;
  float* wsp = ws + ((size_t)bk * NS + split) * G * (HD + 2);
  if (k0 >= k1) {  // empty split (short context): neutral partial
    for (int i = tid; i < G * (HD + 2); i += NTH) wsp[i] = (i % (HD + 2)) == HD ? -INFINITY : 0.f;
    return;
  }
  const int n = k1 - k0;
  bf16_t* kb = kc + ((size_t)b * Hkv + kvh) * S * HD + (size_t)k0 * HD;
  bf16_t* vb = vc + ((size_t)b * Hkv + kvh) * S * HD + (size_t)k0 * HD;
  const bool own_new = FUSED && p_new < S && p_new >= k0 && p_new < k1;
  const int knew = own_new ? p_new - k0 : -1;
  const int pr = min(p_new, S - 1);

  // ---- K: MFMA tiles t = wave + NW*i (lane loads key row t*16 + hj, dims
  // (c4 + 4m)*8), or RS rows grp + GPB*u (dims sub*8); then the first VE value
  // rows (row grp + GPB*u, dims sub*8).  KF: issued before q, so the K/V
  // stream starts without waiting for q (and the RoPE tables); q then lands
  // behind them in the vmcnt queue, which the scores wait for anyway
  bf16x8 ka[RS ? 1 : KT][NKC];
  bf16x8 kr[KR];
  bf16x8 vr[VU];
  auto issue_kv = [&]() __attribute__((always_inline)) {
    if constexpr (!RS) {
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        const int kk = min((wave + NW * i) * 16 + hj, n - 1);
#pragma unroll
        for (int m = 0; m < NKC; ++m) {
          const bf16x8* kp = reinterpret_cast<const bf16x8*>(kb + (size_t)kk * HD + (c4 + 4 * m) * 8);
          ka[i][m] = KNT ? __builtin_nontemporal_load(kp) : *kp;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const bf16x8* kp = reinterpret_cast<const bf16x8*>(kb + (size_t)min(grp + GPB * u, n - 1) * HD + sub * 8);
        kr[u] = KNT ? __builtin_nontemporal_load(kp) : *kp;
      }
    }
#pragma unroll
    for (int u = 0; u < VE; ++u) {
      const bf16x8* vp = reinterpret_cast<const bf16x8*>(vb + (size_t)min(grp + GPB * u, n - 1) * HD + sub * 8);
      vr[u] = NT ? __builtin_nontemporal_load(vp) : *vp;
    }
  };
  if constexpr (KF) {
    issue_kv();
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- 1. q (MFMA: q^T B operand with columns >= G zero, new key in A layout;
  // RS: bf16 pairs of this thread's 8 dims per head), new k/v (row layout)
  bf16x8 qB[NKC], nkA[NKC];
  uint32_t qp[RS ? G : 1][4];
  if constexpr (!RS) {
#pragma unroll
    for (int m = 0; m < NKC; ++m) {
      float t8[8];
      const int hq = min(hj, G - 1);
      if constexpr (FUSED) {
        load_head8<HD, ROPE>(q + (size_t)b * ldq + (kvh * G + hq) * HD, c4 + 4 * m, cosT, sinT, pr, t8);
      } else {
        const bf16x8 pq =
            *reinterpret_cast<const bf16x8*>(q + ((size_t)b * H + kvh * G + hq) * HD + (c4 + 4 * m) * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) t8[j] = bf2f_s(pq[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) qB[m][j] = hj < G ? (short)f2bf(t8[j]) : (short)0;
      if constexpr (FUSED) {
        load_head8<HD, ROPE>(q + (size_t)b * ldq + (H + kvh) * HD, c4 + 4 * m, cosT, sinT, pr, t8);
#pragma unroll
        for (int j = 0; j < 8; ++j) nkA[m][j] = (short)f2bf(t8[j]);
      }
    }
  } else {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float t8[8];
      if constexpr (FUSED) {
        load_head8<HD, ROPE>(q + (size_t)b * ldq + (kvh * G + g) * HD, sub, cosT, sinT, pr, t8);
      } else {
        const bf16x8 pq = *reinterpret_cast<const bf16x8*>(q + ((size_t)b * H + kvh * G + g) * HD + sub * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) t8[j] = bf2f_s(pq[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) qp[g][j] = pack2bf(t8[2 * j], t8[2 * j + 1]);
    }
  }
  uint32_t nkp[4] = {0, 0, 0, 0}, nvp[4] = {0, 0, 0, 0};  // this thread's 8 dims of the new row (bf16 pairs)
  if constexpr (FUSED) {
    float nk[8], nv[8];
    load_head8<HD, ROPE>(q + (size_t)b * ldq + (H + kvh) * HD, sub, cosT, sinT, pr, nk);
    load_head8<HD, false>(q + (size_t)b * ldq + (H + Hkv + kvh) * HD, sub, nullptr, nullptr, 0, nv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      nkp[j] = pack2bf(nk[2 * j], nk[2 * j + 1]);
      nvp[j] = pack2bf(nv[2 * j], nv[2 * j + 1]);
    }
  }
  if constexpr (!KF) issue_kv();
  __builtin_amdgcn_sched_barrier(0);

  // ---- 2. scores (scaled to log2 units) + this wave's max per head
  if constexpr (!RS) {
    float mx = -INFINITY;  // lane's head hj
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      const int t = wave + NW * i;
      if (t * 16 >= n) break;  // wave-uniform
      if (FUSED && t * 16 + hj == knew) {
#pragma unroll
        for (int m = 0; m < NKC; ++m) ka[i][m] = nkA[m];
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NKC; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[i][m], qB[m], acc, 0, 0, 0);
      if (hj < G) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = t * 16 + c4 * 4 + r;
          if (key < n) {
            const float s = acc[r] * scale_log2;
            sc[key * G + hj] = s;
            mx = fmaxf(mx, s);
          }
        }
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (lane < G) wmax[wave][lane] = mx;
  } else {
    float mx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) mx[g] = -INFINITY;
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      if (GPB * u >= n) break;  // workgroup-uniform
      const int row = grp + GPB * u;
      uint32_t kp[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) kp[j] = (uint32_t)(uint16_t)kr[u][2 * j] | ((uint32_t)(uint16_t)kr[u][2 * j + 1] << 16);
      if (FUSED && row == knew) {
#pragma unroll
        for (int j = 0; j < 4; ++j) kp[j] = nkp[j];
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, qp[g][j]), __builtin_bit_cast(bf16x2v, kp[j]),
                                              d, false);
        d = group_sum<LPK>(d) * scale_log2;
        if (row < n) {
          if (sub == 0) sc[row * G + g] = d;
          mx[g] = fmaxf(mx[g], d);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float m = wave_max(mx[g]);
      if (lane == 0) wmax[wave][g] = m;
    }
  }
  // ---- 3. the remaining value rows (the K registers are free now)
#pragma unroll
  for (int u = VE; u < VU; ++u) {
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vb + (size_t)min(grp + GPB * u, n - 1) * HD + sub * 8);
    vr[u] = NT ? __builtin_nontemporal_load(vp) : *vp;
  }
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();
  float mg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = wmax[0][g];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = fmaxf(m, wmax[w][g]);
    mg[g] = m;
  }
  // ---- 4. probabilities, once per (key, head): the whole workgroup
  // exponentiates the score array in place (a thread of P.V would otherwise
  // take the same exponential as the other LPK - 1 lanes of its row)
  for (int i = tid; i < n * G; i += NTH) {
    const int g = i % G;
    float m = mg[0];
#pragma unroll
    for (int gg = 1; gg < G; ++gg) m = g == gg ? mg[gg] : m;
    sc[i] = __builtin_amdgcn_exp2f(sc[i] - m);
  }
  __syncthreads();
  // ---- 5. P.V: key pairs (u, u+1) share this thread's 8 dims; the
  // probabilities of 4 rows are read together (one ds_read per row) so the
  // LDS round trips overlap instead of one read -> wait -> use per head
  float acc[G][8], ls[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    ls[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }
  static_assert(VU % 4 == 0, "P.V reads probabilities 4 rows at a time");
#pragma unroll
  for (int u0 = 0; u0 < VU; u0 += 4) {
    if (GPB * u0 >= n) break;  // workgroup-uniform
    float pr4[4][G];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = grp + GPB * (u0 + q);
      const float* sp = sc + min(row, n - 1) * G;
      if constexpr (G == 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(sp);
#pragma unroll
        for (int g = 0; g < 4; ++g) pr4[q][g] = row < n ? v[g] : 0.f;
      } else if constexpr (G == 2) {
        const f32x2 v = *reinterpret_cast<const f32x2*>(sp);
#pragma unroll
        for (int g = 0; g < 2; ++g) pr4[q][g] = row < n ? v[g] : 0.f;
      } else {
#pragma unroll
        for (int g = 0; g < G; ++g) pr4[q][g] = row < n ? sp[g] : 0.f;
      }
    }
#pragma unroll
    for (int u = u0; u < u0 + 4; u += 2) {
      const int ka_ = grp + GPB * u, kz = ka_ + GPB;
      uint32_t wa[4], wz[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wa[j] = (uint32_t)(uint16_t)vr[u][2 * j] | ((uint32_t)(uint16_t)vr[u][2 * j + 1] << 16);
        wz[j] = (uint32_t)(uint16_t)vr[u + 1][2 * j] | ((uint32_t)(uint16_t)vr[u + 1][2 * j + 1] << 16);
      }
      if (FUSED && ka_ == knew) {
#pragma unroll
        for (int j = 0; j < 4; ++j) wa[j] = nvp[j];
      }
      if (FUSED && kz == knew) {
#pragma unroll
        for (int j = 0; j < 4; ++j) wz[j] = nvp[j];
      }
      uint32_t prr[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        prr[2 * j] = __builtin_amdgcn_perm(wz[j], wa[j], 0x05040100u);
        prr[2 * j + 1] = __builtin_amdgcn_perm(wz[j], wa[j], 0x07060302u);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pa = pr4[u - u0][g], pz = pr4[u - u0 + 1][g];
        ls[g] += pa + pz;
        const bf16x2v pp = __builtin_bit_cast(bf16x2v, pack2bf(pa, pz));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[g][j] = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2v, prr[j]), acc[g][j], false);
      }
    }
  }
  // ---- 6. reduce over the row groups: first across the wave's 64 / LPK row
  // groups by lane shuffles (xor LPK, 2 LPK, ...), then the NW wave sums
  // through LDS -- [NW][G][HD] instead of [GPB][G][HD] (Llama-3 8B: 16 KB
  // instead of 64 KB of LDS, so two GQA workgroups fit on a CU)
  float* red = red1p;                  // [NW][G][HD]
  float* lred = red1p + NW * G * HD;   // [NW][G]
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] += __shfl_xor(acc[g][j], off, 64);
      ls[g] += __shfl_xor(ls[g], off, 64);
    }
  }
  if (lane < LPK) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4* dst = reinterpret_cast<f32x4*>(red + ((size_t)wave * G + g) * HD + sub * 8);
      dst[0] = f32x4{acc[g][0], acc[g][1], acc[g][2], acc[g][3]};
      dst[1] = f32x4{acc[g][4], acc[g][5], acc[g][6], acc[g][7]};
      if (sub == 0) lred[wave * G + g] = ls[g];
    }
  }
  __syncthreads();
  for (int i = tid; i < G * HD; i += NTH) {
    const int g = i / HD, d = i % HD;
    float s = 0.f, l = 0.f;
#pragma unroll
    for (int r = 0; r < NW; ++r) {
      s += red[((size_t)r * G + g) * HD + d];
      l += lred[r * G + g];
    }
    if (NS == 1) {
      o_direct[(size_t)b * H * HD + (kvh * G + g) * HD + d] = f2bf(l > 0.f ? s / l : 0.f);
    } else {
      wsp[g * (HD + 2) + d] = s;
      if (d == 0) {
        wsp[g * (HD + 2) + HD] = mg[g];
        wsp[g * (HD + 2) + HD + 1] = l;
      }
    }
  }
  // the new key / value row into the cache, last (behind every K/V load of this wave)
  if (own_new && grp == 0) {
    uint4 wk, wv;
    wk.x = nkp[0]; wk.y = nkp[1]; wk.z = nkp[2]; wk.w = nkp[3];
    wv.x = nvp[0]; wv.y = nvp[1]; wv.z = nvp[2]; wv.w = nvp[3];
    bf16_t* kr = kc + ((size_t)b * Hkv + kvh) * S * HD + (size_t)p_new * HD + sub * 8;
    bf16_t* vrp = vc + ((size_t)b * Hkv + kvh) * S * HD + (size_t)p_new * HD + sub * 8;
    *reinterpret_cast<uint4*>(kr) = wk;
    *reinterpret_cast<uint4*>(vrp) = wv;
  }
}

// (Folding this pass into the attention kernel — the last-arriving split
// combines, tickets behind an agent-scope release / acquire — measured 20 %
// slower on Llama-3 8B B=32 decode, 4.49 -> 5.39 ms/step: every split pays the
// release fence's L2 write-back.  profiles/archive/r2_decode_fold_combine_ab.jsonl;
// write-through sc1 stores + sc1 loads without the fences read stale partials.)
// Up to NSMAX splits: every partial of the thread's head dim is requested
// before the first use (one memory round trip instead of the loop below's
// three dependent ones); the same arithmetic in the same order, so the output
// is bit-identical.
template <int NSMAX>
__global__ void decode_combine_fast_kernel(const float* __restrict__ ws, bf16_t* __restrict__ o, int B, int H,
                                           int Hkv, int HD, int NS) {
  const int bh = blockIdx.x;  // b*H + h
  const int b = bh / H, hh = bh % H;
  const int G = H / Hkv, kvh = hh / G, g = hh % G;
  const float* base = ws + ((size_t)(b * Hkv + kvh) * NS) * G * (HD + 2) + g * (HD + 2);
  const size_t step = (size_t)G * (HD + 2);
  float ms[NSMAX], ls[NSMAX], os[NSMAX];
#pragma unroll
  for (int s = 0; s < NSMAX; ++s) {
    const bool ok = s < NS;
    const float* p = base + (ok ? s : 0) * step;
    ms[s] = ok ? p[HD] : -INFINITY;
    ls[s] = ok ? p[HD + 1] : 0.f;
    os[s] = (ok && (int)threadIdx.x < HD) ? p[threadIdx.x] : 0.f;
  }
  float m = -INFINITY;
#pragma unroll
  for (int s = 0; s < NSMAX; ++s) m = fmaxf(m, ms[s]);
  float l = 0.f, acc = 0.f;
#pragma unroll
  for (int s = 0; s < NSMAX; ++s) {
    if (ms[s] != -INFINITY) {
      const float e = exp2f(ms[s] - m);
      l += ls[s] * e;
      acc += os[s] * e;
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if ((int)threadIdx.x < HD) o[(size_t)b * H * HD + hh * HD + threadIdx.x] = f2bf(acc * inv);
}

__global__ void decode_combine_kernel(const float* __restrict__ ws, bf16_t* __restrict__ o, int B, int H, int Hkv,
                                      int HD, int NS) {
  const int bh = blockIdx.x;  // b*H + h
  const int b = bh / H, hh = bh % H;
  const int G = H / Hkv, kvh = hh / G, g = hh % G;
  const float* base = ws + ((size_t)(b * Hkv + kvh) * NS) * G * (HD + 2) + g * (HD + 2);
  float m = -INFINITY;
  for (int s = 0; s < NS; ++s) m = fmaxf(m, base[(size_t)s * G * (HD + 2) + HD]);
  float l = 0.f;
  for (int s = 0; s < NS; ++s) {
    const float ms = base[(size_t)s * G * (HD + 2) + HD];
    if (ms != -INFINITY) l += base[(size_t)s * G * (HD + 2) + HD + 1] * exp2f(ms - m);
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  for (int d = threadIdx.x; d < HD; d += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < NS; ++s) {
      const float ms = base[(size_t)s * G * (HD + 2) + HD];
      if (ms != -INFINITY) acc += base[(size_t)s * G * (HD + 2) + d] * exp2f(ms - m);
    }
    o[(size_t)b * H * HD + hh * HD + d] = f2bf(acc * inv);
  }
}

}  // namespace dnn

using namespace dnn;

extern "C" int dnn_qkv_split(const void* qkv, void* q, void* kc, void* vc, int B, int T, int H, int Hkv, int hd, int S,
                             const int* pos, const float* cos, const float* sin, int rope, hipStream_t st, int kv8) {
  if (hd % 16 != 0 || H % Hkv != 0) return -1;
  const long total = (long)B * T * (H + 2 * Hkv) * (hd / 16);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(qkv_split_kernel, dim3(blocks), dim3(256), 0, st, (const bf16_t*)qkv, (bf16_t*)q, (bf16_t*)kc,
                     (bf16_t*)vc, B, T, H, Hkv, hd, S, pos, cos, sin, rope, kv8);
  return (int)hipGetLastError();
}

template <int HD, bool QKV, bool KV8>
static void launch_flash(dim3 grid, hipStream_t st, const bf16_t* q, const bf16_t* kc, const bf16_t* vc, bf16_t* o,
                         int T, int H, int Hkv, int S, const int* pos, float sl2, int ldq, bf16_t* kco, bf16_t* vco) {
  // double-buffered K/V LDS, one barrier per block (default): GPT-2 B=64 T=512 0.1075 -> 0.1063 ms,
  // hd 128 T=512 0.251 -> 0.243, T=4096 1.123 -> 1.092 (profiles/r3_flash_double_buffer.jsonl);
  // DNN_FLASH_DB=0 keeps the single buffer (A/B)
  const char* e = getenv("DNN_FLASH_DB");
  if constexpr (HD == 64) {  // hd 128: three buffers would leave one workgroup per CU
    const char* ep = getenv("DNN_FLASH_PIPE");
    if ((e == nullptr || atoi(e) != 0) && ep != nullptr && atoi(ep) != 0) {
      hipLaunchKernelGGL((flash_attn_kernel<HD, QKV, KV8, true, true>), grid, dim3(256), 0, st, q, kc, vc, o, T, H,
                         Hkv, S, pos, sl2, ldq, kco, vco);
      return;
    }
  }
  if (e == nullptr || atoi(e) != 0)
    hipLaunchKernelGGL((flash_attn_kernel<HD, QKV, KV8, true>), grid, dim3(256), 0, st, q, kc, vc, o, T, H, Hkv, S,
                       pos, sl2, ldq, kco, vco);
  else
    hipLaunchKernelGGL((flash_attn_kernel<HD, QKV, KV8, false>), grid, dim3(256), 0, st, q, kc, vc, o, T, H, Hkv, S,
                       pos, sl2, ldq, kco, vco);
}

extern "C" int dnn_flash_attn(const void* q, const void* kc, const void* vc, void* o, int B, int T, int H, int Hkv,
                              int hd, int S, const int* pos, float scale, hipStream_t st, int kv8) {
  if (H % Hkv != 0) return -1;
  dim3 grid(H, B, (T + FA_QB - 1) / FA_QB);
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_t *q_ = (const bf16_t*)q, *k_ = (const bf16_t*)kc, *v_ = (const bf16_t*)vc;
  bf16_t* o_ = (bf16_t*)o;
  if (kv8) {  // e4m3 cache: every key / value row widened as it is fetched
    if (hd == 64)
      launch_flash<64, false, true>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, 0, nullptr, nullptr);
    else if (hd == 128)
      launch_flash<128, false, true>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, 0, nullptr, nullptr);
    else
      return -2;
  } else if (hd == 64) {
    launch_flash<64, false, false>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, 0, nullptr, nullptr);
  } else if (hd == 128) {
    launch_flash<128, false, false>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, 0, nullptr, nullptr);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

// Prefill straight from the c_attn output (no RoPE): see flash_attn_kernel<HD, true>.
extern "C" int dnn_flash_attn_qkv(const void* qkv, int ldqkv, void* kc, void* vc, void* o, int B, int T, int H,
                                  int Hkv, int hd, int S, const int* pos, float scale, hipStream_t st, int kv8) {
  if (H % Hkv != 0 || ldqkv < (H + 2 * Hkv) * hd || (ldqkv % 8) != 0) return -1;
  dim3 grid(H, B, (T + FA_QB - 1) / FA_QB);
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_t *q_ = (const bf16_t*)qkv, *k_ = (const bf16_t*)kc, *v_ = (const bf16_t*)vc;
  bf16_t *o_ = (bf16_t*)o, *ko = (bf16_t*)kc, *vo = (bf16_t*)vc;
  if (kv8) {  // e4m3 cache (unit scale)
    if (hd == 64)
      launch_flash<64, true, true>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, ldqkv, ko, vo);
    else if (hd == 128)
      launch_flash<128, true, true>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, ldqkv, ko, vo);
    else
      return -2;
  } else if (hd == 64) {
    launch_flash<64, true, false>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, ldqkv, ko, vo);
  } else if (hd == 128) {
    launch_flash<128, true, false>(grid, st, q_, k_, v_, o_, T, H, Hkv, S, pos, sl2, ldqkv, ko, vo);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

// the split merge: the one-round-trip kernel for up to 8 splits (head dim <= 256)
static void launch_decode_combine(const float* ws, bf16_t* o, int B, int H, int Hkv, int hd, int ns, hipStream_t st) {
  if (ns <= 8 && hd <= 256) {
    const int th = hd <= 64 ? 64 : (hd <= 128 ? 128 : 256);
    if (ns <= 2)
      hipLaunchKernelGGL(decode_combine_fast_kernel<2>, dim3(B * H), dim3(th), 0, st, ws, o, B, H, Hkv, hd, ns);
    else if (ns <= 4)
      hipLaunchKernelGGL(decode_combine_fast_kernel<4>, dim3(B * H), dim3(th), 0, st, ws, o, B, H, Hkv, hd, ns);
    else
      hipLaunchKernelGGL(decode_combine_fast_kernel<8>, dim3(B * H), dim3(th), 0, st, ws, o, B, H, Hkv, hd, ns);
    return;
  }
  hipLaunchKernelGGL(decode_combine_kernel, dim3(B * H), dim3(128), 0, st, ws, o, B, H, Hkv, hd, ns);
}

struct Dec1pArgs {
  const bf16_t* q;
  int ldq;
  bf16_t *kc, *vc;
  float* ws;
  int H, Hkv, S;
  const int* lens;
  const float *cosT, *sinT;
  float sl2;
  bf16_t* o;
  bool kf;  // K/V loads issued before q (attn_decode_1p_kernel KF)
};
template <int HD, int G, int NW, int KT, int VE, int VU, bool RS, int FM, bool NT, bool KNT>
static void launch_1p_k(const Dec1pArgs& a, dim3 grid, hipStream_t st) {
  const size_t smem = sizeof(float) * (size_t)NW * G * (HD + 1);  // [NW][G][HD] + [NW][G] (step 6)
  if (a.kf)
    hipLaunchKernelGGL((attn_decode_1p_kernel<HD, G, FM, NT, NW, KT, VE, VU, RS, KNT, true>), grid, dim3(NW * 64),
                       smem, st, a.q, a.ldq, a.kc, a.vc, a.ws, a.H, a.Hkv, a.S, a.lens, a.cosT, a.sinT, a.sl2, a.o);
  else
    hipLaunchKernelGGL((attn_decode_1p_kernel<HD, G, FM, NT, NW, KT, VE, VU, RS, KNT, false>), grid, dim3(NW * 64),
                       smem, st, a.q, a.ldq, a.kc, a.vc, a.ws, a.H, a.Hkv, a.S, a.lens, a.cosT, a.sinT, a.sl2, a.o);
}
template <int HD, int G, int NW, int KT, int VE, int VU, bool RS, int FM>
static void launch_1p_f(const Dec1pArgs& a, bool nt, bool knt, dim3 grid, hipStream_t st) {
  if (!nt)
    launch_1p_k<HD, G, NW, KT, VE, VU, RS, FM, false, false>(a, grid, st);
  else if (knt)
    launch_1p_k<HD, G, NW, KT, VE, VU, RS, FM, true, true>(a, grid, st);
  else
    launch_1p_k<HD, G, NW, KT, VE, VU, RS, FM, true, false>(a, grid, st);
}
template <int HD, int G, int NW, int KT, int VE, int VU, bool RS>
static void launch_1p(const Dec1pArgs& a, int fm, bool nt, bool knt, dim3 grid, hipStream_t st) {
  if (fm == 2)
    launch_1p_f<HD, G, NW, KT, VE, VU, RS, 2>(a, nt, knt, grid, st);
  else if (fm == 1)
    launch_1p_f<HD, G, NW, KT, VE, VU, RS, 1>(a, nt, knt, grid, st);
  else
    launch_1p_f<HD, G, NW, KT, VE, VU, RS, 0>(a, nt, knt, grid, st);
}

// One-pass decode attention (bf16 cache): returns 1 when the shape is not
// covered (the caller falls back to the batched kernel).  Splits of at most
// DEC1P_CAP keys; more than one split only when the caller's workspace holds
// them; grids below 128 workgroups keep the split-K kernel (its splits fill
// the chip at batch 1).
constexpr int DEC1P_CAP = 640;
static int attn_decode_1p_launch(const void* q, int ldq, void* kc, void* vc, void* o, int B, int H, int Hkv, int hd,
                                 int S, const int* lens, const float* cosT, const float* sinT, float sl2, int splits,
                                 float* ws, int fm, bool nt, bool force, hipStream_t st) {
  const int G = H / Hkv;
  int ns = (S + DEC1P_CAP - 1) / DEC1P_CAP;
  // DNN_DECODE_1P_NS=n: at least n key splits (A/B; needs the caller's workspace)
  const char* ns_e = getenv("DNN_DECODE_1P_NS");
  const int ns_min = ns_e != nullptr ? atoi(ns_e) : 0;
  if (ns_min > ns) ns = ns_min;
  if (ns > 1 && ns > splits) return 1;
  if (!force && (long)B * Hkv * ns < 128) return 1;
  // GQA past one workgroup per CU: the 86 KiB of LDS per workgroup keeps one
  // resident per CU, so a second round of workgroups runs serially and the
  // batched kernel wins (Llama-3 B=64: 36.5 vs 30.9 us,
  // profiles/r3_attn_1p_shapes.jsonl); MHA's 4-wave workgroups are small
  if (!force && ns_min <= 1 && G > 1 && (long)B * Hkv * ns > 256) return 1;
  dim3 grid(B * Hkv, ns);
  // row-layout scores for MHA, MFMA key tiles for GQA: at MHA hd 64 an MFMA tile
  // uses 1 of 16 head columns and its half-row key loads ran 10 % slower than
  // whole rows (GPT-2 B=64 22.0 vs 19.9 us, profiles/r3_attn_1p_probe.jsonl)
  const char* rs_e = getenv("DNN_DECODE_1P_RS");    // A/B override: 0 MFMA tiles, 1 row layout
  const char* kn_e = getenv("DNN_DECODE_1P_KNT");   // key loads non-temporal (A/B; default: as the values)
  const bool rs = rs_e != nullptr ? atoi(rs_e) == 1 : G == 1;
  // key loads: non-temporal for MHA, default policy for GQA (Llama-3 B=32
  // 19.54 -> 19.11 us; GPT-2 B=64 19.28 -> 20.01 the other way)
  const bool knt = nt && (kn_e != nullptr ? atoi(kn_e) != 0 : G == 1);
  // K/V loads before q for GQA (Llama-3 B=32 19.40 -> 19.12 us, decode 3.930 -> 3.902 ms/step), after q for
  // MHA (GPT-2 B=64 19.50 -> 19.91 us the other way; profiles/r3_attn_1p_probe_v3.jsonl)
  const char* kf_e = getenv("DNN_DECODE_1P_KF");    // A/B override: 1 before q, 0 after
  const bool kf = kf_e != nullptr ? atoi(kf_e) == 1 : G > 1;
  Dec1pArgs a{(const bf16_t*)q, ldq, (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, cosT, sinT, sl2, (bf16_t*)o, kf};
  // hd 128 GQA (Llama-3 G = 4, llama3-tiny G = 2): 8 waves x 5 key tiles; hd 64 MHA (GPT-2): 4 waves x 10
  // (row-layout scores for GQA measured 22.3 vs 19.0 us at Llama-3 B=32: not built)
  if (hd == 128 && G == 4)
    launch_1p<128, 4, 8, 5, 8, 20, false>(a, fm, nt, knt, grid, st);
  else if (hd == 128 && G == 2)
    launch_1p<128, 2, 8, 5, 8, 20, false>(a, fm, nt, knt, grid, st);
  else if (hd == 64 && G == 1 && rs)
    launch_1p<64, 1, 4, 10, 2, 20, true>(a, fm, nt, knt, grid, st);
  else if (hd == 64 && G == 1)
    launch_1p<64, 1, 4, 10, 6, 20, false>(a, fm, nt, knt, grid, st);
  else
    return 1;
  if (ns > 1)
    launch_decode_combine(ws, (bf16_t*)o, B, H, Hkv, hd, ns, st);
  return (int)hipGetLastError();
}

static int attn_decode_launch(const void* q, int ldq, void* kc, void* vc, void* o, int B, int H, int Hkv, int hd,
                              int S, const int* lens, const float* cosT, const float* sinT, float scale, int splits,
                              float* ws, bool fused, hipStream_t st, bool kv8 = false) {
  const int G = H / Hkv;
  if (H % Hkv != 0 || G > DEC_MAXG || splits <= 0) return -1;
  if (!kv8) {
    // DNN_DECODE_1P=0 keeps the batched kernel everywhere (A/B), =2 takes the
    // one-pass kernel on small grids too (tests)
    const char* e1 = getenv("DNN_DECODE_1P");
    const int m1 = e1 != nullptr ? atoi(e1) : 1;
    if (m1 != 0) {
      const bool nt1 = (double)B * Hkv * S * hd * 4.0 > 32.0 * 1024 * 1024;
      const int r = attn_decode_1p_launch(q, ldq, kc, vc, o, B, H, Hkv, hd, S, lens, cosT, sinT,
                                          scale * 1.4426950408889634f, splits, ws,
                                          fused ? (cosT != nullptr ? 2 : 1) : 0, nt1, m1 == 2, st);
      if (r != 1) return r;
    }
  }
  if (kv8 && G != 1 && hd != 128) return -4;  // e4m3 cache: MHA, or GQA at hd 128 (Llama-3)
  const int chunk_cap = (S + splits - 1) / splits;
  const int gpb = 256 / (hd / (kv8 ? 16 : 8));
  size_t smem = sizeof(float) * (size_t)G * (size_t)(chunk_cap > gpb * hd ? chunk_cap : gpb * hd);
  if (smem > 160 * 1024) return -3;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(B * Hkv, splits);
  // cache bytes this launch may stream (capacity bound): > 32 MB -> non-temporal
  const bool nt = (double)B * Hkv * S * hd * (kv8 ? 2.0 : 4.0) > 32.0 * 1024 * 1024;
  // MFMA scores: GQA (G >= 2) by default; DNN_DECODE_MFMA=0/1 forces it off/on (A/B)
  const char* mf_e = getenv("DNN_DECODE_MFMA");
  const bool mf = mf_e ? atoi(mf_e) == 1 : G >= 2;
  const int fm = fused ? (cosT != nullptr ? 2 : 1) : 0;
  if (kv8) {
    // DNN_KV8_U=8: 8 rows in flight per thread instead of 10 (A/B)
    const char* u_e = getenv("DNN_KV8_U");
    const bool u8 = u_e != nullptr && atoi(u_e) == 8;
#define DEC8(HDV, NTV, FMV)                                                                                          \
  if (hd == HDV && nt == NTV && fm == FMV) {                                                                          \
    if (u8)                                                                                                           \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, 1, FMV, NTV, false, true, 8>), grid, dim3(256), smem, st,           \
                         (const bf16_t*)q, ldq, (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, nullptr, nullptr, sl2,  \
                         chunk_cap, (bf16_t*)o);                                                                      \
    else                                                                                                              \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, 1, FMV, NTV, false, true, 10>), grid, dim3(256), smem, st,          \
                         (const bf16_t*)q, ldq, (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, nullptr, nullptr, sl2,  \
                         chunk_cap, (bf16_t*)o);                                                                      \
  } else
    if (G > 1) {  // GQA: MFMA key tiles (hd 128: Llama-3 G = 4, llama3-tiny G = 2)
#define DEC8G(GV, NTV, FMV)                                                                                           \
  if (G == GV && nt == NTV && fm == FMV)                                                                              \
    hipLaunchKernelGGL((attn_decode_kernel<128, GV, FMV, NTV, true, true>), grid, dim3(256), smem, st,                \
                       (const bf16_t*)q, ldq, (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, cosT, sinT, sl2,         \
                       chunk_cap, (bf16_t*)o);                                                                        \
  else
      DEC8G(4, true, 2) DEC8G(4, false, 2) DEC8G(4, true, 1) DEC8G(4, false, 1) DEC8G(4, true, 0) DEC8G(4, false, 0)
      DEC8G(2, true, 2) DEC8G(2, false, 2) DEC8G(2, true, 1) DEC8G(2, false, 1) DEC8G(2, true, 0) DEC8G(2, false, 0)
      { return -2; }
#undef DEC8G
    } else
    DEC8(64, true, 1) DEC8(64, false, 1) DEC8(128, true, 1) DEC8(128, false, 1) DEC8(64, true, 0) DEC8(64, false, 0)
    DEC8(128, true, 0) DEC8(128, false, 0) { return -2; }
#undef DEC8
    if (splits > 1)
      launch_decode_combine(ws, (bf16_t*)o, B, H, Hkv, hd, splits, st);
    return (int)hipGetLastError();
  }
#define DEC_FM(HDV, GV, NTV, MFV)                                                                                     \
  if (fm == 2)                                                                                                        \
    hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 2, NTV, MFV>), grid, dim3(256), smem, st, (const bf16_t*)q, ldq,  \
                       (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, cosT, sinT, sl2, chunk_cap, (bf16_t*)o);        \
  else if (fm == 1)                                                                                                   \
    hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 1, NTV, MFV>), grid, dim3(256), smem, st, (const bf16_t*)q, ldq,  \
                       (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, nullptr, nullptr, sl2, chunk_cap, (bf16_t*)o);  \
  else                                                                                                                \
    hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 0, NTV, MFV>), grid, dim3(256), smem, st, (const bf16_t*)q, ldq,  \
                       (bf16_t*)kc, (bf16_t*)vc, ws, H, Hkv, S, lens, nullptr, nullptr, sl2, chunk_cap, (bf16_t*)o);
#define DEC_NT(HDV, GV, NTV)                                                                                          \
  if (mf) {                                                                                                           \
    DEC_FM(HDV, GV, NTV, true)                                                                                        \
  } else {                                                                                                            \
    DEC_FM(HDV, GV, NTV, false)                                                                                       \
  }
#define DEC(HDV, GV)                                                                                                  \
  if (hd == HDV && G == GV) {                                                                                         \
    if (nt) {                                                                                                         \
      DEC_NT(HDV, GV, true)                                                                                           \
    } else {                                                                                                          \
      DEC_NT(HDV, GV, false)                                                                                          \
    }                                                                                                                 \
  } else
  DEC(64, 1) DEC(64, 2) DEC(64, 4) DEC(64, 8) DEC(128, 1) DEC(128, 2) DEC(128, 4) DEC(128, 8) { return -2; }
#undef DEC
#undef DEC_NT
#undef DEC_FM
  if (splits > 1)
    launch_decode_combine(ws, (bf16_t*)o, B, H, Hkv, hd, splits, st);
  return (int)hipGetLastError();
}

#ifdef DNN_DEC_PROBE
extern "C" int dnn_dec_probe_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dec_probe_ts), sizeof(unsigned long long) * 32);
}
#endif

extern "C" int dnn_attn_decode(const void* q, const void* kc, const void* vc, void* o, int B, int H, int Hkv, int hd,
                               int S, const int* lens, float scale, int splits, float* ws, hipStream_t st, int kv8) {
  return attn_decode_launch(q, H * hd, const_cast<void*>(kc), const_cast<void*>(vc), o, B, H, Hkv, hd, S, lens,
                            nullptr, nullptr, scale, splits, ws, false, st, kv8 != 0);
}

// Decode step straight from the QKV projection: qkv rows (B, ldqkv) laid out
// [q H*hd | k Hkv*hd | v Hkv*hd]; pos[b] = tokens already cached.  RoPE when
// cos/sin are given.  Writes the new k/v into the cache and the attention
// output (B, H*hd).
extern "C" int dnn_attn_decode_qkv(const void* qkv, int ldqkv, void* kc, void* vc, void* o, int B, int H, int Hkv,
                                   int hd, int S, const int* pos, const float* cosT, const float* sinT, float scale,
                                   int splits, float* ws, hipStream_t st, int kv8) {
  if (ldqkv < (H + 2 * Hkv) * hd || (ldqkv % 8) != 0) return -1;
  return attn_decode_launch(qkv, ldqkv, kc, vc, o, B, H, Hkv, hd, S, pos, cosT, sinT, scale, splits, ws, true, st,
                            kv8 != 0);
}
