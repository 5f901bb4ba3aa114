// LayerNorm / RMSNorm and the GPT-2 token+position embedding (gfx950).
//
// LayerNorm with bias replaces nanoGPT's ln_1 / ln_2 / ln_f
// (partitions/gpt_model_parts.py:41,48 and the Block internals); RMSNorm serves
// Llama-3. One wave per row, 16-byte vector loads (guide G13), the row cached
// in registers between the statistics pass and the normalise pass, fp32 math,
// bf16 out. The embedding kernel fuses wte gather + wpe add
// (gpt_model_parts.py:16-19) and reads per-sequence start positions from device
// memory so one HIP graph serves every decode step.
#include "common.h"

#include <cstdlib>

namespace dnn {

template <int NC, bool RMS>
__global__ __launch_bounds__(256) void norm_kernel(const bf16_t* __restrict__ x, int ldx, const float* __restrict__ w,
                                                   const float* __restrict__ b, bf16_t* __restrict__ y, int ldy, int M,
                                                   int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (size_t)row * ldx;
  float v[NC][8];
  float s = 0.f;
  // gamma/beta are issued together with the row (one memory round trip before
  // the reductions instead of a dependent second one after them)
  constexpr bool PF = NC <= 8;
  f32x4 wpf[PF ? NC : 1][2], bpf[PF ? NC : 1][2];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < N) {
      const bf16x8 p = *reinterpret_cast<const bf16x8*>(xr + c);
      if constexpr (PF) {
        wpf[i][0] = *reinterpret_cast<const f32x4*>(w + c);
        wpf[i][1] = *reinterpret_cast<const f32x4*>(w + c + 4);
        if (!RMS && b != nullptr) {
          bpf[i][0] = *reinterpret_cast<const f32x4*>(b + c);
          bpf[i][1] = *reinterpret_cast<const f32x4*>(b + c + 4);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[i][j] = bf2f_s(p[j]); s += v[i][j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < N) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / N + eps);
  bf16_t* yr = y + (size_t)row * ldy;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < N) {
      f32x4 w0, w1, b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
      if constexpr (PF) {
        w0 = wpf[i][0];
        w1 = wpf[i][1];
        if (!RMS && b != nullptr) { b0 = bpf[i][0]; b1 = bpf[i][1]; }
      } else {
        w0 = *reinterpret_cast<const f32x4*>(w + c);
        w1 = *reinterpret_cast<const f32x4*>(w + c + 4);
        if (!RMS && b != nullptr) {
          b0 = *reinterpret_cast<const f32x4*>(b + c);
          b1 = *reinterpret_cast<const f32x4*>(b + c + 4);
        }
      }
      const float ww[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
      const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      uint4 o;
      uint32_t* op = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a0 = (v[i][2 * j] - mean) * rstd * ww[2 * j] + bb[2 * j];
        const float a1 = (v[i][2 * j + 1] - mean) * rstd * ww[2 * j + 1] + bb[2 * j + 1];
        op[j] = pack2bf(a0, a1);
      }
      *reinterpret_cast<uint4*>(yr + c) = o;
    }
  }
}

// Row statistics only (prefill LayerNorm / RMSNorm folded into the next GEMM,
// ops/gemm.py linear_norm): one wave per row, the row in registers, two-pass
// mean / variance (no E[x^2] - mean^2 cancellation); writes {rstd, -mean rstd}
// per row (RMS: {rstd, 0}).  Reads the activation once and writes 8 B per row
// instead of the normalised copy the norm kernel writes and the GEMM re-reads.
//
// R rows per wave (prefill, M in the tens of thousands): all R rows' loads are
// issued before the first reduction, so a wave pays one load round trip for R
// rows and the grid is R times smaller — one row per wave left 32768 waves in
// four residency rounds of a latency-bound load + two wave sums each.
template <int NC, bool RMS, int R = 1>
__global__ __launch_bounds__(256) void row_stats_kernel(const bf16_t* __restrict__ x, int ldx, float2* __restrict__ st,
                                                        int M, int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  bf16x8 raw[R][NC];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bf16_t* xr = x + (size_t)min(row0 + r, M - 1) * ldx;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      raw[r][i] = c < N ? *reinterpret_cast<const bf16x8*>(xr + c) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += bf2f_s(raw[r][i][j]);
    const float mean = RMS ? 0.f : wave_sum(s) / N;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      if (c < N) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = bf2f_s(raw[r][i][j]) - mean; q += d * d; }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / N + eps);
    if (lane == 0 && row0 + r < M) st[row0 + r] = make_float2(rstd, -mean * rstd);
  }
}

// Normalise + quantise in one pass (fp8 prefill): the normalised row (fp32,
// still in registers) is scaled by its own amax/448 and written as OCP e4m3
// with the K padding zeroed, plus the per-row scale — the layout
// quant_fp8_rows produces — so the activation never round-trips through bf16.
// R rows per wave (DNN_NORMQ8_R; default 1 — with gamma / beta loaded once
// per wave next to the rows, more rows per wave only lowered occupancy).
// MX: one e8m0 scale per (row, 128-column block) instead of the row scale
// (common.h mx_index; the 16 lanes of a block agree on it by 4 shuffles).
template <int NC, bool RMS, bool SPLIT = false, int R = 1, bool MX = false>
__global__ __launch_bounds__(256) void norm_q8_kernel(const bf16_t* __restrict__ x, int ldx, const float* __restrict__ w,
                                                      const float* __restrict__ b, uint8_t* __restrict__ q, int ldq,
                                                      float* __restrict__ sq, int M, int N, int kpad, float eps,
                                                      uint8_t* __restrict__ sx = nullptr) {
  static_assert(!(MX && SPLIT), "MX scales with one e4m3 byte per activation");
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  bf16x8 raw[R][NC];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bf16_t* xr = x + (size_t)min(row0 + r, M - 1) * ldx;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      raw[r][i] = c < N ? *reinterpret_cast<const bf16x8*>(xr + c) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // gamma / beta as 16-B vectors issued with the rows and shared by the R rows
  // (per-element loads after the reductions were one dependent round trip per
  // row and column chunk: 103 us per GPT-2 XL prefill pass against 28 us for the
  // plain MX quantiser, profiles/r5_gpt2xl_fp8_b64_kernels_mx.md)
  f32x4 wpf[NC][2], bpf[NC][2];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = (lane + 64 * i) * 8;
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    wpf[i][0] = wpf[i][1] = bpf[i][0] = bpf[i][1] = z;
    if (c < N) {
      wpf[i][0] = *reinterpret_cast<const f32x4*>(w + c);
      wpf[i][1] = *reinterpret_cast<const f32x4*>(w + c + 4);
      if (!RMS && b != nullptr) {
        bpf[i][0] = *reinterpret_cast<const f32x4*>(b + c);
        bpf[i][1] = *reinterpret_cast<const f32x4*>(b + c + 4);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = row0 + r;
    float v[NC][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f_s(raw[r][i][j]);
        s += v[i][j];
      }
    float mean = 0.f;
    if (!RMS) mean = wave_sum(s) / N;
    float qs = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      if (c < N) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; qs += d * d; }
      }
    }
    const float rstd = rsqrtf(wave_sum(qs) / N + eps);
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      if (c < N) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[i][j] = (v[i][j] - mean) * rstd * wpf[i][j >> 2][j & 3] + bpf[i][j >> 2][j & 3];
          amax = fmaxf(amax, fabsf(v[i][j]));
        }
      }
    }
    if constexpr (MX) {
      if (row >= M) continue;  // wave-uniform
      uint8_t* qr = q + (size_t)row * ldq;
      const int mpad = mx_mpad(M);
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const int c = (lane + 64 * i) * 8;
        float am = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) am = c < N ? fmaxf(am, fabsf(v[i][j])) : am;
        am = group_max<16>(am);  // the 128-column block of lanes 16g..16g+15
        float inv;
        const uint32_t e = e8m0_of(am, inv);
        if (c < kpad) {
          int lo = 0, hi = 0;
          if (c < N) {
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, lo, false);
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, hi, false);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
          }
          *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
          if ((lane & 15) == 0) sx[mx_index(row, c >> 7, mpad)] = (uint8_t)e;
        }
      }
      continue;
    }
    amax = wave_max(amax);
    if (row >= M) continue;  // wave-uniform (after the reductions)
    const float sc = amax > 0.f ? amax / 448.f : 1.f;
    const float inv = 1.f / sc;
    if (lane == 0) sq[row] = sc;
    uint8_t* qr = q + (size_t)row * ldq;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (lane + 64 * i) * 8;
      if (c < kpad) {
        if constexpr (SPLIT) {  // hi plane + residual plane at +kpad (quant_fp8_rows' split layout)
          float y[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = c < N ? v[i][j] * inv : 0.f;
          int h0, h1, l0, l1;
          q8_split8(y, h0, h1, l0, l1);
          *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)h0, (uint32_t)h1);
          *reinterpret_cast<uint2*>(qr + kpad + c) = make_uint2((uint32_t)l0, (uint32_t)l1);
          continue;
        }
        int lo = 0, hi = 0;
        if (c < N) {
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, lo, false);
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, hi, false);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
        }
        *reinterpret_cast<uint2*>(qr + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
      }
    }
  }
}

// out[r, :] = wte[idx[r], :] (+ wpe[pos[b] + t, :]) with r = b*T + t.
__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                    const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out, int B,
                                                    int T, int d, const int* __restrict__ pos, int V, int P) {
  const int chunks = d / 8;
  const long total = (long)B * T * chunks;
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < total; g += (long)gridDim.x * blockDim.x) {
    const int c = (int)(g % chunks);
    const long r = g / chunks;
    const int b = (int)(r / T), t = (int)(r % T);
    // ids and positions clamped to the tables: a bad id or a position past
    // block_size reads a valid row (wrong but bounded) instead of faulting;
    // the host rejects such runs at config load (cli.check_config_capacity)
    const int tok = min(max(idx[r], 0), V - 1);
    const bf16x8 e = *reinterpret_cast<const bf16x8*>(wte + (size_t)tok * d + c * 8);
    uint4 o;
    if (wpe != nullptr) {
      const int p = min((pos != nullptr ? pos[b] : 0) + t, P - 1);
      const bf16x8 q = *reinterpret_cast<const bf16x8*>(wpe + (size_t)p * d + c * 8);
      uint32_t* op = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        op[j] = pack2bf(bf2f_s(e[2 * j]) + bf2f_s(q[2 * j]), bf2f_s(e[2 * j + 1]) + bf2f_s(q[2 * j + 1]));
    } else {
      o = *reinterpret_cast<const uint4*>(&e);
    }
    *reinterpret_cast<uint4*>(out + r * d + c * 8) = o;
  }
}

}  // namespace dnn

using namespace dnn;

extern "C" int dnn_layernorm(const void* x, int ldx, const float* w, const float* b, void* y, int ldy, int M, int N,
                             float eps, int rms, hipStream_t st) {
  if (N % 8 != 0 || N > 8192) return -1;
  const int nc = (N / 8 + 63) / 64;
  dim3 grid((M + 3) / 4), blk(256);
#define L(NCV)                                                                                                      \
  if (nc <= NCV) {                                                                                                  \
    if (rms) hipLaunchKernelGGL((norm_kernel<NCV, true>), grid, blk, 0, st, (const bf16_t*)x, ldx, w, b, (bf16_t*)y, \
                                ldy, M, N, eps);                                                                    \
    else hipLaunchKernelGGL((norm_kernel<NCV, false>), grid, blk, 0, st, (const bf16_t*)x, ldx, w, b, (bf16_t*)y,   \
                            ldy, M, N, eps);                                                                        \
    return (int)hipGetLastError();                                                                                  \
  }
  L(1) L(2) L(4) L(8) L(16)
#undef L
  return -1;
}

extern "C" int dnn_row_stats(const void* x, int ldx, float* stats, int M, int N, float eps, int rms, hipStream_t st) {
  if (N % 8 != 0 || N > 8192 || M <= 0) return M <= 0 ? 0 : -1;
  const int nc = (N / 8 + 63) / 64;
  // 4 rows per wave once the grid would exceed one residency round (8192 waves);
  // DNN_ROWSTATS_R=1 forces one row per wave (A/B)
  const char* re = getenv("DNN_ROWSTATS_R");
  const int R = re != nullptr ? atoi(re) : (M >= 8192 && nc <= 4 ? 4 : 1);
  dim3 blk(256);
#define L(NCV)                                                                                                       \
  if (nc <= NCV) {                                                                                                   \
    if (R == 4 && NCV <= 4) {                                                                                        \
      dim3 grid((M + 15) / 16);                                                                                      \
      if (rms) hipLaunchKernelGGL((row_stats_kernel<NCV, true, 4>), grid, blk, 0, st, (const bf16_t*)x, ldx,        \
                                  reinterpret_cast<float2*>(stats), M, N, eps);                                      \
      else hipLaunchKernelGGL((row_stats_kernel<NCV, false, 4>), grid, blk, 0, st, (const bf16_t*)x, ldx,           \
                              reinterpret_cast<float2*>(stats), M, N, eps);                                          \
    } else {                                                                                                         \
      dim3 grid((M + 3) / 4);                                                                                        \
      if (rms) hipLaunchKernelGGL((row_stats_kernel<NCV, true>), grid, blk, 0, st, (const bf16_t*)x, ldx,           \
                                  reinterpret_cast<float2*>(stats), M, N, eps);                                      \
      else hipLaunchKernelGGL((row_stats_kernel<NCV, false>), grid, blk, 0, st, (const bf16_t*)x, ldx,              \
                              reinterpret_cast<float2*>(stats), M, N, eps);                                          \
    }                                                                                                                \
    return (int)hipGetLastError();                                                                                   \
  }
  L(1) L(2) L(4) L(8) L(16)
#undef L
  return -1;
}

extern "C" int dnn_embed_gpt2(const int* idx, const void* wte, const void* wpe, void* out, int B, int T, int d,
                              const int* pos, int V, int P, hipStream_t st) {
  if (d % 8 != 0 || V <= 0 || (wpe != nullptr && P <= 0)) return -1;
  const long total = (long)B * T * (d / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(embed_kernel, dim3(blocks), dim3(256), 0, st, idx, (const bf16_t*)wte, (const bf16_t*)wpe,
                     (bf16_t*)out, B, T, d, pos, V, P);
  return (int)hipGetLastError();
}

// Normalise (w, b; LayerNorm or RMSNorm) and quantise rows to e4m3 with per-row
// scales: q [M][ldq bytes] (columns N..kpad-1 zeroed), sq [M].
// Normalise + MX-quantise (e8m0 per (row, 128-column block), common.h
// mx_index): sx holds mx_mpad(M) * kpad / 128 bytes.
extern "C" int dnn_layernorm_q8_mx(const void* x, int ldx, const float* w, const float* b, void* q, int ldq, void* sx,
                                   int M, int N, int kpad, float eps, int rms, hipStream_t st) {
  if (N % 8 != 0 || N > 8192 || kpad < N || kpad % 128 != 0 || ldq < kpad || (ldq & 7) != 0 || sx == nullptr)
    return -1;
  if (M <= 0) return 0;
  const int nc = (kpad / 8 + 63) / 64;
  // one row per wave: with gamma / beta issued with the rows, GPT-2 XL's
  // 32768 x 1600 pass takes 38.5 us at R = 1, 45.7 at 2, 52.9 at 4
  // (profiles/r5_norm_q8_probe.jsonl); DNN_NORMQ8_R=2/4 for A/B
  const char* re = getenv("DNN_NORMQ8_R");
  const int R = re != nullptr ? atoi(re) : 1;
  dim3 blk(256);
#define LQM(NCV, RV)                                                                                              \
  {                                                                                                               \
    dim3 grid((M + 4 * RV - 1) / (4 * RV));                                                                       \
    if (rms) hipLaunchKernelGGL((norm_q8_kernel<NCV, true, false, RV, true>), grid, blk, 0, st, (const bf16_t*)x, \
                                ldx, w, b, (uint8_t*)q, ldq, (float*)nullptr, M, N, kpad, eps, (uint8_t*)sx);    \
    else hipLaunchKernelGGL((norm_q8_kernel<NCV, false, false, RV, true>), grid, blk, 0, st, (const bf16_t*)x,    \
                            ldx, w, b, (uint8_t*)q, ldq, (float*)nullptr, M, N, kpad, eps, (uint8_t*)sx);        \
    return (int)hipGetLastError();                                                                                \
  }
#define LQ(NCV)                         \
  if (nc <= NCV) {                      \
    if (R == 4 && NCV <= 4) LQM(NCV, 4) \
    if (R == 2 && NCV <= 4) LQM(NCV, 2) \
    LQM(NCV, 1)                         \
  }
  LQ(1) LQ(2) LQ(4) LQ(8) LQ(16)
#undef LQ
#undef LQM
  return -1;
}

extern "C" int dnn_layernorm_q8(const void* x, int ldx, const float* w, const float* b, void* q, int ldq, float* sq,
                                int M, int N, int kpad, float eps, int rms, hipStream_t st, int split) {
  if (N % 8 != 0 || N > 8192 || kpad < N || kpad % 8 != 0 || ldq < kpad * (split ? 2 : 1) || sq == nullptr) return -1;
  if (M <= 0) return 0;
  const int nc = (kpad / 8 + 63) / 64;
  // one row per wave (as dnn_layernorm_q8_mx); DNN_NORMQ8_R=2/4 for A/B
  const char* re = getenv("DNN_NORMQ8_R");
  const int R = re != nullptr ? atoi(re) : 1;
  dim3 blk(256);
#define LQK(NCV, RV)                                                                                               \
  {                                                                                                                \
    dim3 grid((M + 4 * RV - 1) / (4 * RV));                                                                        \
    if (split) {                                                                                                   \
      if (rms) hipLaunchKernelGGL((norm_q8_kernel<NCV, true, true, RV>), grid, blk, 0, st, (const bf16_t*)x, ldx,  \
                                  w, b, (uint8_t*)q, ldq, sq, M, N, kpad, eps);                                    \
      else hipLaunchKernelGGL((norm_q8_kernel<NCV, false, true, RV>), grid, blk, 0, st, (const bf16_t*)x, ldx, w,  \
                              b, (uint8_t*)q, ldq, sq, M, N, kpad, eps);                                           \
    } else if (rms) {                                                                                              \
      hipLaunchKernelGGL((norm_q8_kernel<NCV, true, false, RV>), grid, blk, 0, st, (const bf16_t*)x, ldx, w, b,    \
                         (uint8_t*)q, ldq, sq, M, N, kpad, eps);                                                   \
    } else {                                                                                                       \
      hipLaunchKernelGGL((norm_q8_kernel<NCV, false, false, RV>), grid, blk, 0, st, (const bf16_t*)x, ldx, w, b,   \
                         (uint8_t*)q, ldq, sq, M, N, kpad, eps);                                                   \
    }                                                                                                              \
    return (int)hipGetLastError();                                                                                 \
  }
#define LQ(NCV)                      \
  if (nc <= NCV) {                   \
    if (R == 4 && NCV <= 4) LQK(NCV, 4) \
    if (R == 2 && NCV <= 4) LQK(NCV, 2) \
    LQK(NCV, 1)                      \
  }
  LQ(1) LQ(2) LQ(4) LQ(8) LQ(16)
#undef LQ
#undef LQK
  return -1;
}
