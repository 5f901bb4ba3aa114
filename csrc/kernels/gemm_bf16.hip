// bf16 GEMM on CDNA4 MFMA with fused epilogues.
//
//   C[M,N] = act(A[M,K] . W[N,K]^T + bias[N]) (+ residual[M,N])
//
// W is the nn.Linear layout [out, in], so both operands are K-contiguous and
// every MFMA fragment is one 16-byte LDS read. Replaces the implicit torch ops
// of the reference's stage forwards: CIFAR fc1 (cifar_model_parts.py:13,55),
// nanoGPT c_attn / c_proj / c_fc / lm_head (partitions/gpt_model_parts.py:20-21,
// 32-33,46-49) and the Llama projections.
//
// Structure (cdna_hip_programming.md §5, "minimum 2-phase"): 128x128x64 tiles,
// 4 waves in 2x2, each wave 64x64 = 4x4 mfma_f32_16x16x32_bf16 tiles; operands
// staged global->LDS with 16-byte global_load_lds into a double buffer whose
// 128-B rows are XOR-swizzled on the SOURCE address (chunk ^= (row>>1)&7), which
// makes the ds_read_b128 fragment reads conflict-free (rule 21 / T2).
// Block ids are remapped so tiles sharing A panels run on one XCD (T1).
//
// Small-M variant (decode, M <= 64): split-K 64xBN tiles reduce through fp32
// atomics into a workspace is avoided; instead gemm_skinny streams W straight to
// VGPRs (the 'GEMV / M <= 16' row of the guide) — see gemm_skinny below.
#include "common.h"

namespace dnn {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SILU_MUL = 3 };

constexpr int GB_M = 128, GB_N = 128, GB_K = 64;
constexpr int G_TILE_BYTES = GB_M * GB_K * 2;  // 16 KiB per operand tile

__device__ __forceinline__ int swz_chunk(int row) { return (row >> 1) & 7; }

// Stage one 128x64 bf16 tile (rows r0.., clamped to nrows-1) into LDS `dst`.
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ src, int ld, int r0, int nrows,
                                           int k0, char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;            // 1 KiB = 8 rows per wave-instruction
    const int rl = piece * 8 + (lane >> 3);    // row within the tile
    const int cp = lane & 7;                   // destination 16B chunk (linear)
    const int cs = cp ^ swz_chunk(rl);         // source chunk (inverse swizzle)
    int r = r0 + rl;
    r = r < nrows ? r : nrows - 1;
    const bf16_t* g = src + (size_t)r * ld + k0 + cs * 8;
    glds16(g, dst + piece * 1024);
  }
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(tile + row * 128 + ((chunk ^ swz_chunk(row)) << 4));
}

template <int ACT, bool OUT_F32>
__global__ __launch_bounds__(256, 2) void gemm_bf16_tn_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, int ldw, void* __restrict__ Cv,
    int ldc, const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[4 * G_TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + GB_N - 1) / GB_N, ntm = (M + GB_M - 1) / GB_M;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = tile / ntn, tn = tile % ntn;
  const int m0 = tm * GB_M, n0 = tn * GB_N;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GB_K;
  stage_tile(A, lda, m0, M, 0, smem, wave, lane);
  stage_tile(W, ldw, n0, N, 0, smem + G_TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    char* a_s = smem + cur * 2 * G_TILE_BYTES;
    char* b_s = a_s + G_TILE_BYTES;
    if (t + 1 < nk) {
      char* na = smem + (cur ^ 1) * 2 * G_TILE_BYTES;
      stage_tile(A, lda, m0, M, (t + 1) * GB_K, na, wave, lane);
      stage_tile(W, ldw, n0, N, (t + 1) * GB_K, na + G_TILE_BYTES, wave, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(a_s, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(b_s, wn * 64 + j * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // Epilogue: C/D map of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + r.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    if (ACT == ACT_SILU_MUL) continue;
    const float b = (bias != nullptr && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N) {
          float v = acc[i][j][r] + b;
          if (ACT == ACT_RELU) v = fmaxf(v, 0.f);
          if (ACT == ACT_GELU) v = gelu_erf(v);
          if (R != nullptr) v += bf2f(R[(size_t)m * ldr + n]);
          if (OUT_F32) reinterpret_cast<float*>(Cv)[(size_t)m * ldc + n] = v;
          else reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + n] = f2bf(v);
        }
      }
    }
  }
  if (ACT == ACT_SILU_MUL) {
    // Packed gate/up weights: within each 32-column group, columns 0..15 are
    // gate rows and 16..31 the matching up rows (ops/gemm.py pack_gate_up), so a
    // lane holds g (tile j even) and u (tile j+1) for the same output column.
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const int ncol = (n0 + wn * 64 + j * 16) / 2 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          if (m < M && ncol < N / 2) {
            const float v = silu(acc[i][j][r]) * acc[i][j + 1][r];
            if (OUT_F32) reinterpret_cast<float*>(Cv)[(size_t)m * ldc + ncol] = v;
            else reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + ncol] = f2bf(v);
          }
        }
    }
  }
}

// ---------------------------------------------------------------------------
// Skinny GEMM for decode-sized M (<= 16 rows): weight-streaming, one wave per
// 16 output columns, split over K across the 4 waves of a workgroup, W loaded
// straight to VGPRs (no LDS round trip: guide §5 table, GEMV row). A (tiny) is
// read through L1/L2. Uses mfma_f32_16x16x32_bf16 with M padded to 16.
// ---------------------------------------------------------------------------
template <int ACT, bool OUT_F32, int MT>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, int ldw, void* __restrict__ Cv,
    int ldc, const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr, int M, int N, int K) {
  // MT 16-row M tiles share every W fragment (M <= 16*MT rows).
  __shared__ __attribute__((aligned(16))) f32x4 red[4][MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int n = n0 + (lane & 15);
  const int nc = n < N ? n : N - 1;
  const int kq = (lane >> 4) * 8;
  f32x4 acc[MT];
  const bf16_t* ap[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int mrow = t * 16 + (lane & 15);
    ap[t] = A + (size_t)(mrow < M ? mrow : M - 1) * lda;
  }
  // K split into 4 contiguous quarters (one per wave), each a multiple of 32
  const int kper = ((K / 32 + 3) / 4) * 32;
  const int kbeg = wave * kper;
  const int kend = min(K, kbeg + kper);
  const bf16_t* wp = W + (size_t)nc * ldw;
  int k = kbeg;
  for (; k + 128 <= kend; k += 128) {
    bf16x8 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const bf16x8*>(wp + k + u * 32 + kq);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      bf16x8 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const bf16x8*>(ap[t] + k + u * 32 + kq);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[u], acc[t], 0, 0, 0);
    }
  }
  for (; k < kend; k += 32) {
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(wp + k + kq);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(ap[t] + k + kq);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  // reduction + epilogue: wave w handles M tiles t = w, w+4, ...
  const float bb = (bias != nullptr && n < N) ? bias[n] : 0.f;
  for (int t = wave; t < MT; t += 4) {
    f32x4 s = red[0][t][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) s += red[w][t][lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = t * 16 + (lane >> 4) * 4 + r;
      if (m < M && n < N) {
        float v = s[r] + bb;
        if (ACT == ACT_RELU) v = fmaxf(v, 0.f);
        if (ACT == ACT_GELU) v = gelu_erf(v);
        if (R != nullptr) v += bf2f(R[(size_t)m * ldr + n]);
        if (OUT_F32) reinterpret_cast<float*>(Cv)[(size_t)m * ldc + n] = v;
        else reinterpret_cast<bf16_t*>(Cv)[(size_t)m * ldc + n] = f2bf(v);
      }
    }
  }
}

// SwiGLU for the skinny path: h[m, j] = silu(g[m, j]) * u[m, j] where the skinny
// GEMM produced the packed [M, 2F] fp32/bf16 output.
__global__ void silu_mul_packed_kernel(const bf16_t* __restrict__ gu, int ld_in, bf16_t* __restrict__ out,
                                       int ld_out, int M, int F) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * F) return;
  const int m = idx / F, j = idx % F;
  const int grp = j / 16, c = j % 16;
  const float g = bf2f(gu[(size_t)m * ld_in + grp * 32 + c]);
  const float u = bf2f(gu[(size_t)m * ld_in + grp * 32 + 16 + c]);
  out[(size_t)m * ld_out + j] = f2bf(silu(g) * u);
}

}  // namespace dnn

// ------------------------------- host API ----------------------------------
using namespace dnn;

template <int ACT, bool F32>
static void launch_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                        const void* R, int ldr, int M, int N, int K, hipStream_t st) {
  if (M <= 64 && ACT != ACT_SILU_MUL) {
    dim3 grid((N + 15) / 16);
#define SK(MTV)                                                                                         \
  hipLaunchKernelGGL((gemm_skinny_kernel<ACT, F32, MTV>), grid, dim3(256), 0, st, (const bf16_t*)A, lda, \
                     (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, K)
    if (M <= 16) SK(1);
    else if (M <= 32) SK(2);
    else SK(4);
#undef SK
    return;
  }
  const int tiles = ((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N);
  hipLaunchKernelGGL((gemm_bf16_tn_kernel<ACT, F32>), dim3(tiles), dim3(256), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, K);
}

extern "C" int dnn_gemm_bf16(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                             const void* R, int ldr, int M, int N, int K, int act, int out_f32, hipStream_t st) {
  if (K % 64 != 0 || M <= 0 || N <= 0) return -1;
#define DISPATCH(a)                                                                     \
  if (act == a) {                                                                       \
    if (out_f32) launch_gemm<a, true>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, st); \
    else launch_gemm<a, false>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, st);        \
    return (int)hipGetLastError();                                                      \
  }
  DISPATCH(ACT_NONE)
  DISPATCH(ACT_RELU)
  DISPATCH(ACT_GELU)
  DISPATCH(ACT_SILU_MUL)
#undef DISPATCH
  return -2;
}

extern "C" int dnn_silu_mul_packed(const void* gu, int ld_in, void* out, int ld_out, int M, int F, hipStream_t st) {
  const int n = M * F;
  hipLaunchKernelGGL(silu_mul_packed_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const bf16_t*)gu, ld_in,
                     (bf16_t*)out, ld_out, M, F);
  return (int)hipGetLastError();
}
