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
// Decode-sized M (<= 64) goes to the weight-streaming kernels of gemm_skinny.hip.
#include <type_traits>

#include "api.h"
#include "gemm_epilogue.h"

namespace dnn {

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

// Tile order: the XCD remap gives each XCD a contiguous run of logical ids;
// inside it tiles go GROUP_M rows of M-tiles at a time, M fastest, so the ~32-64
// tiles co-resident on one XCD share a few A and W panels in its L2.
__device__ __forceinline__ void tile_coords(int logical, int ntm, int ntn, int& tm, int& tn) {
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * ntn;
  const int grp = logical / per_group;
  const int first = grp * GROUP_M;
  const int gm = min(ntm - first, GROUP_M);
  const int r = logical - grp * per_group;
  tm = first + r % gm;
  tn = r / gm;
}

// Epilogue on a TRANSPOSED accumulator: the MFMAs are issued as W.A^T, so a
// lane holds 4 consecutive output columns n..n+3 of one row m (C/D map of the
// 16x16 MFMA with the operands swapped) and writes them as one 8-B (bf16) or
// 16-B (fp32) store instead of four scattered 2-B stores.
template <int ACT, bool OUT_F32>
__global__ __launch_bounds__(256, 2) void gemm_bf16_tn_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, int ldw, void* __restrict__ Cv,
    int ldc, const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr, int M, int N, int K,
    const float2* __restrict__ rowstat, const float* __restrict__ colsum) {
  __shared__ __attribute__((aligned(16))) char smem[4 * G_TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + GB_N - 1) / GB_N, ntm = (M + GB_M - 1) / GB_M;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, tm, tn);
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

  // two K-tiles per trip: the double-buffer index is a compile-time constant
  auto ktile = [&](const int t, auto ccst) {
    constexpr int cur = decltype(ccst)::value;
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
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});

  // Epilogue (transposed accumulators): lane holds row m = .. + (lane&15), cols n..n+3.
  if (rowstat != nullptr) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = epi_norm4(acc[i][j], m0 + wm * 64 + i * 16 + (lane & 15), n0 + wn * 64 + j * 16 + (lane >> 4) * 4,
                              M, N, rowstat, colsum);
  }
  const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
  const bool pair = vec && epi_pair_ok(Cv, ldc, bias, R, ldr);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (ACT == ACT_SILU_MUL) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
        epi_silu_pair<OUT_F32>(acc[i][2 * jp], acc[i][2 * jp + 1], m, (n0 + wn * 64 + jp * 32) / 2, M, N / 2, Cv,
                               ldc, vec, lane);
    } else if (!OUT_F32 && pair) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int nb = n0 + wn * 64 + jp * 32;
        if (nb + 31 < N)
          epi_pair_bf16<ACT>(acc[i][2 * jp], acc[i][2 * jp + 1], m, nb, M, reinterpret_cast<bf16_t*>(Cv), ldc, bias,
                             R, ldr, lane);
        else
#pragma unroll
          for (int j = 2 * jp; j < 2 * jp + 2; ++j)
            epi_t4<ACT, OUT_F32>(acc[i][j], m, n0 + wn * 64 + j * 16 + (lane >> 4) * 4, M, N, Cv, ldc, bias, R, ldr,
                                 vec);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        epi_t4<ACT, OUT_F32>(acc[i][j], m, n0 + wn * 64 + j * 16 + (lane >> 4) * 4, M, N, Cv, ldc, bias, R, ldr, vec);
    }
  }
}

// ---------------------------------------------------------------------------
// Large-tile GEMM: 256x256x64, 8 waves (2 M x 4 N), ~1 block per CU, the
// 4-phase-per-K-tile schedule of the guide's 256^2 template (§5 "8-phase"):
//
//   LDS = [2 buffers][A0 A1 B0 B1] half-tiles of 128 rows x 64 k (16 KiB each),
//   one __shared__ array (trap 4(a)).  Half-tile h of A holds the rows of every
//   wave's output quadrant-row h, so a wave's 128x64 output is 2x2 quadrants of
//   64x32 and each phase is one quadrant x K=64 = 16 MFMAs:
//
//     ph1: read B0 (4 ds_read_b128), A0 (8)  | stage A1[t+1] -> buf^1 | C00
//     ph2: read B1 (4)                       | stage B0[t+1] -> buf^1 | C01
//     ph3: read A1 (8)                       | stage A0[t+2] -> buf   | C11
//     ph4: read B0 (4)                       | stage B1[t+2] -> buf   | C10
//          + s_waitcnt vmcnt(4)  (retires everything of tile t+1)
//
//   Every restage lands >= 2 phases after the last read of that half-tile
//   (WAR), every read is >= 1 phase after the vmcnt+barrier that retired its
//   DMA (RAW).  Each phase = [ds_reads + 2 glds] s_barrier [lgkmcnt(0),
//   setprio(1), 16 MFMA] s_barrier; waves of M-row 1 run one barrier behind
//   M-row 0, so on every SIMD one wave issues LDS reads while its partner
//   issues MFMAs.  glds stays in flight across barriers (raw s_barrier, counted
//   vmcnt, never __syncthreads in the loop).  Loads past the last K-tile are
//   clamped to it (harmless refills of dead buffers) so the vmcnt count is
//   uniform.
// ---------------------------------------------------------------------------
constexpr int BG_M = 256, BG_N = 256, BG_K = 64;
constexpr int BG_HALF = 128 * BG_K * 2;  // 16 KiB

// Stage one 128x64 half-tile: 2 glds per thread, 8 rows per wave-instruction.
__device__ __forceinline__ void stage_half(const bf16_t* __restrict__ src, int ld, int r0, int nrows, int k0,
                                           char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = i * 8 + wave;
    const int rl = piece * 8 + (lane >> 3);
    const int cs = (lane & 7) ^ swz_chunk(rl);
    int r = r0 + rl;
    r = r < nrows ? r : nrows - 1;
    glds16(src + (size_t)r * ld + k0 + cs * 8, dst + piece * 1024);
  }
}

// Epilogue operands of a 256^2 tile by LDS-DMA, into EPI_LDS bytes past the
// operand buffers, issued before the first staging DMA (so the prologue's
// counted wait retires them and no register carries them through the main
// loop): wave 0 the bias of the tile's 256 columns, wave 1 the per-column
// scale (fp8 channel scales / folded-norm column sums), waves 2-3 the row
// statistics (float2) of its 256 rows, wave 4 the per-row fp8 activation
// scales.  After the main loop every output group then reads them from LDS:
// loaded there per group they cost one dependent memory round trip each (16
// per tile), a load under a branch being waited for at the merge.  Addresses
// past the matrix clamp to its last 16 B (host/kernel: N % 4 == 0, M even,
// 16-B aligned vectors; those columns / rows are never stored).
// Anatomy probe of the 256^2 kernels (bench/probes/gemm_anatomy.py; 0 in every
// product launch): bit 1 skips the epilogue's stores (the accumulators stay
// live through one sentinel compare), bit 2 skips the main loop (prologue DMAs,
// their wait and the epilogue only), bit 8 runs the whole epilogue but
// predicates its plain-path stores off, bit 4 reads the residual by per-lane
// gathers instead of the LDS-DMA tile -- what a tile's fixed cost is made of
// (profiles/r6_gemm_anatomy.jsonl: ~8-10 us of stores per tile at M = 32768;
// row-staged, non-temporal or start-staggered stores were measured and
// reverted, docs/ARCHITECTURE.md "Tried and reverted").
__device__ int g_gemm_anatomy = 0;

constexpr int EPI_LDS = 5 * 1024;
constexpr int EPI_B = 0, EPI_C = 1024, EPI_RS = 2048, EPI_SA = 4096;  // byte offsets

__device__ __forceinline__ void epi_operands_dma(const float* bias, const float* col, const float2* rowstat,
                                                 const float* sa, int n0, int N, int m0, int M, char* dst, int wave,
                                                 int lane) {
  if (wave == 0 && bias != nullptr) glds16(bias + min(n0 + 4 * lane, N - 4), dst + EPI_B);
  if (wave == 1 && col != nullptr) glds16(col + min(n0 + 4 * lane, N - 4), dst + EPI_C);
  if ((wave == 2 || wave == 3) && rowstat != nullptr)
    glds16(rowstat + min(m0 + (wave - 2) * 128 + 2 * lane, M - 2), dst + EPI_RS + (wave - 2) * 1024);
  if (wave == 4 && sa != nullptr) glds16(sa + min(m0 + 4 * lane, M - 4), dst + EPI_SA);
}

__device__ __forceinline__ void bg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int MI, int NJ>
__device__ __forceinline__ void bg_mfma(f32x4 (&acc)[MI][NJ], const bf16x8 (&a)[MI][2], const bf16x8 (&b)[NJ][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[i][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

template <int N>
__device__ __forceinline__ void bg_read(bf16x8 (&f)[N][2], const char* half, int row0, int lane) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) f[i][s] = lds_frag(half, row0 + i * 16 + (lane & 15), s * 4 + (lane >> 4));
}

// QKV scatter epilogue (prefill c_attn, no RoPE): output column c of row
// m = b*T + t lands head-major — q -> q[b][h][t][:], k / v -> the KV caches at
// position pos[b] + t — instead of in a (M, (H+2Hkv) hd) qkv row, so the flash
// prefill reads contiguous K/V from the cache and no longer copies them there
// (bench/flash_copy_probe.py: 21 us of a 116 us GPT-2 attention layer).
struct QkvScatter {
  bf16_t* q;
  bf16_t* k;
  bf16_t* v;
  const int* pos;
  int T, H, Hkv, hd_shift, S;  // head dim = 1 << hd_shift
  float invT;                  // 1 / T (row -> sequence without an integer division)
  int c_off = 0;               // first qkv column of this launch (the tail-split launch covers the last 256)
};

// 8 consecutive output columns c..c+7 (one head) of row m -> destination.  The
// store count is 32 per lane and tile, so the index math avoids integer
// division: b = m / T from the fp32 reciprocal with a one-step correction
// (exact for m < 2^24), head / dim by shifts (hd a power of two).
__device__ __forceinline__ int qkv_batch(const QkvScatter& sc, int m) {
  int b = (int)(((float)m + 0.5f) * sc.invT);
  b -= b * sc.T > m ? 1 : 0;
  b += (b + 1) * sc.T <= m ? 1 : 0;
  return b;
}
// the cache position of row m (pos[b] + t), loaded for a lane's 8 rows before
// the epilogue's first store: loaded per 32-column pair it waited, through the
// in-order vmcnt, for every store issued before it
__device__ __forceinline__ int qkv_row_pos(const QkvScatter& sc, int m) {
  const int b = qkv_batch(sc, m);
  return sc.pos[b] + (m - b * sc.T);
}
__device__ __forceinline__ bf16_t* qkv_dest(const QkvScatter& sc, int m, int c, int p) {
  const int b = qkv_batch(sc, m);
  const int t = m - b * sc.T;
  const int hs = sc.hd_shift, hmask = (1 << hs) - 1;
  const int qw = sc.H << hs, kw = sc.Hkv << hs;
  if (c < qw) return sc.q + ((((size_t)b * sc.H + (c >> hs)) * sc.T + t) << hs) + (c & hmask);
  if (p >= sc.S) return nullptr;  // past the cache capacity: dropped, as in qkv_split
  const bool isk = c < qw + kw;
  const int cc = isk ? c - qw : c - qw - kw;
  return (isk ? sc.k : sc.v) + ((((size_t)b * sc.Hkv + (cc >> hs)) * sc.S + p) << hs) + (cc & hmask);
}

// One widened 16-B store per lane (as epi_pair_bf16) of a whole 32-column pair
// to its head-major / cache destination (bias added first, no activation).
__device__ __forceinline__ void epi_pair_scatter(f32x4 a0, f32x4 a1, int m, int nb, int M,
                                                 const float* __restrict__ bias, int lane, const QkvScatter& sc,
                                                 int p) {
  const int q = lane >> 4;
  if (bias != nullptr) {
    a0 += *reinterpret_cast<const f32x4*>(bias + nb + q * 4);
    a1 += *reinterpret_cast<const f32x4*>(bias + nb + 16 + q * 4);
  }
  const uint32_t x0 = pack2bf(a0[0], a0[1]), x1 = pack2bf(a0[2], a0[3]);
  const uint32_t y0 = pack2bf(a1[0], a1[1]), y1 = pack2bf(a1[2], a1[3]);
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  if (m < M) {
    bf16_t* d = qkv_dest(sc, m, nb + ((q & 1) << 4) + ((q >> 1) << 3), p);
    if (d != nullptr) *reinterpret_cast<uint4*>(d) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  }
}

// NQ = 2: 256x256 tiles (4 phases per K-tile, below).  NQ = 1: 256x128 tiles
// for N where the 256^2 grid leaves its last round of 256 CUs half empty
// (GPT-2's 768-wide projections at M = 32768: 384 tiles = 1.5 rounds; as
// 256x128 768 tiles = 3 full rounds of half-size tiles).
// Same waves (2 M x 4 N) and LDS images; a wave owns 2 x 1 quadrants of 64x32
// and a K-tile is two phases:
//     ph1: read B0 (4), A0 (8)  | stage A0, B0 [t+1] -> buf^1 | vmcnt(4) | C00
//     ph2: read A1 (8)          | stage A1 [t+1]     -> buf^1 | vmcnt(2) | C10
// (one tile ahead: every restage lands 2 phases after the last read of its
// half-tile, every read 1 phase after the wait + barrier that retired it).
template <int ACT, bool OUT_F32, bool SCATTER = false, int NQ = 2>
__global__ __launch_bounds__(512, 1) void gemm_bf16_256_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, int ldw, void* __restrict__ Cv,
    int ldc, const float* __restrict__ bias, const bf16_t* __restrict__ R, int ldr, int M, int N, int K,
    int res_pre, const float2* __restrict__ rowstat, const float* __restrict__ colsum, QkvScatter scat = {}) {
  static_assert(NQ == 1 || NQ == 2, "256x256 or 256x128 tiles");
  constexpr int TN = 128 * NQ;
  __shared__ __attribute__((aligned(1024))) char smem[8 * BG_HALF + EPI_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + TN - 1) / TN, ntm = (M + BG_M - 1) / BG_M;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, tm, tn);
  const int m0 = tm * BG_M, n0 = tn * TN;
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / BG_K;
  const int gan = g_gemm_anatomy;
  // epilogue operands in LDS (epi_operands_dma); uniform.  SCATTER: the bias
  // is indexed by the global column (the tail launch's c_off).
  char* epi = smem + 8 * BG_HALF;
  const int boff = SCATTER ? scat.c_off : 0;
  const bool epv = (N & 3) == 0 && (M & 1) == 0 && M >= 2 && N >= 4 &&
                   ((reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(colsum) |
                     reinterpret_cast<uintptr_t>(rowstat)) & 15) == 0;
  if (epv)
    epi_operands_dma(bias != nullptr ? bias + boff : nullptr, colsum, rowstat, nullptr, n0, N, m0, M, epi, wave, lane);

  f32x4 acc[2][NQ][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NQ; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half-tile h of buffer u: A0=0, A1=1, B0=2, B1=3
  auto half = [&](int u, int h) { return smem + (u * 4 + h) * BG_HALF; };
  auto stA = [&](int u, int h, int t) {
    t = t < nk ? t : nk - 1;
    stage_half(A, lda, m0 + h * 128, M, t * BG_K, half(u, h), wave, lane);
  };
  auto stB = [&](int u, int h, int t) {
    t = t < nk ? t : nk - 1;
    stage_half(W, ldw, n0 + h * 128, N, t * BG_K, half(u, 2 + h), wave, lane);
  };

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = wr * 64, brow = wc * 32;
  if constexpr (NQ == 1) {
    // prologue: tile 0 complete
    stA(0, 0, 0);
    stB(0, 0, 0);
    stA(0, 1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bg_barrier();
    if (wr == 1) bg_barrier();
    auto ktile1 = [&](const int t, auto ucst) {
      constexpr int u = decltype(ucst)::value;
      // ph1
      bg_read<2>(b0, half(u, 2), brow, lane);
      __builtin_amdgcn_sched_barrier(0);
      bg_read<4>(af, half(u, 0), arow, lane);
      stA(u ^ 1, 0, t + 1);
      stB(u ^ 1, 0, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A1 of tile t landed
      bg_barrier();
      bg_mfma<4, 2>(acc[0][0], af, b0);
      bg_barrier();
      // ph2
      bg_read<4>(af, half(u, 1), arow, lane);
      stA(u ^ 1, 1, t + 1);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A0 / B0 of tile t+1 landed
      bg_barrier();
      bg_mfma<4, 2>(acc[1][0], af, b0);
      bg_barrier();
    };
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      ktile1(t, std::integral_constant<int, 0>{});
      ktile1(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nk) ktile1(t, std::integral_constant<int, 0>{});
  } else {
  // prologue: tile 0 complete, A0/B1 of tile 1 in flight
  stA(0, 0, 0);
  stB(0, 1, 0);
  stA(0, 1, 0);
  stB(0, 0, 0);
  stA(1, 0, 1);
  stB(1, 1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bg_barrier();
  if (wr == 1) bg_barrier();

  // One K-tile; the loop runs two per iteration so the buffer index u is a
  // compile-time constant and every LDS address an immediate offset.
  auto ktile = [&](const int t, auto ucst) {
    constexpr int u = decltype(ucst)::value;
    // ph1
    bg_read<2>(b0, half(u, 2), brow, lane);
    __builtin_amdgcn_sched_barrier(0);
    bg_read<4>(af, half(u, 0), arow, lane);
    stA(u ^ 1, 1, t + 1);
    bg_barrier();
    bg_mfma<4, 2>(acc[0][0], af, b0);
    bg_barrier();
    // ph2
    bg_read<2>(b1, half(u, 3), brow, lane);
    stB(u ^ 1, 0, t + 1);
    bg_barrier();
    bg_mfma<4, 2>(acc[0][1], af, b1);
    bg_barrier();
    // ph3
    bg_read<4>(af, half(u, 1), arow, lane);
    stA(u, 0, t + 2);
    bg_barrier();
    bg_mfma<4, 2>(acc[1][1], af, b1);
    bg_barrier();
    // ph4
    bg_read<2>(b0, half(u, 2), brow, lane);
    stB(u, 1, t + 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    bg_barrier();
    bg_mfma<4, 2>(acc[1][0], af, b0);
    bg_barrier();
  };
  int t = (gan & 2) ? nk : 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wr == 0) bg_barrier();
  if (gan & 1) {  // anatomy probe: no stores
    if (acc[0][0][0][0][0] == 1.2345e-30f) reinterpret_cast<bf16_t*>(Cv)[0] = 0;
    return;
  }

  // Epilogue (transposed accumulators):
  //   row m = m0 + mq*128 + wr*64 + i*16 + (lane&15), cols n..n+3 with
  //   n = n0 + nq*128 + wc*32 + j*16 + (lane>>4)*4.
  if (rowstat != nullptr) {  // folded pre-norm (prefill QKV / up projections)
    // 8 row statistics and 4 column-sum vectors per lane (from the LDS copy)
    float2 rs[2][4];
    f32x4 cs[NQ][2];
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = mq * 128 + arow + i * 16 + (lane & 15);
        rs[mq][i] = epv ? reinterpret_cast<const float2*>(epi + EPI_RS)[rl] : rowstat[min(m0 + rl, M - 1)];
      }
#pragma unroll
    for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + nq * 128 + wc * 32 + j * 16 + (lane >> 4) * 4;
        cs[nq][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (colsum != nullptr) {
          if (epv) {
            cs[nq][j] = *reinterpret_cast<const f32x4*>(epi + EPI_C + 4 * (n - n0));
          } else if (n + 3 < N) {
            cs[nq][j] = *reinterpret_cast<const f32x4*>(colsum + n);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[nq][j][r] = n + r < N ? colsum[n + r] : 0.f;
          }
        }
      }
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq][nq][i][j] = acc[mq][nq][i][j] * rs[mq][i].x + rs[mq][i].y * cs[nq][j];
  }
  // the bias from the LDS copy, added here: the output calls get none to load
  const bool badd = epv && bias != nullptr && ACT != ACT_SILU_MUL;  // uniform
  if (badd) {
#pragma unroll
    for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(epi + EPI_B + 4 * (nq * 128 + wc * 32 + j * 16 + (lane >> 4) * 4));
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[mq][nq][i][j] += b4;
      }
  }
  const float* bias_e = badd ? nullptr : bias;
  // SCATTER: the cache positions of the lane's 8 rows, loaded before any store (qkv_row_pos)
  int spos[2][4] = {};
  if constexpr (SCATTER) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) spos[mq][i] = qkv_row_pos(scat, min(m0 + mq * 128 + arow + i * 16 + (lane & 15), M - 1));
  }
  const bool vec = epi_vec_ok(Cv, ldc, bias, R, ldr);
  const bool pair = vec && epi_pair_ok(Cv, ldc, bias, R, ldr);
  // Residual epilogue: every residual load of the tile (32 x 8 B per lane, into
  // the fragment registers the main loop no longer needs) is issued before the
  // first output is computed, so the tile pays one memory round trip for R
  // instead of one per output row group (-20..-25 % GEMM throughput otherwise,
  // profiles/archive/r2_gemm_epilogue_cost.jsonl).
  if (res_pre && !OUT_F32 && ACT != ACT_SILU_MUL && pair && R != nullptr && n0 + TN - 1 < N && (gan & 4) == 0 &&
      (ldr & 7) == 0 && (reinterpret_cast<uintptr_t>(R) & 15) == 0) {
    // the residual tile by LDS-DMA into the dead operand buffers (res_tile_dma;
    // anatomy bit 4 = the per-lane gathers below)
    __syncthreads();  // every wave past its last operand read and DMA (vmcnt(0) above)
    res_tile_dma<TN>(R, ldr, m0, n0, M, smem, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = mq * 128 + arow + i * 16 + (lane & 15), cl = nq * 128 + wc * 32 + (lane >> 4) * 4;
          epi_pair_bf16<ACT, true>(acc[mq][nq][i][0], acc[mq][nq][i][1], m0 + rl, n0 + nq * 128 + wc * 32, M,
                                   reinterpret_cast<bf16_t*>(Cv), ldc, bias_e, R, ldr, lane,
                                   res_tile_read<TN>(smem, rl, cl), res_tile_read<TN>(smem, rl, cl + 16));
        }
    return;
  }
  if (res_pre && !OUT_F32 && ACT != ACT_SILU_MUL && pair && R != nullptr && n0 + TN - 1 < N) {
    bf16x4 rr[2][NQ][4][2];
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          epi_pair_res_load(m0 + mq * 128 + arow + i * 16 + (lane & 15), n0 + nq * 128 + wc * 32, M, R, ldr, lane,
                            rr[mq][nq][i][0], rr[mq][nq][i][1]);
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          epi_pair_bf16<ACT, true>(acc[mq][nq][i][0], acc[mq][nq][i][1], m0 + mq * 128 + arow + i * 16 + (lane & 15),
                                   n0 + nq * 128 + wc * 32, M, reinterpret_cast<bf16_t*>(Cv), ldc, bias_e, R, ldr, lane,
                                   rr[mq][nq][i][0], rr[mq][nq][i][1]);
    return;
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + mq * 128 + arow + i * 16 + (lane & 15);
        const int nb = n0 + nq * 128 + wc * 32;
        if (ACT == ACT_SILU_MUL) {
          epi_silu_pair<OUT_F32>(acc[mq][nq][i][0], acc[mq][nq][i][1], m, nb / 2, M, N / 2, Cv, ldc, vec, lane);
        } else if (SCATTER) {
          // widened 16-B stores as in epi_pair_bf16, to the head-major / cache
          // destination of the lane's 8 columns (host: ACT_NONE, bf16 out, no
          // residual, N % 32 == 0, hd % 8 == 0 -> a 32-column pair is whole or
          // past N, wave-uniformly)
          if (nb < N)
            epi_pair_scatter(acc[mq][nq][i][0], acc[mq][nq][i][1], m, nb + scat.c_off, M, bias_e, lane, scat,
                             spos[mq][i]);
        } else if (!OUT_F32 && pair && nb + 31 < N) {
          epi_pair_bf16<ACT>(acc[mq][nq][i][0], acc[mq][nq][i][1], m, nb, (gan & 8) ? 0 : M, reinterpret_cast<bf16_t*>(Cv), ldc,
                             bias_e, R, ldr, lane);
        } else {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            epi_t4<ACT, OUT_F32>(acc[mq][nq][i][j], m, nb + j * 16 + (lane >> 4) * 4, M, N, Cv, ldc, bias_e, R,
                                 ldr, vec);
        }
      }
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3fn) on the same 256^2 4-phase schedule: a K-tile is 128 fp8 =
// 128 B per row, so every LDS half-tile, glds piece and swizzle is
// byte-identical to the bf16 kernel's BK = 64 and the staging code is shared.
// Per (i, j) and K-tile ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 block
// scales, 2x the bf16 rate) replaces the two bf16 16x16x32: lane group g feeds
// chunks g and 4+g of its row as its 32 "k" bytes — the same permutation of k
// for both operands, so the dot product is unchanged and the fragment reads are
// exactly the bf16 kernel's (conflict-free) ones.  Epilogue: per-token scale
// sa[m] and per-channel scale sw[n] on the fp32 accumulators, then the shared
// bias / act / residual / SwiGLU epilogues (16-B paired stores).
// ---------------------------------------------------------------------------
typedef int i32x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ i32x8_t f8_cat(const bf16x8& lo, const bf16x8& hi) {
  i32x8_t r;
  const i32x4 a = __builtin_bit_cast(i32x4, lo), b = __builtin_bit_cast(i32x4, hi);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

template <int MI, int NJ>
__device__ __forceinline__ void bg_mfma_f8(f32x4 (&acc)[MI][NJ], const bf16x8 (&a)[MI][2], const bf16x8 (&b)[NJ][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(f8_cat(b[j][0], b[j][1]), f8_cat(a[i][0], a[i][1]),
                                                                   acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  __builtin_amdgcn_s_setprio(0);
}

// MX e8m0 scales of the activations on the scaled MFMA (MXA, common.h
// mx_index: one dword per lane per 128-row half-tile and K-tile, byte i =
// fragment i): acc carries the activation scales, the epilogue only the
// weight channel scale.
template <int MI, int NJ>
__device__ __forceinline__ void bg_mfma_f8x(f32x4 (&acc)[MI][NJ], const bf16x8 (&a)[MI][2], const bf16x8 (&b)[NJ][2],
                                            uint32_t s) {
  static_assert(MI == 4, "one op_sel byte per A fragment");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const i32x8_t bj = f8_cat(b[j][0], b[j][1]);
    acc[0][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bj, f8_cat(a[0][0], a[0][1]), acc[0][j], 0, 0, 0,
                                                                 0x7f7f7f7f, 0, s);
    acc[1][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bj, f8_cat(a[1][0], a[1][1]), acc[1][j], 0, 0, 0,
                                                                 0x7f7f7f7f, 1, s);
    acc[2][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bj, f8_cat(a[2][0], a[2][1]), acc[2][j], 0, 0, 0,
                                                                 0x7f7f7f7f, 2, s);
    acc[3][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bj, f8_cat(a[3][0], a[3][1]), acc[3][j], 0, 0, 0,
                                                                 0x7f7f7f7f, 3, s);
  }
  __builtin_amdgcn_s_setprio(0);
}

// QOUT (GELU c_fc of the MX prefill): the epilogue quantises its own output
// tile for the next GEMM — e4m3 bytes q_out[M][ldq] with one e8m0 scale per
// (row, 128 columns) from the tile's columns alone (the 4 waves sharing a row
// agree through LDS), so the c_proj input never exists in bf16 and no
// quantise pass reads it back.  Columns >= N are written as zeros up to kpo.
template <int ACT, bool SCATTER = false, int NQ = 2, bool MXA = false, bool QOUT = false>
__global__ __launch_bounds__(512, 1) void gemm_fp8_256_kernel(
    const uint8_t* __restrict__ A8, const float* __restrict__ sa, const uint8_t* __restrict__ W8,
    const float* __restrict__ sw, bf16_t* __restrict__ C, int ldc, const float* __restrict__ bias,
    const bf16_t* __restrict__ R, int ldr, int M, int N, int Kb, QkvScatter scat = {},
    const uint32_t* __restrict__ sx = nullptr, uint8_t* __restrict__ qo = nullptr, int ldq = 0,
    uint8_t* __restrict__ sxo = nullptr, int kpo = 0) {
  // (QOUT reuses the operand LDS after the main loop: see the epilogue)
  static_assert(NQ == 1 || NQ == 2, "256x256 or 256x128 tiles");
  static_assert(!MXA || NQ == 2, "MX activations: 256^2 tiles");
  static_assert(!QOUT || (MXA && ACT == ACT_GELU && !SCATTER), "quantised output: the MX c_fc");
  constexpr int TN = 128 * NQ;  // NQ = 1: the 256x128 variant (tail-split launches), as the bf16 kernel's
  __shared__ __attribute__((aligned(1024))) char smem[8 * BG_HALF + EPI_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + TN - 1) / TN, ntm = (M + BG_M - 1) / BG_M;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, tm, tn);
  const int m0 = tm * BG_M, n0 = tn * TN;
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = Kb / 128;
  const int gan = g_gemm_anatomy;
  // epilogue operands in LDS (epi_operands_dma): channel scales, bias (SCATTER:
  // by the global column), per-row activation scales (not MXA); uniform
  char* epi = smem + 8 * BG_HALF;
  const int boff = SCATTER ? scat.c_off : 0;
  const bool epv = (N & 3) == 0 && (MXA || (M & 3) == 0) && M >= 4 && N >= 4 &&
                   ((reinterpret_cast<uintptr_t>(sw) | reinterpret_cast<uintptr_t>(bias) |
                     reinterpret_cast<uintptr_t>(sa)) & 15) == 0;
  if (epv)
    epi_operands_dma(bias != nullptr ? bias + boff : nullptr, sw, nullptr, MXA ? nullptr : sa, n0, N, m0, M, epi,
                     wave, lane);
  // byte-identical staging: view the e4m3 rows as bf16 rows of half the length
  const bf16_t* A = reinterpret_cast<const bf16_t*>(A8);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(W8);
  const int lda = Kb / 2, ldw = Kb / 2;

  f32x4 acc[2][NQ][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NQ; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto half = [&](int u, int h) { return smem + (u * 4 + h) * BG_HALF; };
  auto stA = [&](int u, int h, int t) {
    t = t < nk ? t : nk - 1;
    stage_half(A, lda, m0 + h * 128, M, t * BG_K, half(u, h), wave, lane);
  };
  auto stB = [&](int u, int h, int t) {
    t = t < nk ? t : nk - 1;
    stage_half(W, ldw, n0 + h * 128, N, t * BG_K, half(u, 2 + h), wave, lane);
  };

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = wr * 64, brow = wc * 32;
  if constexpr (NQ == 1) {
    // the bf16 kernel's 2-phase K-tile (256x128), one scaled MFMA per tile pair
    stA(0, 0, 0);
    stB(0, 0, 0);
    stA(0, 1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bg_barrier();
    if (wr == 1) bg_barrier();
    auto ktile1 = [&](const int t, auto ucst) {
      constexpr int u = decltype(ucst)::value;
      bg_read<2>(b0, half(u, 2), brow, lane);
      __builtin_amdgcn_sched_barrier(0);
      bg_read<4>(af, half(u, 0), arow, lane);
      stA(u ^ 1, 0, t + 1);
      stB(u ^ 1, 0, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A1 of tile t landed
      bg_barrier();
      bg_mfma_f8<4, 2>(acc[0][0], af, b0);
      bg_barrier();
      bg_read<4>(af, half(u, 1), arow, lane);
      stA(u ^ 1, 1, t + 1);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A0 / B0 of tile t+1 landed
      bg_barrier();
      bg_mfma_f8<4, 2>(acc[1][0], af, b0);
      bg_barrier();
    };
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      ktile1(t, std::integral_constant<int, 0>{});
      ktile1(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nk) ktile1(t, std::integral_constant<int, 0>{});
  } else {
  // MXA: the scale dwords of K-tile t (half-tiles 0 / 1 of A) in scl[t & 1];
  // tile t + 1's are loaded in tile t's first phase, so the phase-4 vmcnt(4)
  // (which retires everything but the last four DMAs) has retired them too
  uint32_t scl[2][2] = {{0x7f7f7f7fu, 0x7f7f7f7fu}, {0x7f7f7f7fu, 0x7f7f7f7fu}};
  const int nb64 = mx_mpad(M) >> 6;
  auto ldsx = [&](int t, uint32_t (&d)[2]) {
    t = t < nk ? t : nk - 1;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      d[h] = sx[((size_t)t * nb64 + min((m0 >> 6) + 2 * h + wr, nb64 - 1)) * 16 + (lane & 15)];
  };
  if constexpr (MXA) ldsx(0, scl[0]);
  stA(0, 0, 0);
  stB(0, 1, 0);
  stA(0, 1, 0);
  stB(0, 0, 0);
  stA(1, 0, 1);
  stB(1, 1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bg_barrier();
  if (wr == 1) bg_barrier();

  auto mm = [&](f32x4 (&c)[4][2], const bf16x8 (&bb)[2][2], uint32_t s) {
    if constexpr (MXA) bg_mfma_f8x<4, 2>(c, af, bb, s);
    else bg_mfma_f8<4, 2>(c, af, bb);
  };
  auto ktile = [&](const int t, auto ucst) {
    constexpr int u = decltype(ucst)::value;
    bg_read<2>(b0, half(u, 2), brow, lane);
    __builtin_amdgcn_sched_barrier(0);
    bg_read<4>(af, half(u, 0), arow, lane);
    stA(u ^ 1, 1, t + 1);
    if constexpr (MXA) ldsx(t + 1, scl[u ^ 1]);
    bg_barrier();
    mm(acc[0][0], b0, scl[u][0]);
    bg_barrier();
    bg_read<2>(b1, half(u, 3), brow, lane);
    stB(u ^ 1, 0, t + 1);
    bg_barrier();
    mm(acc[0][1], b1, scl[u][0]);
    bg_barrier();
    bg_read<4>(af, half(u, 1), arow, lane);
    stA(u, 0, t + 2);
    bg_barrier();
    mm(acc[1][1], b1, scl[u][1]);
    bg_barrier();
    bg_read<2>(b0, half(u, 2), brow, lane);
    stB(u, 1, t + 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    bg_barrier();
    mm(acc[1][0], b0, scl[u][1]);
    bg_barrier();
  };
  int t = (gan & 2) ? nk : 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wr == 0) bg_barrier();
  if (gan & 1) {  // anatomy probe: no stores
    if (acc[0][0][0][0][0] == 1.2345e-30f) C[0] = 0;
    return;
  }

  if constexpr (QOUT) {
    // bias + GELU in place, then per (row, 128-column half nq) amax: the lane's
    // 8 columns, the 4 lane rows of the wave (xor 16 / 32), the 4 waves of the
    // wave row through LDS (the operand buffers are dead), one barrier
    float* red = reinterpret_cast<float*>(smem);  // [mq][nq][i][wr][16][wc]
    __syncthreads();  // every wave past its last operand read and DMA (vmcnt(0) above)
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float am = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + nq * 128 + wc * 32 + j * 16 + (lane >> 4) * 4;
            // 16-B channel-scale / bias loads (per-element ones were 8 scalar
            // loads per quad)
            f32x4 cs, bs = f32x4{0.f, 0.f, 0.f, 0.f};
            if (epv) {  // the LDS copy (columns past N are zeroed below)
              cs = *reinterpret_cast<const f32x4*>(epi + EPI_C + 4 * (n - n0));
              if (bias != nullptr) bs = *reinterpret_cast<const f32x4*>(epi + EPI_B + 4 * (n - n0));
            } else if (n + 3 < N) {
              cs = *reinterpret_cast<const f32x4*>(sw + n);
              if (bias != nullptr) bs = *reinterpret_cast<const f32x4*>(bias + n);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                cs[r] = n + r < N ? sw[n + r] : 0.f;
                bs[r] = (bias != nullptr && n + r < N) ? bias[n + r] : 0.f;
              }
            }
            f32x4 v = acc[mq][nq][i][j] * cs + bs;
            const f32x2 g0 = gelu_erf2(f32x2{v[0], v[1]}), g1 = gelu_erf2(f32x2{v[2], v[3]});
            v = f32x4{g0[0], g0[1], g1[0], g1[1]};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = n + r < N ? v[r] : 0.f;
              am = fmaxf(am, fabsf(v[r]));
            }
            acc[mq][nq][i][j] = v;
          }
          am = fmaxf(am, __shfl_xor(am, 16, 64));
          am = fmaxf(am, __shfl_xor(am, 32, 64));
          if (lane < 16) red[((((mq * 2 + nq) * 4 + i) * 2 + wr) * 16 + lane) * 4 + wc] = am;
        }
    __syncthreads();
    const int mpad = mx_mpad(M);
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 a4 =
              *reinterpret_cast<const f32x4*>(red + ((((mq * 2 + nq) * 4 + i) * 2 + wr) * 16 + (lane & 15)) * 4);
          float inv;
          const uint32_t e = e8m0_of(fmaxf(fmaxf(a4[0], a4[1]), fmaxf(a4[2], a4[3])), inv);
          const f32x4 v0 = acc[mq][nq][i][0] * inv, v1 = acc[mq][nq][i][1] * inv;
          int x = __builtin_amdgcn_cvt_pk_fp8_f32(v0[0], v0[1], 0, false);
          x = __builtin_amdgcn_cvt_pk_fp8_f32(v0[2], v0[3], x, true);
          int y = __builtin_amdgcn_cvt_pk_fp8_f32(v1[0], v1[1], 0, false);
          y = __builtin_amdgcn_cvt_pk_fp8_f32(v1[2], v1[3], y, true);
          // as epi_pair_bf16: one permlane16_swap hands every lane 8 contiguous columns
          const auto sw2 = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)y, false, false);
          const int m = m0 + mq * 128 + arow + i * 16 + (lane & 15);
          const int q = lane >> 4;
          const int cb = n0 + nq * 128 + wc * 32;
          const int c = cb + ((q & 1) << 4) + ((q >> 1) << 3);
          if (m < M && c < kpo) *reinterpret_cast<uint2*>(qo + (size_t)m * ldq + c) = make_uint2(sw2[0], sw2[1]);
          const int t = (n0 + nq * 128) >> 7;
          if (wc == 0 && q == 0 && m < M && t * 128 < kpo) sxo[mx_index(m, t, mpad)] = (uint8_t)e;
        }
    return;
  }
  const bool badd = epv && bias != nullptr && ACT != ACT_SILU_MUL;  // uniform: bias added from the LDS copy
  const float* bias_e = badd ? nullptr : bias;
  // SCATTER: the cache positions of the lane's 8 rows, loaded before any store (qkv_row_pos)
  int spos[2][4] = {};
  if constexpr (SCATTER) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) spos[mq][i] = qkv_row_pos(scat, min(m0 + mq * 128 + arow + i * 16 + (lane & 15), M - 1));
  }
  const bool vec = epi_vec_ok(C, ldc, bias, R, ldr);
  const bool pair = vec && epi_pair_ok(C, ldc, bias, R, ldr);
  // residual rows of the whole tile in flight before the first output (as in the bf16 kernel)
  const bool rpre = ACT != ACT_SILU_MUL && pair && R != nullptr && n0 + TN - 1 < N;
  // the residual tile by LDS-DMA into the dead operand buffers (res_tile_dma;
  // anatomy bit 4 = the per-lane gathers below)
  const bool rdma = rpre && (gan & 4) == 0 && (ldr & 7) == 0 && (reinterpret_cast<uintptr_t>(R) & 15) == 0;
  bf16x4 rr[2][NQ][4][2];
  if (rdma) {
    __syncthreads();  // every wave past its last operand read and DMA (vmcnt(0) above)
    res_tile_dma<TN>(R, ldr, m0, n0, M, smem, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if (rpre) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          epi_pair_res_load(m0 + mq * 128 + arow + i * 16 + (lane & 15), n0 + nq * 128 + wc * 32, M, R, ldr, lane,
                            rr[mq][nq][i][0], rr[mq][nq][i][1]);
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < NQ; ++nq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + mq * 128 + arow + i * 16 + (lane & 15);
        const int nb = n0 + nq * 128 + wc * 32;
        // MXA: the activation scales are in acc
        const float rs = MXA ? 1.f
                             : (epv ? reinterpret_cast<const float*>(epi + EPI_SA)[m - m0] : (m < M ? sa[m] : 0.f));
        f32x4 v[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = nb + j * 16 + (lane >> 4) * 4;
          f32x4 cs;
          if (epv) {
            cs = *reinterpret_cast<const f32x4*>(epi + EPI_C + 4 * (n - n0));
          } else if (n + 3 < N) {
            cs = *reinterpret_cast<const f32x4*>(sw + n);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[r] = n + r < N ? sw[n + r] : 0.f;
          }
          v[j] = acc[mq][nq][i][j] * (cs * rs);
          if (badd) v[j] += *reinterpret_cast<const f32x4*>(epi + EPI_B + 4 * (n - n0));
        }
        if (SCATTER) {
          if (nb < N) epi_pair_scatter(v[0], v[1], m, nb + scat.c_off, M, bias_e, lane, scat, spos[mq][i]);
        } else if (ACT == ACT_SILU_MUL) {
          epi_silu_pair<false>(v[0], v[1], m, nb / 2, M, N / 2, C, ldc, vec, lane);
        } else if (rdma) {
          const int rl = m - m0, cl = nb - n0 + (lane >> 4) * 4;
          epi_pair_bf16<ACT, true>(v[0], v[1], m, nb, M, C, ldc, bias_e, R, ldr, lane, res_tile_read<TN>(smem, rl, cl),
                                   res_tile_read<TN>(smem, rl, cl + 16));
        } else if (rpre) {
          epi_pair_bf16<ACT, true>(v[0], v[1], m, nb, M, C, ldc, bias_e, R, ldr, lane, rr[mq][nq][i][0],
                                   rr[mq][nq][i][1]);
        } else if (pair && nb + 31 < N) {
          epi_pair_bf16<ACT>(v[0], v[1], m, nb, (gan & 8) ? 0 : M, C, ldc, bias_e, R, ldr, lane);
        } else {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            epi_t4<ACT, false>(v[j], m, nb + j * 16 + (lane >> 4) * 4, M, N, C, ldc, bias_e, R, ldr, vec);
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

// Large-GEMM tile selection: 0 = auto (256x256 when it still yields >= 256
// blocks), 128 / 256 force a tile (A/B benchmarking, tests).
static int g_gemm_tile = 0;

// Rows up to which every bf16 GEMM streams its weights on the skinny kernels
// (A/B switch).  At M = 64 a wide-N head with warm weights runs faster on the
// 128^2 MFMA tiles (GPT-2 50304 x 768: 28.3 -> 22.5 us, x 1600: 52.7 -> 33.6,
// profiles/archive/r2_head_probe.jsonl), but inside the decode step (weights cold behind
// 1.27 GB of K/V) GPT-2 B=64 ran 0.588 -> 0.603 ms/step that way and GPT-2 XL
// B=64 4.507 -> 4.493 (profiles/archive/r2_decode_ab_skinny_max_m.jsonl): 64 stays.
static int g_skinny_max_m = 64;

extern "C" int dnn_gemm_set_skinny_max_m(int m) {
  if (m < 0 || m > 64) return -1;
  g_skinny_max_m = m;
  return 0;
}

// 256^2 epilogue: residual rows loaded ahead of the outputs (1) or per output row group (0)
static int g_res_prefetch = 1;

extern "C" int dnn_gemm_set_res_prefetch(int on) {
  g_res_prefetch = on ? 1 : 0;
  return 0;
}

extern "C" int dnn_gemm_set_anatomy(int bits) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_anatomy), &bits, sizeof(int));
}

extern "C" int dnn_gemm_set_tile(int tile) {
  if (tile != 0 && tile != 128 && tile != 256 && tile != 255) return -1;  // 255: force 256x128
  g_gemm_tile = tile;
  return 0;
}

// Relative time of one 256x128 tile against one 256x256 tile (the auto rule
// picks 256x128 when ceil(tiles/256) x this beats the 256^2 rounds).  Off by
// default (measured, profiles/r4_gemm_tiles*.jsonl): at M = 32768 the 256x128
// tiles ran N=768 K=768 752 -> 672 TF/s, K=3072 1052 -> 1070, N=2304 885 ->
// 768, and the GPT-2 4-stage prefill 3.85 -> 3.76 M tok/s — the 2-phase
// schedule, one K-tile ahead, loses more per tile than the full last round
// saves; tile 255 keeps it selectable.
// the 256^2 + 256x128 tail split (A/B switch, a bit mask: 1 the bf16 kernel, 2 the fp8 one; DNN_SPLIT_TAIL
// sets the start value).  fp8 is off by default: GPT-2 XL prefill 259.5 -> 257.4 k tok/s with it
// (profiles/r4_prefill_ab_tail_split_gpt2xl.jsonl), bf16 GPT-2 +1.6 %
static int g_split_tail = [] {
  const char* e = getenv("DNN_SPLIT_TAIL");
  return e != nullptr ? atoi(e) : 1;
}();
extern "C" int dnn_gemm_set_split_tail(int on) {
  g_split_tail = on;
  return 0;
}

// Tail split rule: the columns of the 256^2 part (a multiple of 256), or 0.
// Applies when the 256^2 grid is whole rounds of 256 tiles plus one last
// column of tiles (1..256 columns wide) that fits one more round as 256x128
// tiles: GPT-2 (N 768 / 2304) and GPT-2 XL (N 1600 / 4800 / 6400) at M = 32768.
static int tail_split_cols(int M, int N, bool fp8 = false) {
  // fp8: bit 2 every tail, bit 4 only tails of >= 128 columns (GPT-2 XL c_attn / c_fc, not the 64-column
  // tail of the 1600-wide O / c_proj)
  if (!(g_split_tail & (fp8 ? 6 : 1)) || g_gemm_tile != 0) return 0;
  const int ntm = (M + 255) / 256, ntn = (N + 255) / 256;
  if (ntn < 2 || (ntm * (ntn - 1)) % 256 != 0) return 0;
  const int Na = (ntn - 1) * 256;
  if (fp8 && !(g_split_tail & 2) && N - Na < 128) return 0;
  if (ntm * ((N - Na + 127) / 128) > 256) return 0;
  return Na;
}

static float g_half_cost = 1e9f;
extern "C" int dnn_gemm_set_half_cost(float c) {
  if (!(c > 0.f)) return -1;
  g_half_cost = c;
  return 0;
}

template <int ACT, bool F32>
static void launch_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                        const void* R, int ldr, int M, int N, int K, hipStream_t st, const void* Wsh,
                        const float2* rowstat, const float* colsum, void* ws, long long ws_bytes) {
  // decode-sized: the weight-streaming skinny kernels (gemm_skinny.hip); medium
  // M (<= 256) too while the 128^2 tiles would not fill 3/4 of the CUs (same
  // rule as ops/gemm.py skinny_rows)
  // (a folded-norm GEMM (rowstat) always takes the tile kernels: the skinny
  // path folds its norm itself, dnn_gemm_skinny_norm)
  if (rowstat == nullptr &&
      (M <= g_skinny_max_m || (M <= 256 && ((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N) < 192))) {
    dnn_gemm_skinny(A, lda, nullptr, W, ldw, nullptr, C, ldc, bias, R, ldr, M, N, K, ACT, F32 ? 1 : 0, 0, st, Wsh, ws,
                    ws_bytes);
    return;
  }
  // Auto choice by wave quantisation: the 256^2 kernel runs 1 block/CU (256
  // slots) and is ~1.3x the 128^2 kernel (2 blocks/CU, 512 slots) per slot
  // when both fill the chip; 1.4 also sends M=32768 N=768 (1.5 waves of 256^2
  // tiles) to the 256^2 kernel, 6 % faster at K=3072 and equal at K=768
  // (profiles/archive/r1_gemm_bench_v2_widened_epilogue.jsonl).
  const int tiles256 = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  const int tiles128 = ((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N);
  auto fill = [](int tiles, int slots) {
    const int waves = (tiles + slots - 1) / slots;
    return (double)tiles / ((double)waves * slots);
  };
  const bool big = g_gemm_tile == 256 || g_gemm_tile == 255 ||
                   (g_gemm_tile == 0 && M >= 256 && N >= 256 && 1.4 * fill(tiles256, 256) > fill(tiles128, 512));
  const int tilesH = ((M + BG_M - 1) / BG_M) * ((N + 127) / 128);
  const bool half = g_gemm_tile == 255 ||
                    (big && g_gemm_tile == 0 && (float)((tilesH + 255) / 256) * g_half_cost < (float)((tiles256 + 255) / 256));
  if (half) {
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT, F32, false, 1>), dim3(tilesH), dim3(512), 0, st, (const bf16_t*)A,
                       lda, (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, K, g_res_prefetch,
                       rowstat, colsum);
    return;
  }
  // Tail split (round 4): when the 256^2 grid is full rounds plus a last
  // column of tiles that fills at most one more round as 256x128 tiles (GPT-2's
  // 768-wide O / c_proj at M = 32768: 256 tiles + a 128-tile column), the
  // first N - 256 columns run as 256^2 tiles and the last 256 as 256x128 tiles
  // in a second launch — 1 + 1/2 rounds instead of 2 full ones, no workspace
  // and no reduction (the two launches write disjoint columns).
  const int ntm256 = (M + BG_M - 1) / BG_M;
  const int Na = (big && ACT != ACT_SILU_MUL) ? tail_split_cols(M, N) : 0;
  if (Na > 0) {
    const int Nt = N - Na;
    const size_t cb = F32 ? sizeof(float) : sizeof(bf16_t);
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT, F32>), dim3(ntm256 * (Na / 256)), dim3(512), 0, st,
                       (const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, Na, K,
                       g_res_prefetch, rowstat, colsum);
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT, F32, false, 1>), dim3(ntm256 * ((Nt + 127) / 128)), dim3(512), 0,
                       st, (const bf16_t*)A, lda, (const bf16_t*)W + (size_t)Na * ldw, ldw,
                       (void*)((char*)C + (size_t)Na * cb), ldc, bias != nullptr ? bias + Na : nullptr,
                       R != nullptr ? (const bf16_t*)R + Na : nullptr, ldr, M, Nt, K, g_res_prefetch, rowstat,
                       colsum != nullptr ? colsum + Na : nullptr);
    return;
  }
  if (big) {
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT, F32>), dim3(tiles256), dim3(512), 0, st, (const bf16_t*)A, lda,
                       (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, K, g_res_prefetch, rowstat,
                       colsum);
    return;
  }
  hipLaunchKernelGGL((gemm_bf16_tn_kernel<ACT, F32>), dim3(tiles128), dim3(256), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)W, ldw, C, ldc, bias, (const bf16_t*)R, ldr, M, N, K, rowstat, colsum);
}

// rowstat (M float2 {rstd, -mean rstd}) / colsum (N floats, LayerNorm only):
// folded pre-norm epilogue, v = rstd acc - mean rstd colsum, before bias / act /
// residual (ops/gemm.py linear_norm at prefill sizes); nullptr = plain GEMM.
extern "C" int dnn_gemm_bf16(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                             const void* R, int ldr, int M, int N, int K, int act, int out_f32, hipStream_t st,
                             const void* Wsh, const float* rowstat, const float* colsum, void* ws,
                             long long ws_bytes) {
  if (K % 64 != 0 || M <= 0 || N <= 0) return -1;
  if (colsum != nullptr && rowstat == nullptr) return -1;
  const float2* rs = reinterpret_cast<const float2*>(rowstat);
#define DISPATCH(a)                                                                                  \
  if (act == a) {                                                                                    \
    if (out_f32) launch_gemm<a, true>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, st, Wsh, rs, colsum, ws, ws_bytes); \
    else launch_gemm<a, false>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, st, Wsh, rs, colsum, ws, ws_bytes);        \
    return (int)hipGetLastError();                                                                   \
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

// Prefill c_attn with the QKV scatter epilogue (gemm_bf16_256_kernel SCATTER):
// y = x W^T + bias (folded pre-norm when rowstat) written head-major: q ->
// (B, H, T, hd), k / v -> the (B, Hkv, S, hd) caches at rows pos[b] + t.  M =
// B*T.  Returns -3 when the shape does not fit the 256^2 path (the caller then
// uses the qkv row output + qkv_split).
extern "C" int dnn_gemm_bf16_qkv_scatter(const void* A, int lda, const void* W, int ldw, const float* bias,
                                         const float* rowstat, const float* colsum, void* q, void* kc, void* vc,
                                         const int* pos, int B, int T, int H, int Hkv, int hd, int S, int K,
                                         hipStream_t st) {
  const int M = B * T, N = (H + 2 * Hkv) * hd;
  if (K % 64 != 0 || M <= 0 || hd % 8 != 0 || (colsum != nullptr && rowstat == nullptr)) return -1;
  if (N % 32 != 0 || M < 256 || ((uintptr_t)bias & 15) != 0) return -3;
  const int tiles = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  if ((hd & (hd - 1)) != 0 || M >= (1 << 24)) return -3;
  QkvScatter sc{(bf16_t*)q, (bf16_t*)kc, (bf16_t*)vc, pos, T, H, Hkv, __builtin_ctz(hd), S, 1.0f / (float)T};
  // tail split as launch_gemm's (GPT-2 c_attn at M = 32768: 1024 + 128 tiles
  // -> 4 rounds of 256^2 + 1 round of 256x128); the bias is indexed by the
  // global column (c_off), the folded norm's colsum by the launch's own
  const int ntm256 = (M + BG_M - 1) / BG_M;
  const int Na = tail_split_cols(M, N);
  if (Na > 0) {
    const int Nt = N - Na;
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT_NONE, false, true>), dim3(ntm256 * (Na / 256)), dim3(512), 0, st,
                       (const bf16_t*)A, lda, (const bf16_t*)W, ldw, q, hd, bias, (const bf16_t*)nullptr, 0, M, Na, K,
                       0, reinterpret_cast<const float2*>(rowstat), colsum, sc);
    QkvScatter tail = sc;
    tail.c_off = Na;
    hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT_NONE, false, true, 1>), dim3(ntm256 * ((Nt + 127) / 128)),
                       dim3(512), 0, st, (const bf16_t*)A, lda, (const bf16_t*)W + (size_t)Na * ldw, ldw, q, hd, bias,
                       (const bf16_t*)nullptr, 0, M, Nt, K, 0, reinterpret_cast<const float2*>(rowstat),
                       colsum != nullptr ? colsum + Na : nullptr, tail);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_bf16_256_kernel<ACT_NONE, false, true>), dim3(tiles), dim3(512), 0, st, (const bf16_t*)A,
                     lda, (const bf16_t*)W, ldw, q, hd, bias, (const bf16_t*)nullptr, 0, M, N, K, 0,
                     reinterpret_cast<const float2*>(rowstat), colsum, sc);
  return (int)hipGetLastError();
}

// fp8 (W8A8) c_attn with the QKV scatter epilogue: A8 / sa the per-token
// e4m3 activations (layernorm_q8), W8 / sw the e4m3 weight, Kb its row bytes.
extern "C" int dnn_gemm_fp8_qkv_scatter(const void* A8, const float* sa, const void* W8, const float* sw,
                                        const float* bias, void* q, void* kc, void* vc, const int* pos, int B, int T,
                                        int H, int Hkv, int hd, int S, int Kb, hipStream_t st) {
  const int M = B * T, N = (H + 2 * Hkv) * hd;
  if (Kb % 128 != 0 || M <= 0 || hd % 8 != 0 || sa == nullptr || sw == nullptr) return -1;
  if (N % 32 != 0 || M < 256 || ((uintptr_t)bias & 15) != 0) return -3;
  const int tiles = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  if ((hd & (hd - 1)) != 0 || M >= (1 << 24)) return -3;
  QkvScatter sc{(bf16_t*)q, (bf16_t*)kc, (bf16_t*)vc, pos, T, H, Hkv, __builtin_ctz(hd), S, 1.0f / (float)T};
  const int Na = tail_split_cols(M, N, true);  // GPT-2 XL c_attn (N = 4800): 2304 + 256 half tiles
  if (Na > 0) {
    const int ntm256 = (M + BG_M - 1) / BG_M, Nt = N - Na;
    hipLaunchKernelGGL((gemm_fp8_256_kernel<ACT_NONE, true>), dim3(ntm256 * (Na / 256)), dim3(512), 0, st,
                       (const uint8_t*)A8, sa, (const uint8_t*)W8, sw, (bf16_t*)q, hd, bias, (const bf16_t*)nullptr, 0,
                       M, Na, Kb, sc);
    QkvScatter tail = sc;
    tail.c_off = Na;
    hipLaunchKernelGGL((gemm_fp8_256_kernel<ACT_NONE, true, 1>), dim3(ntm256 * ((Nt + 127) / 128)), dim3(512), 0,
                       st, (const uint8_t*)A8, sa, (const uint8_t*)W8 + (size_t)Na * Kb, sw + Na, (bf16_t*)q, hd, bias,
                       (const bf16_t*)nullptr, 0, M, Nt, Kb, tail);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_fp8_256_kernel<ACT_NONE, true>), dim3(tiles), dim3(512), 0, st, (const uint8_t*)A8, sa,
                     (const uint8_t*)W8, sw, (bf16_t*)q, hd, bias, (const bf16_t*)nullptr, 0, M, N, Kb, sc);
  return (int)hipGetLastError();
}

// fp8 256^2 GEMM (see gemm_fp8_256_kernel); Kb = row bytes of A and W (multiple
// of 128), sa per-row, sw per-column scales.  Called by dnn_gemm_fp8 when the
// 256^2 tiles fill the chip.
extern "C" int dnn_gemm_fp8_256(const void* A, const float* sa, const void* W, const float* sw, void* C, int ldc,
                                const float* bias, const void* R, int ldr, int M, int N, int Kb, int act,
                                hipStream_t st) {
  if (Kb % 128 != 0 || M <= 0 || N <= 0 || sa == nullptr || sw == nullptr) return -1;
  if (act == ACT_SILU_MUL && N % 16 != 0) return -1;
  const int tiles = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  // tail split (as launch_gemm's): GPT-2 XL O / c_proj (N = 1600) and c_fc (N = 6400) at M = 32768
  const int Na = act != ACT_SILU_MUL ? tail_split_cols(M, N, true) : 0;
  const int ntm256 = (M + BG_M - 1) / BG_M, Nt = N - Na;
#define F8L(a)                                                                                                    \
  if (act == a) {                                                                                                 \
    if (Na > 0) {                                                                                                 \
      hipLaunchKernelGGL((gemm_fp8_256_kernel<a>), dim3(ntm256 * (Na / 256)), dim3(512), 0, st,                   \
                         (const uint8_t*)A, sa, (const uint8_t*)W, sw, (bf16_t*)C, ldc, bias, (const bf16_t*)R,    \
                         ldr, M, Na, Kb);                                                                         \
      hipLaunchKernelGGL((gemm_fp8_256_kernel<a, false, 1>), dim3(ntm256 * ((Nt + 127) / 128)), dim3(512), 0, st, \
                         (const uint8_t*)A, sa, (const uint8_t*)W + (size_t)Na * Kb, sw + Na, (bf16_t*)C + Na,    \
                         ldc, bias != nullptr ? bias + Na : nullptr,                                              \
                         R != nullptr ? (const bf16_t*)R + Na : nullptr, ldr, M, Nt, Kb);                         \
      return (int)hipGetLastError();                                                                              \
    }                                                                                                             \
    hipLaunchKernelGGL((gemm_fp8_256_kernel<a>), dim3(tiles), dim3(512), 0, st, (const uint8_t*)A, sa,            \
                       (const uint8_t*)W, sw, (bf16_t*)C, ldc, bias, (const bf16_t*)R, ldr, M, N, Kb);            \
    return (int)hipGetLastError();                                                                                \
  }
  F8L(ACT_NONE) F8L(ACT_RELU) F8L(ACT_GELU) F8L(ACT_SILU_MUL)
#undef F8L
  return -2;
}

// MX-scaled W8A8 GEMM on the 256^2 kernel: A8 [M][Kb]
// e4m3 with e8m0 scales sx per (row, 128-column K-tile) (common.h mx_index;
// dnn_quant_fp8_mx / dnn_layernorm_q8_mx / a QOUT epilogue write them), W8 /
// sw per-channel e4m3.  qo != nullptr (act GELU): the output is quantised in
// the epilogue instead (QOUT: qo [M][ldq] e4m3 with scales sxo, kpo columns,
// the next GEMM's MX input) and C is not written.  -3: not a 256^2 shape (the
// caller keeps the per-row path).
extern "C" int dnn_gemm_fp8_mx(const void* A8, const void* sx, const void* W8, const float* sw, void* C, int ldc,
                               const float* bias, const void* R, int ldr, int M, int N, int Kb, int act, void* qo,
                               int ldq, void* sxo, int kpo, hipStream_t st) {
  if (Kb % 128 != 0 || M <= 0 || N <= 0 || sx == nullptr || sw == nullptr) return -1;
  if (M < 256 || N < 256) return -3;
  if (qo != nullptr && (act != ACT_GELU || sxo == nullptr || kpo % 128 != 0 || kpo < N || ldq < kpo ||
                        (ldq & 7) != 0 || ((uintptr_t)qo & 7) != 0))
    return -1;
  if (act == ACT_SILU_MUL && N % 16 != 0) return -1;
  const int tiles = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  const uint32_t* sxw = reinterpret_cast<const uint32_t*>(sx);
  if (qo != nullptr) {
    hipLaunchKernelGGL((gemm_fp8_256_kernel<ACT_GELU, false, 2, true, true>), dim3(tiles), dim3(512), 0, st,
                       (const uint8_t*)A8, (const float*)nullptr, (const uint8_t*)W8, sw, (bf16_t*)nullptr, 0, bias,
                       (const bf16_t*)nullptr, 0, M, N, Kb, QkvScatter{}, sxw, (uint8_t*)qo, ldq, (uint8_t*)sxo, kpo);
    return (int)hipGetLastError();
  }
#define F8M(a)                                                                                                      \
  if (act == a) {                                                                                                   \
    hipLaunchKernelGGL((gemm_fp8_256_kernel<a, false, 2, true>), dim3(tiles), dim3(512), 0, st, (const uint8_t*)A8, \
                       (const float*)nullptr, (const uint8_t*)W8, sw, (bf16_t*)C, ldc, bias, (const bf16_t*)R, ldr, M, \
                       N, Kb, QkvScatter{}, sxw);                                                                   \
    return (int)hipGetLastError();                                                                                  \
  }
  F8M(ACT_NONE) F8M(ACT_RELU) F8M(ACT_GELU) F8M(ACT_SILU_MUL)
#undef F8M
  return -2;
}

// fp8 c_attn with the QKV scatter epilogue on MX-scaled activations
// (dnn_layernorm_q8_mx): as dnn_gemm_fp8_qkv_scatter, sx instead of sa.
extern "C" int dnn_gemm_fp8_qkv_scatter_mx(const void* A8, const void* sx, const void* W8, const float* sw,
                                           const float* bias, void* q, void* kc, void* vc, const int* pos, int B, int T,
                                           int H, int Hkv, int hd, int S, int Kb, hipStream_t st) {
  const int M = B * T, N = (H + 2 * Hkv) * hd;
  if (Kb % 128 != 0 || M <= 0 || hd % 8 != 0 || sx == nullptr || sw == nullptr) return -1;
  if (N % 32 != 0 || M < 256 || N < 256 || ((uintptr_t)bias & 15) != 0) return -3;
  if ((hd & (hd - 1)) != 0 || M >= (1 << 24)) return -3;
  QkvScatter sc{(bf16_t*)q, (bf16_t*)kc, (bf16_t*)vc, pos, T, H, Hkv, __builtin_ctz(hd), S, 1.0f / (float)T};
  const int tiles = ((M + BG_M - 1) / BG_M) * ((N + BG_N - 1) / BG_N);
  hipLaunchKernelGGL((gemm_fp8_256_kernel<ACT_NONE, true, 2, true>), dim3(tiles), dim3(512), 0, st, (const uint8_t*)A8,
                     (const float*)nullptr, (const uint8_t*)W8, sw, (bf16_t*)q, hd, bias, (const bf16_t*)nullptr, 0, M,
                     N, Kb, sc, reinterpret_cast<const uint32_t*>(sx));
  return (int)hipGetLastError();
}
