// CIFAR-10 ConvNet stage kernels for gfx950, bf16 compute (the fp32-accurate
// path of the reference precision is cifar_x3.hip).
//
// Stage 0 (reference ModelPart0_2Node, cifar_model_parts.py:37-42):
//   conv1(3->32,3x3,p1)+bias+ReLU+maxpool2 -> conv2(32->64,3x3,p1)+bias+ReLU+maxpool2
//   -> flatten in NCHW order (c*64 + h*8 + w), ONE persistent kernel
//   (cifar_stage0_v4_kernel), bf16 output (B,4096).  Both convolutions are
//   implicit GEMMs on v_mfma_f32_32x32x16_bf16; the 32-row M tile is a 4x8
//   pixel block so that the 2x2 max-pool is done inside each lane's
//   accumulator registers (C/D row = (g&3) + 8*(g>>2) + 4*(lane>>5)).  conv2's
//   B operand (64x288 weights) stays resident in VGPRs for the whole
//   persistent loop (one 32-channel N-tile per wave = 72 VGPRs).
//
// Stage 1 tail (reference ModelPart1_2Node, cifar_model_parts.py:53-58, plus the
// host-side argmax of node.py:61/190, done per row here): after fc1+bias+ReLU
// (gemm_bf16 with ACT_RELU), fc2(512->10)+bias+softmax+argmax on MFMA, 16 rows
// per wave-iteration.
#include "common.h"

namespace dnn {


// fc2 (512->10) + bias + softmax + argmax. hid: (B,512) bf16 (fc1+ReLU output).
// One wave handles 16 rows per iteration with mfma_f32_16x16x32_bf16:
// A = hid rows (lane: row l&15, k 8*(l>>4)+j), B = W2 padded to 16 classes held
// in VGPRs. Softmax across each 16-lane row group with xor-shuffles.
__global__ __launch_bounds__(256) void cifar_head_tail_kernel(const bf16_t* __restrict__ hid, const bf16_t* __restrict__ w2p,
                                                              const float* __restrict__ b2, float* __restrict__ probs,
                                                              int* __restrict__ pred, int B) {
  const int lane = threadIdx.x & 63;
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const int col = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 wf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wf[s] = *reinterpret_cast<const bf16x8*>(w2p + col * 512 + s * 32 + kq);
  const float bias = col < 10 ? b2[col] : 0.f;
  for (int r0 = gw * 16; r0 < B; r0 += nw * 16) {
    const int row = r0 + (lane & 15);
    const int rc = row < B ? row : B - 1;
    const bf16_t* ap = hid + (size_t)rc * 512 + kq;
    bf16x8 a[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = *reinterpret_cast<const bf16x8*>(ap + s * 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], wf[s], acc, 0, 0, 0);
    // acc[r] = logit(row = r0 + (lane>>4)*4 + r, class = col)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = col < 10 ? acc[r] + bias : -INFINITY;
      float mx = z;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float e = col < 10 ? __expf(z - mx) : 0.f;
      float sum = e;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
      // argmax: smallest class index attaining the max (numpy semantics)
      int cand = (z == mx) ? col : 16;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) cand = min(cand, __shfl_xor(cand, o, 64));
      const int m = r0 + (lane >> 4) * 4 + r;
      if (m < B) {
        if (col < 10) probs[(size_t)m * 10 + col] = e / sum;
        if (col == 0) pred[m] = cand;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Stage-0 LDS layouts (shared by the v4 kernel below):
//  * input staged as HWC4 bf16 [34][40][4] (3 channels + 1 zero): conv1's
//    im2col K = (ky, kx<4, c<4) = 48 (3 MFMA k-steps of 16, zero weights on
//    kx=3/c=3), so a lane's 8 A-values for a k-step are the 2 adjacent pixels
//    (x+2h, x+2h+1) x 4 channels = 2 x ds_read_b64 (vs 27 scalar reads in v1);
//    the 320-B row pitch puts the 4 rows of a 4x8 pixel block on disjoint banks.
//  * act1 = padded HWC [18][24 pitch][32 ch + 8 pad] bf16 (80-B pixels): every
//    ds_read_b128 A-fragment of conv2 is conflict-free without an XOR, so all
//    reads are lane_base + compile-time immediates (searched exhaustively over
//    the 4 lane groups x 9 taps x 4 chunks).
//  * conv1 epilogue: two quad DPP exchanges gather 4 channels of one pooled
//    pixel per lane -> one ds_write_b64 (vs 4 ds_write_b16).
//  * conv2 epilogue: the 2 horizontally adjacent pooled pixels are packed ->
//    ds_write_b32 into a 136-B-pitch staging image (2-way instead of 32-way).
// ---------------------------------------------------------------------------
constexpr int V2_XW = 40;                                     // input row pitch (pixels)
constexpr int V2_XIN_BYTES = 34 * V2_XW * 8;                  // 10880
constexpr int V2_A1_OFF = V2_XIN_BYTES;                       // 10880 (16-B aligned)
constexpr int V2_A1W = 24, V2_A1P = 80;                       // act1 pitch (pixels), pixel stride (bytes)
constexpr int V2_A1_BYTES = 18 * V2_A1W * V2_A1P;             // 34560
constexpr int V2_OB_OFF = V2_A1_OFF + V2_A1_BYTES;            // 45440
constexpr int V2_OBP = 136;                                   // obuf channel pitch (bytes)
constexpr int V2_LDS = V2_OB_OFF + 64 * V2_OBP;               // 54144

// conv2 main loop for one wave: 4 M-tiles (mt0..mt0+3) x 18 k-steps of 16.
// A fragments are software-pipelined one k-step ahead in registers and the
// issue order is pinned (4 ds_read_b128 of step s+1, then the 4 MFMAs of step
// s), so each MFMA's operand read is ~4 MFMAs (~128 cycles) old — enough to
// cover the LDS latency that hipcc's own schedule (read 1 ahead) exposed.
//
// hipcc keeps scheduling each operand read one MFMA ahead whatever the source
// order, so the reads are inline-asm ds_read_b128 (immediate offsets from one
// base VGPR) issued a whole k-step ahead, with counted lgkmcnt waits fenced by
// sched_barrier so no MFMA is hoisted above its wait (cdna_hip_programming.md
// §5.7 form iii, rule 18). The caller must have no other LDS op in flight.
template <int S, int I>
__device__ __forceinline__ constexpr int c2_off() {
  return ((4 * (I >> 1) + (S >> 1) / 3) * 24 + 8 * (I & 1) + (S >> 1) % 3) * 80 + (S & 1) * 32;
}

template <int S>
__device__ __forceinline__ void c2_issue(uint32_t base, bf16x8 (&a)[4]) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[0]) : "v"(base), "i"(c2_off<S, 0>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[1]) : "v"(base), "i"(c2_off<S, 1>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[2]) : "v"(base), "i"(c2_off<S, 2>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[3]) : "v"(base), "i"(c2_off<S, 3>()));
}

template <int S>
__device__ __forceinline__ void c2_step(uint32_t base, const bf16x8 (&w2f)[18], f32x16 (&acc)[4], bf16x8 (&cur)[4],
                                        bf16x8 (&nxt)[4]) {
  if constexpr (S + 1 < 18) {
    c2_issue<S + 1>(base, nxt);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // step S's 4 reads have landed
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[i], w2f[S], acc[i], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);  // keep step S+1's issue/wait below these MFMAs
  if constexpr (S + 1 < 18) c2_step<S + 1>(base, w2f, acc, nxt, cur);
}

__device__ __forceinline__ void conv2_mainloop(const char* a1lane, const bf16x8 (&w2f)[18], f32x16 (&acc)[4],
                                               int mt0) {
  // M tiles mt0..mt0+3 = tile rows ty2 = mt0/2 + (i>>1): fold mt0 into the base address
  const uint32_t base = (uint32_t)(uintptr_t)(a1lane + (mt0 >> 1) * 4 * 24 * 80);
  bf16x8 a0[4], a1[4];
  c2_issue<0>(base, a0);
  c2_step<0>(base, w2f, acc, a0, a1);
}

// Force the loads of loop-invariant registers to complete at this point (an
// empty asm that reads them makes hipcc place their s_waitcnt here).
template <int N>
__device__ __forceinline__ void resident_fence(const bf16x8 (&w)[N], float b) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(w[i]));
  asm volatile("" ::"v"(b));
}

__device__ __forceinline__ int dpp_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int dpp_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }


// ---------------------------------------------------------------------------
// Stage-0 pipeline design (v3, refined by v4 below): wave-specialised software pipeline (512 threads, 1 WG per CU).
// Waves 0-3 ("P") stage the input and run conv1 for image k+1 while waves 4-7
// ("C") run conv2 for image k, so every SIMD hosts one VALU/LDS-heavy wave and
// one MFMA-heavy wave at the same time (separate pipes; MI355X_MICROARCH
// "Execution model"). act1 and the output staging image are double-buffered;
// two workgroup barriers per image. Same LDS layouts and lane maps as v2.
//   iteration it:  A) P: input(it) regs -> xin         C: obuf[it-2] -> global
//                  B) P: conv1(it) -> act1[it&1]       C: conv2(it-1) -> obuf[(it-1)&1]
// ---------------------------------------------------------------------------
constexpr int V3_A1_OFF = V2_XIN_BYTES;                                  // 10880
constexpr int V3_OB_OFF = V3_A1_OFF + 2 * V2_A1_BYTES;                   // 80000
constexpr int V3_OB_BYTES = 64 * V2_OBP;                                 // 8704
constexpr int V3_LDS = V3_OB_OFF + 2 * V3_OB_BYTES;                      // 97408

// ---------------------------------------------------------------------------
// Stage 0, v4: v3 with ONE barrier per image.  v3's phase A (input regs -> xin,
// output staging -> global) ran on every wave with no MFMA in flight (~9 % of
// an image by the s_memtime stamps).  Here the input image is double-buffered
// in LDS, so producers stage image it+1 right after their conv1 tiles of image
// it, and consumers copy out image it-2 before their conv2 of image it-1:
//   iteration it:  P: conv1(it) [0,pt) <- xin[it&1];  regs(it+1) -> xin[(it+1)&1];  load regs(it+2)
//                  C: obuf[it&1] -> out[it-2];  conv2(it-1) -> obuf[(it-1)&1];  conv1(it) [pt,32)
//                  barrier
// Every LDS buffer is written and read in different iterations (separated by
// the barrier), or in disjoint halves of a double buffer within one.
// ---------------------------------------------------------------------------
constexpr int V4_XIN1_OFF = V3_LDS;                                      // second input buffer
constexpr int V4_LDS = V4_XIN1_OFF + V2_XIN_BYTES;                       // 108288

__global__ __launch_bounds__(512, 1) void cifar_stage0_v4_kernel(
    const float* __restrict__ x, bf16_t* __restrict__ out, const bf16_t* __restrict__ w1p,
    const float* __restrict__ b1, const bf16_t* __restrict__ w2p, const float* __restrict__ b2, int B, int PT) {
  __shared__ __attribute__((aligned(16))) char smem[V4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave < 4;
  const int rw = wave & 3;
  const int rt = tid & 255;
  const int h = lane >> 5, r32 = lane & 31;
  const int n = B > (int)blockIdx.x ? (B - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;

  for (int i = tid; i < V3_OB_OFF / 16; i += 512) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < V2_XIN_BYTES / 16; i += 512)
    reinterpret_cast<uint4*>(smem + V4_XIN1_OFF)[i] = make_uint4(0, 0, 0, 0);

  bf16x8 w1f[3];
  bf16x8 w2f[18];
#pragma unroll
  for (int s = 0; s < 3; ++s) w1f[s] = *reinterpret_cast<const bf16x8*>(w1p + r32 * 48 + s * 16 + h * 8);
  const float bias1 = b1[r32];
  float bias = 0.f;
  int oc2 = 0;
  if (!producer) {
    oc2 = (rw & 1) * 32 + r32;
#pragma unroll
    for (int s = 0; s < 18; ++s) w2f[s] = *reinterpret_cast<const bf16x8*>(w2p + oc2 * 288 + s * 16 + h * 8);
    bias = b2[oc2];
  }
  resident_fence(w1f, bias1);
  if (!producer) resident_fence(w2f, bias);
  float pf[4][3];
  auto load_img = [&](int k) {
    const float* xb = x + (size_t)(blockIdx.x + (size_t)k * gridDim.x) * 3072;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) pf[i][c] = xb[c * 1024 + rt + 256 * i];
  };
  auto stage_img = [&](char* xin) {  // prefetch registers -> padded HWC4 bf16 image
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = rt + 256 * i, yy = p >> 5, xx = p & 31;
      uint2 v;
      v.x = pack2bf(pf[i][0], pf[i][1]);
      v.y = pack2bf(pf[i][2], 0.f);
      *reinterpret_cast<uint2*>(xin + ((yy + 1) * V2_XW + xx + 1) * 8) = v;
    }
  };
  auto xin_of = [&](int k) { return smem + ((k & 1) ? V4_XIN1_OFF : 0); };
  __syncthreads();  // halos zeroed before any image is staged
  if (producer && n > 0) {
    load_img(0);
    stage_img(xin_of(0));
    if (n > 1) load_img(1);
  }
  __syncthreads();

  const int c1_lane = ((r32 >> 3) * V2_XW + (r32 & 7) + 2 * h) * 8;
  const int c2_lane = ((r32 >> 3) * V2_A1W + (r32 & 7)) * V2_A1P + h * 16;
  const int q = ((r32 & 1) ? 2 : 0) + ((r32 & 2) ? 1 : 0);
  const int cb = r32 & ~3;

  // bias + ReLU + 2x2 max-pool in registers, quad-DPP gather of 4 channels of
  // one pooled pixel per lane, one 8-B store into act1
  auto conv1_epi = [&](int t, const f32x16& acc, char* a1) {
    const int ty = t >> 2, tx = t & 3;
    float v[4];
#pragma unroll
    for (int qy = 0; qy < 2; ++qy)
#pragma unroll
      for (int qx = 0; qx < 2; ++qx) {
        const int g0 = (2 * qy) * 4 + 2 * qx;
        v[qy * 2 + qx] = fmaxf(fmax_nan(fmax_nan(acc[g0], acc[g0 + 1]), fmax_nan(acc[g0 + 4], acc[g0 + 5])) + bias1, 0.f);
      }
    const bool odd = r32 & 1;
    const int s0 = __float_as_int(odd ? v[0] : v[2]), s1 = __float_as_int(odd ? v[1] : v[3]);
    const float r0 = __int_as_float(dpp_xor1(s0)), r1 = __int_as_float(dpp_xor1(s1));
    uint32_t u0, u1;
    if (!odd) { u0 = pack2bf(v[0], r0); u1 = pack2bf(v[1], r1); }
    else { u0 = pack2bf(r0, v[2]); u1 = pack2bf(r1, v[3]); }
    const bool hi2 = r32 & 2;
    const uint32_t rcv = (uint32_t)dpp_xor2((int)(hi2 ? u0 : u1));
    const uint32_t mine = hi2 ? u1 : u0;
    uint2 w;
    w.x = hi2 ? rcv : mine;
    w.y = hi2 ? mine : rcv;
    const int Y = 2 * ty + (q >> 1) + 1, X = 4 * tx + 2 * h + (q & 1) + 1;
    *reinterpret_cast<uint2*>(a1 + (Y * V2_A1W + X) * V2_A1P + cb * 2) = w;
  };
  auto conv1_tile = [&](int t, const char* xin, char* a1) {
    const char* abase = xin + c1_lane + ((4 * (t >> 2)) * V2_XW + 8 * (t & 3)) * 8;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const uint2 lo = *reinterpret_cast<const uint2*>(abase + s * V2_XW * 8);
      const uint2 hi = *reinterpret_cast<const uint2*>(abase + s * V2_XW * 8 + 8);
      const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w1f[s], acc, 0, 0, 0);
    }
    conv1_epi(t, acc, a1);
  };
  // two conv1 tiles at once: all 12 A-fragment reads issued up front and the two
  // accumulation chains interleaved, so one LDS latency and the MFMA result
  // latency of one tile hide under the other's work (the producer wave shares
  // its SIMD with a consumer wave; its stalls are the consumer's MFMA gaps)
  auto conv1_pair = [&](int ta, int tb, const char* xin, char* a1) {
    const char* pa = xin + c1_lane + ((4 * (ta >> 2)) * V2_XW + 8 * (ta & 3)) * 8;
    const char* pb = xin + c1_lane + ((4 * (tb >> 2)) * V2_XW + 8 * (tb & 3)) * 8;
    bf16x8 fa[3], fb[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const uint2 lo = *reinterpret_cast<const uint2*>(pa + s * V2_XW * 8);
      const uint2 hi = *reinterpret_cast<const uint2*>(pa + s * V2_XW * 8 + 8);
      fa[s] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      const uint2 lo2 = *reinterpret_cast<const uint2*>(pb + s * V2_XW * 8);
      const uint2 hi2 = *reinterpret_cast<const uint2*>(pb + s * V2_XW * 8 + 8);
      fb[s] = __builtin_bit_cast(bf16x8, make_uint4(lo2.x, lo2.y, hi2.x, hi2.y));
    }
    f32x16 acca = {}, accb = {};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      acca = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s], w1f[s], acca, 0, 0, 0);
      accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[s], w1f[s], accb, 0, 0, 0);
    }
    conv1_epi(ta, acca, a1);
    conv1_epi(tb, accb, a1);
  };
  auto copy_out = [&](int k) {  // obuf[k&1] (64 channel rows x 128 B) -> out image k, coalesced 16-B stores
    int4* dst = reinterpret_cast<int4*>(out + (size_t)(blockIdx.x + (size_t)k * gridDim.x) * 4096);
    const char* ob = smem + V3_OB_OFF + (k & 1) * V3_OB_BYTES;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = rt + 256 * u, ch = e >> 3, j = e & 7;
      const uint2 a = *reinterpret_cast<const uint2*>(ob + ch * V2_OBP + j * 16);
      const uint2 b = *reinterpret_cast<const uint2*>(ob + ch * V2_OBP + j * 16 + 8);
      dst[e] = make_int4((int)a.x, (int)a.y, (int)b.x, (int)b.y);
    }
  };

  for (int it = 0; it <= n; ++it) {
    if (producer) {
      if (it < n) {
        char* a1 = smem + V3_A1_OFF + (it & 1) * V2_A1_BYTES;
        const char* xin = xin_of(it);
        int t = rw;
        for (; t + 4 < PT; t += 8) conv1_pair(t, t + 4, xin, a1);
        if (t < PT) conv1_tile(t, xin, a1);
        if (it + 1 < n) {
          stage_img(xin_of(it + 1));
          if (it + 2 < n) load_img(it + 2);
        }
      }
    } else {
      if (it >= 2) copy_out(it - 2);
      if (it >= 1) {
        const int k = it - 1;
        const char* a1 = smem + V3_A1_OFF + (k & 1) * V2_A1_BYTES + c2_lane;
        char* ob = smem + V3_OB_OFF + (k & 1) * V3_OB_BYTES;
        f32x16 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = f32x16{};
        const int mt0 = (rw >> 1) * 4;
        conv2_mainloop(a1, w2f, acc, mt0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t2 = mt0 + i, ty2 = t2 >> 1, tx2 = t2 & 1;
#pragma unroll
          for (int qy = 0; qy < 2; ++qy) {
            float pv[2];
#pragma unroll
            for (int qx = 0; qx < 2; ++qx) {
              const int g0 = (2 * qy) * 4 + 2 * qx;
              pv[qx] = fmaxf(fmax_nan(fmax_nan(acc[i][g0], acc[i][g0 + 1]), fmax_nan(acc[i][g0 + 4], acc[i][g0 + 5])) + bias,
                             0.f);
            }
            const int PY = 2 * ty2 + qy, PX = 4 * tx2 + 2 * h;
            *reinterpret_cast<uint32_t*>(ob + oc2 * V2_OBP + (PY * 8 + PX) * 2) = pack2bf(pv[0], pv[1]);
          }
        }
      }
      if (it < n) {
        char* a1w = smem + V3_A1_OFF + (it & 1) * V2_A1_BYTES;
        const char* xin = xin_of(it);
        for (int t = PT + rw; t < 32; t += 4) conv1_tile(t, xin, a1w);
      }
    }
    __syncthreads();
  }
  if (!producer && n >= 1) copy_out(n - 1);
}

}  // namespace dnn

using namespace dnn;


static int g_v4_pt = 32;  // A/B-fitted: producers run all conv1 tiles (paired), consumers only conv2

extern "C" int dnn_cifar_stage0_v4(const float* x, void* out, const void* w1p, const float* b1, const void* w2p,
                                   const float* b2, int B, int grid, hipStream_t st) {
  if (B <= 0) return 0;
  if (grid <= 0) grid = 256;
  if (grid > B) grid = B;
  hipLaunchKernelGGL(cifar_stage0_v4_kernel, dim3(grid), dim3(512), 0, st, x, (bf16_t*)out, (const bf16_t*)w1p, b1,
                     (const bf16_t*)w2p, b2, B, g_v4_pt);
  return (int)hipGetLastError();
}

extern "C" int dnn_cifar_set_v4_pt(int pt) {
  if (pt < 0 || pt > 32 || pt % 4 != 0) return -1;
  g_v4_pt = pt;
  return 0;
}


extern "C" int dnn_cifar_head_tail(const void* hid, const void* w2p, const float* b2, float* probs, int* pred, int B,
                                   hipStream_t st) {
  if (B <= 0) return 0;
  int waves = (B + 15) / 16;
  int blocks = (waves + 3) / 4;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(cifar_head_tail_kernel, dim3(blocks), dim3(256), 0, st, (const bf16_t*)hid, (const bf16_t*)w2p,
                     b2, probs, pred, B);
  return (int)hipGetLastError();
}
