// CIFAR-10 ConvNet at the reference's fp32 precision on bf16 MFMA ("bf16x3").
//
// The reference computes and ships fp32 (cifar_model_parts.py:7-26,
// node.py:45-48).  gfx950 has f32-input MFMA, but at 1/16 of the bf16 rate
// (cdna_hip_programming.md §3 "FP32-input MFMA"), so every fp32 operand here
// is split into two bf16 terms, x = hi + lo with hi = bf16(x), lo = bf16(x - hi)
// (|x - hi - lo| <= 2^-17 |x|), and each product is accumulated in fp32 as
//     a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi        (a_lo*b_lo < 2^-16 |ab| dropped)
// = 3 bf16 MFMAs per fp32 product: 5.3x the f32-MFMA rate at ~2^-16 relative
// error per product before fp32 accumulation.
//
// Kernels:
//  * cifar_stage0_x3_kernel: conv1+bias+ReLU+pool -> conv2+bias+ReLU+pool ->
//    NCHW flatten, fp32 in, fp32 (B,4096) out (reference ModelPart0_2Node,
//    cifar_model_parts.py:37-42).  Persistent, 512 threads: waves 0-3
//    ("producers") stage input image it+1 and run conv1 of image it, waves 4-7
//    ("consumers") run conv2 of image it-1, one barrier per image, so each SIMD
//    pairs a VALU/LDS-heavy wave with an MFMA-heavy one.  Per image: 32 conv1
//    tiles x 3 k-steps x 3 terms + 16 conv2 tiles x 18 k-steps x 3 terms = 1152
//    v_mfma_f32_32x32x16_bf16.  LDS (126,464 B): input double-buffered as
//    hi/lo HWC4 planes [34][40][4] (pitch 40: conflict-free conv1 b64 reads),
//    pooled conv1 map double-buffered as hi/lo planes [18][18][32] with the
//    16-B chunk XORed by (Y & 3), which makes every conv2 ds_read_b128 fragment
//    (four 16-lane groups) conflict-free; conv2 results leave straight from
//    the accumulators as 8-B fp32 stores (no LDS staging).
//  * cifar_fc1_x3_kernel: fc1 + bias + ReLU on the fp32 boundary tensor, the
//    split done in registers while staging A (no split copy in HBM): 256x256x32
//    tiles, 8 waves of 128x64, per k32 step 3 x 32 mfma_f32_16x16x32_bf16 per
//    wave (A_hi W_hi + A_hi W_lo + A_lo W_hi) on 24 conflict-free ds_read_b128.
//  * cifar_split3_kernel: fp32 (B,K) -> bf16 (B,3K) = [hi | hi | lo], the A
//    operand of the small-batch fc1 (one skinny bf16 GEMM over K' = 3K against
//    W' = [W_hi | W_lo | W_hi]) when the 256^2 tiles cannot fill the chip.
//  * cifar_head_tail_x3_kernel: fc2 (512->10) + bias + softmax + per-row argmax
//    on fp32 hidden rows, 3-term split on mfma_f32_16x16x32_bf16.
#include <type_traits>

#include "gemm_epilogue.h"

namespace dnn {
namespace x3 {

// 2 floats -> packed bf16 hi pair and lo pair (element a in the low half)
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pack2bf(a, b);
  const float ah = __uint_as_float(hi << 16), bh = __uint_as_float(hi & 0xffff0000u);
  lo = pack2bf(a - ah, b - bh);
}

__device__ __forceinline__ int dpp_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int dpp_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }

constexpr int XW = 40;                        // xin row pitch (pixels); HWC4 bf16 = 8 B/pixel
constexpr int XPL = 34 * XW * 8;              // 10880: one input plane
constexpr int A1PL = 18 * 18 * 64;            // 20736: one pooled-conv1 plane [18][18][32] bf16
constexpr int A1_OFF = 4 * XPL;               // 43520
constexpr int LDS_BYTES = A1_OFF + 4 * A1PL;  // 126464

__device__ __forceinline__ int xin_off(int k, int lo) { return ((k & 1) * 2 + lo) * XPL; }
__device__ __forceinline__ int a1_off(int k, int lo) { return A1_OFF + ((k & 1) * 2 + lo) * A1PL; }

// conv2 A-fragment immediate offset for k-step S (tap = S>>1, kx = tap % 3),
// tile column I (tx2) and plane (LO): the lane/ky/parity part lives in the base.
template <int S, int I, int LO>
__device__ __forceinline__ constexpr int c2_imm() {
  return (8 * I + (S >> 1) % 3) * 64 + LO * A1PL;
}

// 4 reads of k-step S: [hi t0, hi t1, lo t0, lo t1]
template <int S>
__device__ __forceinline__ void c2_issue(const uint32_t (&b)[3][2], bf16x8 (&a)[4]) {
  constexpr int ky = (S >> 1) / 3, par = S & 1;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[0]) : "v"(b[ky][par]), "i"(c2_imm<S, 0, 0>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[1]) : "v"(b[ky][par]), "i"(c2_imm<S, 1, 0>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[2]) : "v"(b[ky][par]), "i"(c2_imm<S, 0, 1>()));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[3]) : "v"(b[ky][par]), "i"(c2_imm<S, 1, 1>()));
}

// k-step S: issue step S+1's reads, wait for step S's (counted lgkmcnt; the
// caller has no other LDS op in flight), then 6 MFMAs alternating the two
// tiles' accumulators.  sched_barriers keep hipcc from hoisting MFMAs above
// the wait (cdna_hip_programming.md §5.7).
template <int S>
__device__ __forceinline__ void c2_step(const uint32_t (&b)[3][2], const bf16x8 (&wh)[18], const bf16x8 (&wl)[18],
                                        f32x16 (&acc)[2], bf16x8 (&cur)[4], bf16x8 (&nxt)[4]) {
  if constexpr (S + 1 < 18) {
    c2_issue<S + 1>(b, nxt);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
  acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[0], wh[S], acc[0], 0, 0, 0);
  acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[1], wh[S], acc[1], 0, 0, 0);
  acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[0], wl[S], acc[0], 0, 0, 0);
  acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[1], wl[S], acc[1], 0, 0, 0);
  acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2], wh[S], acc[0], 0, 0, 0);
  acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[3], wh[S], acc[1], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (S + 1 < 18) c2_step<S + 1>(b, wh, wl, acc, nxt, cur);
}

template <int N>
__device__ __forceinline__ void resident_fence(const bf16x8 (&w)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(w[i]));
}

}  // namespace x3

using namespace x3;

// SPLIT_OUT: the boundary leaves in the blocked hi/lo encoding
// (cifar_split_blocked_kernel) that cifar_fc1_x3_kernel<true> stages by DMA.
template <bool WIDE, bool SPLIT_OUT>
__global__ __launch_bounds__(512, 1) void cifar_stage0_x3_kernel(
    const float* __restrict__ x, float* __restrict__ out, const bf16_t* __restrict__ w1h,
    const bf16_t* __restrict__ w1l, const float* __restrict__ b1, const bf16_t* __restrict__ w2h,
    const bf16_t* __restrict__ w2l, const float* __restrict__ b2, int B) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave < 4;
  const int rw = wave & 3;
  const int rt = tid & 255;
  const int h = lane >> 5, r32 = lane & 31;
  const int n = B > (int)blockIdx.x ? (B - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;

  // every halo (input and pooled map) is zero for the whole launch; interiors are rewritten per image
  for (int i = tid; i < LDS_BYTES / 16; i += 512) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);

  __syncthreads();  // halos zeroed before any image is staged

  // The two roles run disjoint loops (wave-uniform branch, the same number of
  // barriers on both sides) so their resident operands never share live ranges:
  // producers hold conv1's split weights + the input prefetch, consumers the
  // 144 VGPRs of conv2's split weights.
  if (producer) {
    bf16x8 w1hf[3], w1lf[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      w1hf[s] = *reinterpret_cast<const bf16x8*>(w1h + r32 * 48 + s * 16 + h * 8);
      w1lf[s] = *reinterpret_cast<const bf16x8*>(w1l + r32 * 48 + s * 16 + h * 8);
    }
    const float bias = b1[r32];
    resident_fence(w1hf);
    resident_fence(w1lf);
    asm volatile("" ::"v"(bias));

    float pf[4][3];
    auto load_img = [&](int k) {
      const float* xb = x + (size_t)(blockIdx.x + (size_t)k * gridDim.x) * 3072;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) pf[i][c] = xb[c * 1024 + rt + 256 * i];
    };
    auto stage_img = [&](int k) {  // prefetch registers -> padded HWC4 hi / lo planes
      char* xh = smem + xin_off(k, 0);
      char* xl = smem + xin_off(k, 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = rt + 256 * i, yy = p >> 5, xx = p & 31;
        uint2 vh, vl;
        split2(pf[i][0], pf[i][1], vh.x, vl.x);
        split2(pf[i][2], 0.f, vh.y, vl.y);
        const int o = ((yy + 1) * XW + xx + 1) * 8;
        *reinterpret_cast<uint2*>(xh + o) = vh;
        *reinterpret_cast<uint2*>(xl + o) = vl;
      }
    };
    const int c1_lane = ((r32 >> 3) * XW + (r32 & 7) + 2 * h) * 8;
    const int q = ((r32 & 1) ? 2 : 0) + ((r32 & 2) ? 1 : 0);
    const int cb = r32 & ~3;

    // bias + ReLU + 2x2 max-pool in registers (max(a)+b == max(a+b) exactly), quad-DPP
    // gather of 4 channels of one pooled pixel per lane, hi/lo split, one 8-B store per plane
    auto conv1_epi = [&](int t, const f32x16& acc, int k) {
      const int ty = t >> 2, tx = t & 3;
      float v[4];
#pragma unroll
      for (int qy = 0; qy < 2; ++qy)
#pragma unroll
        for (int qx = 0; qx < 2; ++qx) {
          const int g0 = (2 * qy) * 4 + 2 * qx;
          v[qy * 2 + qx] = fmaxf(fmax_nan(fmax_nan(acc[g0], acc[g0 + 1]), fmax_nan(acc[g0 + 4], acc[g0 + 5])) + bias, 0.f);
        }
      const bool odd = r32 & 1;
      const int s0 = __float_as_int(odd ? v[0] : v[2]), s1 = __float_as_int(odd ? v[1] : v[3]);
      const float r0 = __int_as_float(dpp_xor1(s0)), r1 = __int_as_float(dpp_xor1(s1));
      uint32_t u0h, u0l, u1h, u1l;
      if (!odd) {
        split2(v[0], r0, u0h, u0l);
        split2(v[1], r1, u1h, u1l);
      } else {
        split2(r0, v[2], u0h, u0l);
        split2(r1, v[3], u1h, u1l);
      }
      const bool hi2 = r32 & 2;
      const uint32_t rch = (uint32_t)dpp_xor2((int)(hi2 ? u0h : u1h));
      const uint32_t rcl = (uint32_t)dpp_xor2((int)(hi2 ? u0l : u1l));
      const uint32_t mh = hi2 ? u1h : u0h, ml = hi2 ? u1l : u0l;
      uint2 wh, wl;
      wh.x = hi2 ? rch : mh;
      wh.y = hi2 ? mh : rch;
      wl.x = hi2 ? rcl : ml;
      wl.y = hi2 ? ml : rcl;
      const int Y = 2 * ty + (q >> 1) + 1, X = 4 * tx + 2 * h + (q & 1) + 1;
      const int o = (Y * 18 + X) * 64 + ((((cb >> 3) ^ (Y & 3))) << 4) + (cb & 7) * 2;
      *reinterpret_cast<uint2*>(smem + a1_off(k, 0) + o) = wh;
      *reinterpret_cast<uint2*>(smem + a1_off(k, 1) + o) = wl;
    };
    auto frag = [&](const char* p) {
      const uint2 a = *reinterpret_cast<const uint2*>(p);
      const uint2 b = *reinterpret_cast<const uint2*>(p + 8);
      return __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
    };
    // two conv1 tiles at once: all 24 A-fragment reads up front, two accumulation chains interleaved
    auto conv1_pair = [&](int ta, int tb, int k) {
      const char* xh = smem + xin_off(k, 0);
      const int oa = c1_lane + ((4 * (ta >> 2)) * XW + 8 * (ta & 3)) * 8;
      const int ob = c1_lane + ((4 * (tb >> 2)) * XW + 8 * (tb & 3)) * 8;
      bf16x8 fah[3], fal[3], fbh[3], fbl[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        fah[s] = frag(xh + oa + s * XW * 8);
        fbh[s] = frag(xh + ob + s * XW * 8);
        fal[s] = frag(xh + XPL + oa + s * XW * 8);
        fbl[s] = frag(xh + XPL + ob + s * XW * 8);
      }
      f32x16 acca = {}, accb = {};
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        acca = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fah[s], w1hf[s], acca, 0, 0, 0);
        accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fbh[s], w1hf[s], accb, 0, 0, 0);
        acca = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fah[s], w1lf[s], acca, 0, 0, 0);
        accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fbh[s], w1lf[s], accb, 0, 0, 0);
        acca = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fal[s], w1hf[s], acca, 0, 0, 0);
        accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fbl[s], w1hf[s], accb, 0, 0, 0);
      }
      conv1_epi(ta, acca, k);
      conv1_epi(tb, accb, k);
    };

    if (n > 0) {
      load_img(0);
      stage_img(0);
      if (n > 1) load_img(1);
    }
    __syncthreads();
    for (int it = 0; it <= n; ++it) {
      if (it < n) {
#pragma unroll 1
        for (int t = rw; t < 32; t += 8) conv1_pair(t, t + 4, it);
        if (it + 1 < n) {
          stage_img(it + 1);
          if (it + 2 < n) load_img(it + 2);
        }
      }
      __syncthreads();
    }
  } else {
    const int oc2 = (rw & 1) * 32 + r32;
    bf16x8 w2hf[18], w2lf[18];
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      w2hf[s] = *reinterpret_cast<const bf16x8*>(w2h + oc2 * 288 + s * 16 + h * 8);
      w2lf[s] = *reinterpret_cast<const bf16x8*>(w2l + oc2 * 288 + s * 16 + h * 8);
    }
    const float bias = b2[oc2];
    resident_fence(w2hf);
    resident_fence(w2lf);
    asm volatile("" ::"v"(bias));
    // lane base for (ky, channel-chunk parity): pixel row Y = 4*ty2 + (r32>>3) + ky,
    // Y & 3 = ((r32>>3) + ky) & 3 (4*ty2 = 0 mod 4), chunk = 2*par + h
    uint32_t lb[3][2];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const int yr = (r32 >> 3) + ky;
        lb[ky][par] = (uint32_t)((yr * 18 + (r32 & 7)) * 64 + (((2 * par + h) ^ (yr & 3)) << 4));
      }

    auto conv2_img = [&](int k) {  // conv2 + bias + ReLU + pool of image k -> out (fp32, NCHW flatten)
      float* ob = out + (size_t)(blockIdx.x + (size_t)k * gridDim.x) * 4096 + oc2 * 64;
      const uint32_t plane = (uint32_t)(uintptr_t)(smem + a1_off(k, 0));
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int ty2 = (rw >> 1) * 2 + p;
        const uint32_t rb = plane + ty2 * 4 * 18 * 64;
        uint32_t b[3][2];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int par = 0; par < 2; ++par) b[ky][par] = rb + lb[ky][par];
        f32x16 acc[2] = {f32x16{}, f32x16{}};
        bf16x8 a0[4], a1[4];
        c2_issue<0>(b, a0);
        c2_step<0>(b, w2hf, w2lf, acc, a0, a1);
        if constexpr (WIDE) {
          // 16-B stores: lane half h holds pooled columns 4i+2h..+1 of both
          // tiles; one v_permlane32_swap per dword gives half 0 columns 0-3
          // (its own tile-0 pair + the other half's) and half 1 columns 4-7,
          // so a row leaves as one dwordx4 per lane instead of two dwordx2
#pragma unroll
          for (int qy = 0; qy < 2; ++qy) {
            const int g0 = (2 * qy) * 4;
            float v[2][2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              v[i][0] = fmaxf(fmax_nan(fmax_nan(acc[i][g0], acc[i][g0 + 1]), fmax_nan(acc[i][g0 + 4], acc[i][g0 + 5])) + bias, 0.f);
              v[i][1] = fmaxf(fmax_nan(fmax_nan(acc[i][g0 + 2], acc[i][g0 + 3]), fmax_nan(acc[i][g0 + 6], acc[i][g0 + 7])) + bias,
                              0.f);
            }
            const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0][0]), __float_as_uint(v[1][0]), false,
                                                             false);
            const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0][1]), __float_as_uint(v[1][1]), false,
                                                             false);
            const int PY = 2 * ty2 + qy;
            if constexpr (SPLIT_OUT) {  // k = oc2*64 + PY*8 + 4h + 0..3: one 8-B hi and one 8-B lo store
              uint2 hi, lo;
              split2(__uint_as_float(sx[0]), __uint_as_float(sy[0]), hi.x, lo.x);
              split2(__uint_as_float(sx[1]), __uint_as_float(sy[1]), hi.y, lo.y);
              char* bp = reinterpret_cast<char*>(ob - oc2 * 64) + (oc2 * 2 + (PY >> 2)) * 128 + ((PY & 3) * 8 + 4 * h) * 2;
              *reinterpret_cast<uint2*>(bp) = hi;
              *reinterpret_cast<uint2*>(bp + 64) = lo;
            } else {
              *reinterpret_cast<uint4*>(ob + PY * 8 + 4 * h) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
            }
          }
        } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
          for (int qy = 0; qy < 2; ++qy) {
            float2 pv;
            const int g0 = (2 * qy) * 4;
            pv.x = fmaxf(fmax_nan(fmax_nan(acc[i][g0], acc[i][g0 + 1]), fmax_nan(acc[i][g0 + 4], acc[i][g0 + 5])) + bias, 0.f);
            pv.y = fmaxf(fmax_nan(fmax_nan(acc[i][g0 + 2], acc[i][g0 + 3]), fmax_nan(acc[i][g0 + 6], acc[i][g0 + 7])) + bias,
                         0.f);
            const int PY = 2 * ty2 + qy, PX = 4 * i + 2 * h;
            if constexpr (SPLIT_OUT) {
              uint32_t hi, lo;
              split2(pv.x, pv.y, hi, lo);
              char* bp = reinterpret_cast<char*>(ob - oc2 * 64) + (oc2 * 2 + (PY >> 2)) * 128 + ((PY & 3) * 8 + PX) * 2;
              *reinterpret_cast<uint32_t*>(bp) = hi;
              *reinterpret_cast<uint32_t*>(bp + 64) = lo;
            } else {
              *reinterpret_cast<float2*>(ob + PY * 8 + PX) = pv;
            }
          }
        }
        }
      }
    };

    __syncthreads();
    for (int it = 0; it <= n; ++it) {
      if (it >= 1) conv2_img(it - 1);
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// fc1 at fp32 precision: C = relu(A . W^T + bias), A fp32 [M][K], W = W_hi + W_lo
// (bf16 [N][K] each), C fp32.  A is read from HBM once per tile pair as fp32 and
// split in registers (global_load_dwordx4 -> split2 -> ds_write_b128) while the
// W halves stream into LDS by DMA (global_load_lds, source-side swizzle).  LDS:
// 2 buffers x [A_hi A_lo W_hi W_lo] planes of 256 rows x 32 k (64-B rows, 16 KiB)
// = 128 KiB.  The 16-B chunk c of row r is stored at c ^ ((r >> 2) & 2): the
// four ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) of a fragment read
// (lane: row l & 15, chunk l >> 4) then hit 16 distinct slots, and the A
// writes (8 contiguous lanes = 2 rows x 4 chunks) 8 distinct ds_write slots.
// One barrier per k32 step: the step's next-tile loads are issued before its
// MFMAs and land in the other buffer.
// ---------------------------------------------------------------------------
constexpr int F1_T = 256, F1_K = 32, F1_PLANE = 256 * 64;

__device__ __forceinline__ int f1_swz(int r) { return (r >> 2) & 2; }

__device__ __forceinline__ bf16x8 f1_frag(const char* plane, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(plane + row * 64 + ((chunk ^ f1_swz(row)) << 4));
}

__device__ __forceinline__ void f1_tile_coords(int logical, int ntm, int ntn, int& tm, int& tn) {
  // M fastest inside groups of 8 M-tiles: the ntn column tiles of one A panel
  // run close together on one XCD, so A's second read hits L2 / MALL
  constexpr int G = 8;
  const int per = G * ntn, grp = logical / per, first = grp * G;
  const int gm = min(ntm - first, G), r = logical - grp * per;
  tm = first + r % gm;
  tn = r / gm;
}

// A goes to registers one k-step ahead.  Measured alternatives, dropped: A by
// DMA into a 32 KiB fp32 staging area two k-steps ahead (5 % slower), the
// split+store between the two MFMA halves (flat), a second register set for A
// two k-steps ahead once the loads were coalesced (flat, 6 spilled VGPRs).  Probes
// (profiles/archive/r2_cifar_fc1_probes.jsonl): without the A stream the kernel runs
// 0.51 ms, without any load 0.45 ms (1.8 PF/s), with both 0.80 ms.
//
// SPLIT_IN: A arrives pre-split in the blocked boundary encoding (see
// cifar_split_blocked_kernel: per row and 32-k block, 32 bf16 hi then 32 bf16
// lo — the same 4 bytes per element as fp32, the same hi/lo this kernel would
// form in registers), so A is staged by DMA exactly like W: no VGPR round
// trip, no split ALU, no vmcnt stall on A inside the k loop.
template <bool SPLIT_IN>
__global__ __launch_bounds__(512, 1) void cifar_fc1_x3_kernel(const float* __restrict__ A, int lda,
                                                              const bf16_t* __restrict__ Wh,
                                                              const bf16_t* __restrict__ Wl, int ldw,
                                                              const float* __restrict__ bias, float* __restrict__ C,
                                                              int ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 4 * F1_PLANE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = N / F1_T, ntm = (M + F1_T - 1) / F1_T;
  int tm, tn;
  f1_tile_coords(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, tm, tn);
  const int m0 = tm * F1_T, n0 = tn * F1_T;
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / F1_K;
  auto plane = [&](int u, int p) { return smem + (u * 4 + p) * F1_PLANE; };  // p: 0 A_hi, 1 A_lo, 2 W_hi, 3 W_lo

  // A: 2 chunks (8 fp32 each) per thread; chunk q = tid + 512 i -> row q >> 2, k-chunk q & 3
  // A: 4 pieces of 16 B per thread; piece k: row (tid >> 3) + 64 k, floats
  // 4 (tid & 7) .. +3, so every wave load instruction reads 8 whole 128-B row
  // segments and the split halves land as ds_write_b64 into half of a 16-B LDS
  // chunk.  (The first mapping, 32 contiguous bytes per lane in two loads,
  // touched every 128-B line twice per wave: 0.85 -> 0.68 ms.)
  float4 ar[4];
  auto load_a = [&](int t, auto) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = min(m0 + (tid >> 3) + 64 * k, M - 1);
      ar[k] = *reinterpret_cast<const float4*>(A + (size_t)row * lda + t * F1_K + (tid & 7) * 4);
    }
  };
  auto store_a = [&](int u, auto) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = (tid >> 3) + 64 * k, c = (tid & 7) >> 1, half = tid & 1;
      uint2 hi, lo;
      split2(ar[k].x, ar[k].y, hi.x, lo.x);
      split2(ar[k].z, ar[k].w, hi.y, lo.y);
      const int o = r * 64 + ((c ^ f1_swz(r)) << 4) + half * 8;
      *reinterpret_cast<uint2*>(plane(u, 0) + o) = hi;
      *reinterpret_cast<uint2*>(plane(u, 1) + o) = lo;
    }
  };
  // W: per plane 16 pieces of 16 rows (1 KiB per wave instruction), 2 per wave
  // SPLIT_IN: A hi / lo planes by DMA, 2 pieces of 16 rows per wave and plane (as W)
  auto stage_a = [&](int u, int t) {
    const char* Ab = reinterpret_cast<const char*>(A);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int piece = wave * 2 + j, rl = piece * 16 + (lane >> 2);
        const int c = (lane & 3) ^ f1_swz(rl);
        const int row = min(m0 + rl, M - 1);
        glds16(Ab + (size_t)row * lda * 4 + t * 128 + p * 64 + c * 16, plane(u, p) + piece * 1024);
      }
    }
  };
  auto stage_w = [&](int u, int t) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const bf16_t* W = p ? Wl : Wh;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int piece = wave * 2 + j, rl = piece * 16 + (lane >> 2);
        const int c = (lane & 3) ^ f1_swz(rl);
        glds16(W + (size_t)(n0 + rl) * ldw + t * F1_K + c * 8, plane(u, 2 + p) + piece * 1024);
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  using I0 = std::integral_constant<int, 0>;
  if constexpr (SPLIT_IN) {
    stage_a(0, 0);
    stage_w(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load_a(0, I0{});
    stage_w(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_a(0, I0{});
  }
  __syncthreads();

  const int fr = lane & 15, fc = lane >> 4;
  auto compute = [&](int u) {
    const char* ah_p = plane(u, 0);
    const char* al_p = plane(u, 1);
    const char* bh_p = plane(u, 2);
    const char* bl_p = plane(u, 3);
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = f1_frag(bh_p, wc * 64 + j * 16 + fr, fc);
      bl[j] = f1_frag(bl_p, wc * 64 + j * 16 + fr, fc);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 ah[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ah[i] = f1_frag(ah_p, wr * 128 + (h * 4 + i) * 16 + fr, fc);
        al[i] = f1_frag(al_p, wr * 128 + (h * 4 + i) * 16 + fr, fc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4& a = acc[h * 4 + i][j];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], a, 0, 0, 0);
        }
    }
  };
  // raw barrier (lgkmcnt for this step's LDS writes; the DMAs were waited
  // above): 6 % faster than __syncthreads here
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; ++t) {
    const int u = t & 1;
    if (t + 1 < nk) {
      if constexpr (SPLIT_IN)
        stage_a(u ^ 1, t + 1);
      else
        load_a(t + 1, I0{});
      stage_w(u ^ 1, t + 1);
    }
    compute(u);
    if (t + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (!SPLIT_IN) store_a(u ^ 1, I0{});
    }
    barrier();
  }

  // epilogue (transposed accumulators): row m0 + wr*128 + i*16 + (lane & 15), cols n..n+3
  const bool vec = epi_vec_ok(C, ldc, bias, nullptr, 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      epi_t4<ACT_RELU, true>(acc[i][j], m, n0 + wc * 64 + j * 16 + fc * 4, M, N, C, ldc, bias, nullptr, 0, vec);
  }
}

// Blocked boundary encoding of an fp32 (M,K) tensor, in place of the same
// 4 bytes per element: row r, 32-k block b holds 32 bf16 hi then 32 bf16 lo
// (hi + lo == x to ~2^-17 relative, the exact operand split of the x3 MFMAs).
// dir 0: fp32 -> blocked, dir 1: blocked -> fp32 (hi + lo).  K % 32 == 0.
__global__ __launch_bounds__(256) void cifar_split_blocked_kernel(const float* __restrict__ a, float* __restrict__ o,
                                                                  int M, int K, int dir) {
  const int per_row = K / 8;  // 8-element pieces
  const long total = (long)M * per_row;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int m = (int)(e / per_row), k = (int)(e % per_row) * 8;
    char* rowp = reinterpret_cast<char*>(o + (size_t)m * K);
    const char* rowa = reinterpret_cast<const char*>(a + (size_t)m * K);
    const int hoff = (k >> 5) * 128 + (k & 31) * 2;
    if (dir == 0) {
      const float4 u = *reinterpret_cast<const float4*>(rowa + k * 4);
      const float4 v = *reinterpret_cast<const float4*>(rowa + k * 4 + 16);
      uint4 hi, lo;
      split2(u.x, u.y, hi.x, lo.x);
      split2(u.z, u.w, hi.y, lo.y);
      split2(v.x, v.y, hi.z, lo.z);
      split2(v.z, v.w, hi.w, lo.w);
      *reinterpret_cast<uint4*>(rowp + hoff) = hi;
      *reinterpret_cast<uint4*>(rowp + hoff + 64) = lo;
    } else {
      const uint4 hi = *reinterpret_cast<const uint4*>(rowa + hoff);
      const uint4 lo = *reinterpret_cast<const uint4*>(rowa + hoff + 64);
      const uint32_t h[4] = {hi.x, hi.y, hi.z, hi.w}, l[4] = {lo.x, lo.y, lo.z, lo.w};
      float r[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        r[2 * i] = __uint_as_float(h[i] << 16) + __uint_as_float(l[i] << 16);
        r[2 * i + 1] = __uint_as_float(h[i] & 0xffff0000u) + __uint_as_float(l[i] & 0xffff0000u);
      }
      *reinterpret_cast<float4*>(rowp + k * 4) = float4{r[0], r[1], r[2], r[3]};
      *reinterpret_cast<float4*>(rowp + k * 4 + 16) = float4{r[4], r[5], r[6], r[7]};
    }
  }
}

// fp32 (M,K) -> bf16 (M,3K) rows [hi | hi | lo]; K % 8 == 0, 16-B aligned rows.
// blocked = 1: a is in the blocked hi/lo encoding (the split is already done).
__global__ __launch_bounds__(256) void cifar_split3_kernel(const float* __restrict__ a, int lda,
                                                           bf16_t* __restrict__ o, int ldo, int M, int K,
                                                           int blocked) {
  const int per_row = K / 8;
  const long total = (long)M * per_row;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int m = (int)(e / per_row), c = (int)(e % per_row) * 8;
    uint4 hi, lo;
    if (blocked) {
      const char* rowa = reinterpret_cast<const char*>(a + (size_t)m * lda) + (c >> 5) * 128 + (c & 31) * 2;
      hi = *reinterpret_cast<const uint4*>(rowa);
      lo = *reinterpret_cast<const uint4*>(rowa + 64);
    } else {
      const float4 u = *reinterpret_cast<const float4*>(a + (size_t)m * lda + c);
      const float4 v = *reinterpret_cast<const float4*>(a + (size_t)m * lda + c + 4);
      split2(u.x, u.y, hi.x, lo.x);
      split2(u.z, u.w, hi.y, lo.y);
      split2(v.x, v.y, hi.z, lo.z);
      split2(v.z, v.w, hi.w, lo.w);
    }
    bf16_t* r = o + (size_t)m * ldo + c;
    *reinterpret_cast<uint4*>(r) = hi;
    *reinterpret_cast<uint4*>(r + K) = hi;
    *reinterpret_cast<uint4*>(r + 2 * K) = lo;
  }
}

// fc2 (512->10) + bias + softmax + argmax on fp32 hidden rows (fc1+ReLU output).
// One wave per 16 rows and iteration, mfma_f32_16x16x32_bf16 with the 3-term split:
// A = hid rows (lane: row l&15, k 8*(l>>4)+j), B = W2 hi/lo padded to 16 classes in VGPRs.
__global__ __launch_bounds__(256) void cifar_head_tail_x3_kernel(const float* __restrict__ hid,
                                                                 const bf16_t* __restrict__ w2h,
                                                                 const bf16_t* __restrict__ w2l,
                                                                 const float* __restrict__ b2,
                                                                 float* __restrict__ probs, int* __restrict__ pred,
                                                                 int B) {
  const int lane = threadIdx.x & 63;
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const int col = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 wfh[16], wfl[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    wfh[s] = *reinterpret_cast<const bf16x8*>(w2h + col * 512 + s * 32 + kq);
    wfl[s] = *reinterpret_cast<const bf16x8*>(w2l + col * 512 + s * 32 + kq);
  }
  const float bias = col < 10 ? b2[col] : 0.f;
  for (int r0 = gw * 16; r0 < B; r0 += nw * 16) {
    const int row = r0 + (lane & 15);
    const int rc = row < B ? row : B - 1;
    const float* ap = hid + (size_t)rc * 512 + kq;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float4 u = *reinterpret_cast<const float4*>(ap + s * 32);
      const float4 v = *reinterpret_cast<const float4*>(ap + s * 32 + 4);
      uint4 hi, lo;
      split2(u.x, u.y, hi.x, lo.x);
      split2(u.z, u.w, hi.y, lo.y);
      split2(v.x, v.y, hi.z, lo.z);
      split2(v.z, v.w, hi.w, lo.w);
      const bf16x8 ah = __builtin_bit_cast(bf16x8, hi), al = __builtin_bit_cast(bf16x8, lo);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wfh[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wfl[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wfh[s], acc, 0, 0, 0);
    }
    // acc[r] = logit(row = r0 + (lane>>4)*4 + r, class = col)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = col < 10 ? acc[r] + bias : -INFINITY;
      float mx = z;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float e = col < 10 ? expf(z - mx) : 0.f;
      float sum = e;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
      int cand = (z == mx) ? col : 16;  // smallest class index attaining the max (numpy semantics)
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

}  // namespace dnn

using namespace dnn;

// stage-0 boundary stores: 16-B (permlane32-paired, 1) or 8-B (0); A/B switch
static int g_s0_wide_store = 1;

extern "C" int dnn_cifar_s0_set_wide_store(int on) {
  g_s0_wide_store = on ? 1 : 0;
  return 0;
}

template <bool SPLIT_OUT>
static int launch_stage0_x3(const float* x, float* out, const void* w1h, const void* w1l, const float* b1,
                            const void* w2h, const void* w2l, const float* b2, int B, int grid, hipStream_t st) {
  if (g_s0_wide_store)
    hipLaunchKernelGGL((cifar_stage0_x3_kernel<true, SPLIT_OUT>), dim3(grid), dim3(512), 0, st, x, out,
                       (const bf16_t*)w1h, (const bf16_t*)w1l, b1, (const bf16_t*)w2h, (const bf16_t*)w2l, b2, B);
  else
    hipLaunchKernelGGL((cifar_stage0_x3_kernel<false, SPLIT_OUT>), dim3(grid), dim3(512), 0, st, x, out,
                       (const bf16_t*)w1h, (const bf16_t*)w1l, b1, (const bf16_t*)w2h, (const bf16_t*)w2l, b2, B);
  return (int)hipGetLastError();
}

// split_out = 1: the (B,4096) boundary in the blocked hi/lo encoding, else fp32.
extern "C" int dnn_cifar_stage0_x3(const float* x, float* out, const void* w1h, const void* w1l, const float* b1,
                                   const void* w2h, const void* w2l, const float* b2, int B, int grid,
                                   hipStream_t st, int split_out) {
  if (B <= 0) return 0;
  if (grid <= 0) grid = 256;
  if (grid > B) grid = B;
  return split_out ? launch_stage0_x3<true>(x, out, w1h, w1l, b1, w2h, w2l, b2, B, grid, st)
                   : launch_stage0_x3<false>(x, out, w1h, w1l, b1, w2h, w2l, b2, B, grid, st);
}

extern "C" int dnn_cifar_fc1_x3(const float* A, int lda, const void* Wh, const void* Wl, int ldw, const float* bias,
                                float* C, int ldc, int M, int N, int K, hipStream_t st, int a_split) {
  if (M <= 0) return 0;
  if (N % F1_T != 0 || K % F1_K != 0 || lda % 4 != 0 || ldw % 8 != 0 || ldc % 4 != 0) return -1;
  const int blocks = ((M + F1_T - 1) / F1_T) * (N / F1_T);
  if (a_split)
    hipLaunchKernelGGL(cifar_fc1_x3_kernel<true>, dim3(blocks), dim3(512), 0, st, A, lda, (const bf16_t*)Wh,
                       (const bf16_t*)Wl, ldw, bias, C, ldc, M, N, K);
  else
    hipLaunchKernelGGL(cifar_fc1_x3_kernel<false>, dim3(blocks), dim3(512), 0, st, A, lda, (const bf16_t*)Wh,
                       (const bf16_t*)Wl, ldw, bias, C, ldc, M, N, K);
  return (int)hipGetLastError();
}

extern "C" int dnn_cifar_split_blocked(const float* a, float* o, int M, int K, int dir, hipStream_t st) {
  if (M <= 0) return 0;
  if (K % 32 != 0 || a == o) return -1;
  const long total = (long)M * (K / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cifar_split_blocked_kernel, dim3((int)blocks), dim3(256), 0, st, a, o, M, K, dir);
  return (int)hipGetLastError();
}

extern "C" int dnn_cifar_split3(const float* a, int lda, void* o, int ldo, int M, int K, hipStream_t st, int blocked) {
  if (M <= 0) return 0;
  if (K % 8 != 0 || lda % 4 != 0 || ldo % 8 != 0 || ldo < 3 * K || (blocked && K % 32 != 0)) return -1;
  const long total = (long)M * (K / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cifar_split3_kernel, dim3((int)blocks), dim3(256), 0, st, a, lda, (bf16_t*)o, ldo, M, K, blocked);
  return (int)hipGetLastError();
}

extern "C" int dnn_cifar_head_tail_x3(const float* hid, const void* w2h, const void* w2l, const float* b2,
                                      float* probs, int* pred, int B, hipStream_t st) {
  if (B <= 0) return 0;
  int waves = (B + 15) / 16;
  int blocks = (waves + 3) / 4;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(cifar_head_tail_x3_kernel, dim3(blocks), dim3(256), 0, st, hid, (const bf16_t*)w2h,
                     (const bf16_t*)w2l, b2, probs, pred, B);
  return (int)hipGetLastError();
}
