// C ABI of the kernel library (every function enqueues on `st` and returns the
// hipError_t of the launch; 0 = success, negative = rejected shape).
// GEMM entry points take an optional `Wsh`: the decode (M <= 64) weight in the
// skinny kernel's fragment order (ops/gemm.py shuffle_weight); nullptr = use W;
// and an optional workspace `ws` of `ws_bytes` for the decode stream kernel's
// split-K partials (nullptr: no K split).
#pragma once
#include <hip/hip_runtime.h>

extern "C" {
int dnn_gemm_bf16(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias, const void* R,
                  int ldr, int M, int N, int K, int act, int out_f32, hipStream_t st, const void* Wsh = nullptr,
                  const float* rowstat = nullptr, const float* colsum = nullptr, void* ws = nullptr,
                  long long ws_bytes = 0);
int dnn_row_stats(const void* x, int ldx, float* stats, int M, int N, float eps, int rms, hipStream_t st);
int dnn_gemm_set_tile(int tile);
int dnn_gemm_set_anatomy(int bits);
int dnn_gemm_set_skinny_pin(int id, int ks, int n, int k);
int dnn_gemm_bf16_qkv_scatter(const void* A, int lda, const void* W, int ldw, const float* bias, const float* rowstat,
                              const float* colsum, void* q, void* kc, void* vc, const int* pos, int B, int T, int H,
                              int Hkv, int hd, int S, int K, hipStream_t st);
int dnn_gemm_fp8_qkv_scatter(const void* A8, const float* sa, const void* W8, const float* sw, const float* bias,
                             void* q, void* kc, void* vc, const int* pos, int B, int T, int H, int Hkv, int hd, int S,
                             int Kb, hipStream_t st);
int dnn_gemm_set_res_prefetch(int on);
int dnn_gemm_set_half_cost(float c);
int dnn_gemm_set_skinny_max_m(int m);
int dnn_gemm_fp8_set_tile(int tile);
int dnn_gemm_fp8_256(const void* A, const float* sa, const void* W, const float* sw, void* C, int ldc, const float* bias,
                     const void* R, int ldr, int M, int N, int Kb, int act, hipStream_t st);
int dnn_gemm_skinny_sweep(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc, int M,
                          int N, int K, int nt, int u, int ks, int pipe, int w8, hipStream_t st);
int dnn_gemm_skinny_norm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, const float* bias,
                         const void* R, int ldr, int M, int N, int K, int act, int norm, const float* colsum, float eps,
                         hipStream_t st, const void* Wsh = nullptr, void* ws = nullptr, long long ws_bytes = 0);
int dnn_gemm_skinny_w8(const void* A, int lda, const void* W, int ldw, const float* sw, void* C, int ldc,
                       const float* bias, const void* R, int ldr, int M, int N, int K, int act, int norm,
                       const float* colsum, float eps, hipStream_t st, const void* Wsh = nullptr, void* ws = nullptr,
                       long long ws_bytes = 0);
int dnn_gemm_skinny(const void* A, int lda, const float* sa, const void* W, int ldw, const float* sw, void* C, int ldc,
                    const float* bias, const void* R, int ldr, int M, int N, int K, int act, int out_f32, int fp8,
                    hipStream_t st, const void* Wsh = nullptr, void* ws = nullptr, long long ws_bytes = 0);
// decode stream GEMM (gemm_stream.h) switch: 0 off / 1 auto / 2 forced, the weight-byte threshold (<= 0
// keeps it), and the in-launch split-K combine (fold: 1 on, 0 reduce launch, -1 keep)
int dnn_gemm_set_stream(int on, long long min_bytes, int fold = -1);
// one-shot decode GEMM (gemm_oneshot.h): on 0 off / 1 planned shapes / 2 every eligible shape; a non-zero
// (mt, ntw, steps, splitk) pins that config for every eligible call (A/B probes)
int dnn_gemm_set_oneshot(int on, int mt, int ntw, int steps, int splitk);
int dnn_gemm_set_oneshot_lds_floor(int bytes);
// race probe (gemm_oneshot.h probe bits; abl 0 = off): records per workgroup in rec
int dnn_gemm_set_oneshot_probe(void* rec, int abl);
int dnn_gemm_oneshot_sweep(const void* A, int lda, const void* Wsh, const float* sw, void* C, int ldc, int M, int N,
                           int K, int mt, int ntw, int steps, int splitk, int w8, void* ws, long long ws_bytes,
                           hipStream_t st);
// decode vocabulary head + argmax partials (gemm_head.h): returns partials per row (> 0) or < 0 (not covered)
int dnn_gemm_set_head(int on);
int dnn_gemm_head(const void* A, int lda, const void* Wsh, const float* sw, const float* colsum, const float* bias,
                  float eps, int norm, void* C, int ldc, int M, int N, int K, int w8, void* part, int part_cap,
                  hipStream_t st);
// hist (optional, with pos_inc): hist[row * hist_ld + pos_inc[row]] = id before the advance (token history)
int dnn_argmax_final(const void* part, int S, int M, int* out, int* out2, int* pos_inc, hipStream_t st,
                     int* hist = nullptr, int hist_ld = 0);
// prefill: 256^2 + 256x128 tail split (gemm_bf16.hip launch_gemm)
int dnn_gemm_set_split_tail(int on);
// MX-scaled W8A8 prefill (e8m0 per (row, 128 columns), common.h mx_index)
int dnn_quant_fp8_mx(const void* x, int ldx, void* q, int ldq, void* sx, int M, int K, int kpad, hipStream_t st);
int dnn_layernorm_q8_mx(const void* x, int ldx, const float* w, const float* b, void* q, int ldq, void* sx, int M,
                        int N, int kpad, float eps, int rms, hipStream_t st);
int dnn_gemm_fp8_mx(const void* A8, const void* sx, const void* W8, const float* sw, void* C, int ldc,
                    const float* bias, const void* R, int ldr, int M, int N, int Kb, int act, void* qo, int ldq,
                    void* sxo, int kpo, hipStream_t st);
int dnn_gemm_fp8_qkv_scatter_mx(const void* A8, const void* sx, const void* W8, const float* sw, const float* bias,
                                void* q, void* kc, void* vc, const int* pos, int B, int T, int H, int Hkv, int hd,
                                int S, int Kb, hipStream_t st);
// producer-side row statistics for the next decode GEMM call of this thread (gemm_skinny.hip)
int dnn_gemm_rowstats(void* out, int out_ld, const void* in, int in_ld);
int dnn_gemm_rowstats_written();
// decode GEMM epilogue operands with the first loads (1, default) / after (0)
int dnn_gemm_set_epi_prefetch(int on);
// probe: one-shot launch with parts removed
int dnn_gemm_oneshot_ablate(const void* A, int lda, const void* Wsh, const float* sw, void* C, int ldc, int M, int N,
                            int K, int cfg, int abl, hipStream_t st);
int dnn_silu_mul_packed(const void* gu, int ld_in, void* out, int ld_out, int M, int F, hipStream_t st);
int dnn_cifar_stage0_v4(const float* x, void* out, const void* w1p, const float* b1, const void* w2p, const float* b2,
                        int B, int grid, hipStream_t st);
int dnn_cifar_set_v4_pt(int pt);
int dnn_cifar_stage0_x3(const float* x, float* out, const void* w1h, const void* w1l, const float* b1, const void* w2h,
                        const void* w2l, const float* b2, int B, int grid, hipStream_t st, int split_out = 0);
int dnn_cifar_s0_set_wide_store(int on);
int dnn_cifar_split3(const float* a, int lda, void* o, int ldo, int M, int K, hipStream_t st, int blocked = 0);
int dnn_cifar_fc1_x3(const float* A, int lda, const void* Wh, const void* Wl, int ldw, const float* bias, float* C,
                     int ldc, int M, int N, int K, hipStream_t st, int a_split = 0);
int dnn_cifar_split_blocked(const float* a, float* o, int M, int K, int dir, hipStream_t st);
int dnn_cifar_head_tail_x3(const float* hid, const void* w2h, const void* w2l, const float* b2, float* probs, int* pred,
                           int B, hipStream_t st);
int dnn_cifar_head_tail(const void* hid, const void* w2p, const float* b2, float* probs, int* pred, int B,
                        hipStream_t st);
// split: rows of 2 kpad bytes, e4m3 hi plane then the residual plane (W8A8 prefill with split activations)
int dnn_layernorm_q8(const void* x, int ldx, const float* w, const float* b, void* q, int ldq, float* sq, int M, int N,
                     int kpad, float eps, int rms, hipStream_t st, int split = 0);
int dnn_layernorm(const void* x, int ldx, const float* w, const float* b, void* y, int ldy, int M, int N, float eps,
                  int rms, hipStream_t st);
int dnn_embed_gpt2(const int* idx, const void* wte, const void* wpe, void* out, int B, int T, int d, const int* pos,
                   int V, int P, hipStream_t st);
int dnn_qkv_split(const void* qkv, void* q, void* kc, void* vc, int B, int T, int H, int Hkv, int hd, int S,
                  const int* pos, const float* cos, const float* sin, int rope, hipStream_t st, int kv8 = 0);
int dnn_flash_attn_qkv(const void* qkv, int ldqkv, void* kc, void* vc, void* o, int B, int T, int H, int Hkv,
                       int hd, int S, const int* pos, float scale, hipStream_t st, int kv8 = 0);
int dnn_flash_attn(const void* q, const void* kc, const void* vc, void* o, int B, int T, int H, int Hkv, int hd, int S,
                   const int* pos, float scale, hipStream_t st, int kv8 = 0);
int dnn_attn_decode_qkv(const void* qkv, int ldqkv, void* kc, void* vc, void* o, int B, int H, int Hkv, int hd, int S,
                        const int* pos, const float* cosT, const float* sinT, float scale, int splits, float* ws,
                        hipStream_t st, int kv8 = 0);
int dnn_attn_decode(const void* q, const void* kc, const void* vc, void* o, int B, int H, int Hkv, int hd, int S,
                    const int* lens, float scale, int splits, float* ws, hipStream_t st, int kv8 = 0);
int dnn_sample_topk(const void* x, int ld, int M, int N, int* out, float temperature, int topk, unsigned seed,
                    const int* step, hipStream_t st);
int dnn_argmax_rows(const void* x, int ld, int M, int N, int* out, int f32in, hipStream_t st, int* out2 = nullptr,
                    int* pos_inc = nullptr, void* part = nullptr, int* hist = nullptr, int hist_ld = 0);
int dnn_quant_fp8_rows(const void* x, int ldx, void* q, float* scale, int M, int K, int kpad, hipStream_t st,
                       int split = 0);
int dnn_gemm_fp8(const void* A, const float* sa, const void* W, const float* sw, void* C, int ldc, const float* bias,
                 const void* R, int ldr, int M, int N, int K, int act, hipStream_t st);
}
