// pybind11 bindings for the gfx950 kernel library.
// The ABI is raw device pointers (as Python ints from tensor.data_ptr()) plus
// the hipStream_t of the caller's current stream, so the module links only
// against the HIP runtime (torch's own libamdhip64, already loaded by
// `import torch`), never against torch's C++ ABI. Every entry returns the HIP
// error code of the launch; the Python wrappers raise on non-zero.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>
#include <cstdint>

#include "kernels/api.h"
#include "comm/p2p.h"

#include <string>
#include <vector>

namespace py = pybind11;
#define P(x) reinterpret_cast<void*>(static_cast<uintptr_t>(x))
#define CP(x) reinterpret_cast<const void*>(static_cast<uintptr_t>(x))
#define FP(x) reinterpret_cast<float*>(static_cast<uintptr_t>(x))
#define CFP(x) reinterpret_cast<const float*>(static_cast<uintptr_t>(x))
#define IP(x) reinterpret_cast<int*>(static_cast<uintptr_t>(x))
#define CIP(x) reinterpret_cast<const int*>(static_cast<uintptr_t>(x))
#define ST(x) reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(x))
typedef uint64_t u64;

PYBIND11_MODULE(_dnn_hip, m) {
  m.doc() = "distributed_neural_networks_amd HIP/CDNA4 kernels (gfx950)";
  m.attr("arch") = "gfx950";

  m.def("gemm_bf16", [](u64 A, int lda, u64 W, int ldw, u64 C, int ldc, u64 bias, u64 R, int ldr, int M, int N,
                        int K, int act, int out_f32, u64 st, u64 wsh, u64 rowstat, u64 colsum, u64 ws,
                        long long ws_bytes) {
    return dnn_gemm_bf16(CP(A), lda, CP(W), ldw, P(C), ldc, CFP(bias), CP(R), ldr, M, N, K, act, out_f32, ST(st),
                         CP(wsh), CFP(rowstat), CFP(colsum), P(ws), ws_bytes);
  }, py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"), py::arg("C"), py::arg("ldc"), py::arg("bias"),
     py::arg("R"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("act"), py::arg("out_f32"),
     py::arg("st"), py::arg("wsh") = 0, py::arg("rowstat") = 0, py::arg("colsum") = 0, py::arg("ws") = 0,
     py::arg("ws_bytes") = 0);
  m.def("gemm_skinny", [](u64 A, int lda, u64 sa, u64 W, int ldw, u64 sw, u64 C, int ldc, u64 bias, u64 R, int ldr,
                          int M, int N, int K, int act, int out_f32, int fp8, u64 st) {
    return dnn_gemm_skinny(CP(A), lda, CFP(sa), CP(W), ldw, CFP(sw), P(C), ldc, CFP(bias), CP(R), ldr, M, N, K, act,
                           out_f32, fp8, ST(st));
  });
  m.def("gemm_skinny_norm", [](u64 A, int lda, u64 W, int ldw, u64 C, int ldc, u64 bias, u64 R, int ldr, int M,
                               int N, int K, int act, int norm, u64 colsum, float eps, u64 st, u64 wsh, u64 ws,
                               long long ws_bytes) {
    return dnn_gemm_skinny_norm(CP(A), lda, CP(W), ldw, P(C), ldc, CFP(bias), CP(R), ldr, M, N, K, act, norm,
                                CFP(colsum), eps, ST(st), CP(wsh), P(ws), ws_bytes);
  }, py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"), py::arg("C"), py::arg("ldc"), py::arg("bias"),
     py::arg("R"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("act"), py::arg("norm"),
     py::arg("colsum"), py::arg("eps"), py::arg("st"), py::arg("wsh") = 0, py::arg("ws") = 0, py::arg("ws_bytes") = 0);
  m.def("gemm_skinny_w8", [](u64 A, int lda, u64 W, int ldw, u64 sw, u64 C, int ldc, u64 bias, u64 R, int ldr, int M,
                             int N, int K, int act, int norm, u64 colsum, float eps, u64 st, u64 wsh, u64 ws,
                             long long ws_bytes) {
    return dnn_gemm_skinny_w8(CP(A), lda, CP(W), ldw, CFP(sw), P(C), ldc, CFP(bias), CP(R), ldr, M, N, K, act, norm,
                              CFP(colsum), eps, ST(st), CP(wsh), P(ws), ws_bytes);
  }, py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"), py::arg("sw"), py::arg("C"), py::arg("ldc"),
     py::arg("bias"), py::arg("R"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("act"),
     py::arg("norm"), py::arg("colsum"), py::arg("eps"), py::arg("st"), py::arg("wsh") = 0, py::arg("ws") = 0,
     py::arg("ws_bytes") = 0);
  m.def("gemm_set_stream", [](int on, long long min_bytes, int fold) { return dnn_gemm_set_stream(on, min_bytes, fold); },
        py::arg("on"), py::arg("min_bytes"), py::arg("fold") = -1);
  m.def("gemm_set_oneshot", [](int on, int mt, int ntw, int steps, int splitk) {
    return dnn_gemm_set_oneshot(on, mt, ntw, steps, splitk);
  }, py::arg("on"), py::arg("mt") = 0, py::arg("ntw") = 0, py::arg("steps") = 0, py::arg("splitk") = 0);
  m.def("gemm_set_oneshot_lds_floor", [](int bytes) { return dnn_gemm_set_oneshot_lds_floor(bytes); });
  m.def("gemm_set_oneshot_probe", [](u64 rec, int abl) { return dnn_gemm_set_oneshot_probe(P(rec), abl); });
  m.def("gemm_set_head", [](int on) { return dnn_gemm_set_head(on); });
  m.def("gemm_set_split_tail", [](int on) { return dnn_gemm_set_split_tail(on); });
  m.def("gemm_head", [](u64 A, int lda, u64 Wsh, u64 sw, u64 colsum, u64 bias, float eps, int norm, u64 C, int ldc,
                        int M, int N, int K, int w8, u64 part, int part_cap, u64 st) {
    return dnn_gemm_head(CP(A), lda, CP(Wsh), CFP(sw), CFP(colsum), CFP(bias), eps, norm, P(C), ldc, M, N, K, w8,
                         P(part), part_cap, ST(st));
  });
  m.def("gemm_rowstats", [](u64 out, int out_ld, u64 in, int in_ld) {
    return dnn_gemm_rowstats(reinterpret_cast<void*>(static_cast<uintptr_t>(out)), out_ld, CP(in), in_ld);
  });
  m.def("gemm_rowstats_written", []() { return dnn_gemm_rowstats_written(); });
  m.def("gemm_set_epi_prefetch", [](int on) { return dnn_gemm_set_epi_prefetch(on); });
  m.def("gemm_oneshot_ablate", [](u64 A, int lda, u64 Wsh, u64 sw, u64 C, int ldc, int M, int N, int K, int cfg,
                                  int abl, u64 st) {
    return dnn_gemm_oneshot_ablate(CP(A), lda, CP(Wsh), CFP(sw), P(C), ldc, M, N, K, cfg, abl, ST(st));
  });
  m.def("quant_fp8_mx", [](u64 x, int ldx, u64 q, int ldq, u64 sx, int M, int K, int kpad, u64 st) {
    return dnn_quant_fp8_mx(CP(x), ldx, P(q), ldq, P(sx), M, K, kpad, ST(st));
  });
  m.def("layernorm_q8_mx", [](u64 x, int ldx, u64 w, u64 b, u64 q, int ldq, u64 sx, int M, int N, int kpad, float eps,
                              int rms, u64 st) {
    return dnn_layernorm_q8_mx(CP(x), ldx, CFP(w), CFP(b), P(q), ldq, P(sx), M, N, kpad, eps, rms, ST(st));
  });
  m.def("gemm_fp8_mx", [](u64 a, u64 sx, u64 w, u64 sw, u64 c, int ldc, u64 bias, u64 r, int ldr, int M, int N, int Kb,
                          int act, u64 qo, int ldq, u64 sxo, int kpo, u64 st) {
    return dnn_gemm_fp8_mx(CP(a), CP(sx), CP(w), CFP(sw), P(c), ldc, CFP(bias), CP(r), ldr, M, N, Kb, act, P(qo), ldq,
                           P(sxo), kpo, ST(st));
  });
  m.def("gemm_fp8_qkv_scatter_mx", [](u64 a, u64 sx, u64 w, u64 sw, u64 bias, u64 q, u64 kc, u64 vc, u64 pos, int B,
                                      int T, int H, int Hkv, int hd, int S, int Kb, u64 st) {
    return dnn_gemm_fp8_qkv_scatter_mx(CP(a), CP(sx), CP(w), CFP(sw), CFP(bias), P(q), P(kc), P(vc),
                                       reinterpret_cast<const int*>(static_cast<uintptr_t>(pos)), B, T, H, Hkv, hd, S,
                                       Kb, ST(st));
  });
  m.def("argmax_final", [](u64 part, int S, int M, u64 out, u64 out2, u64 pos_inc, u64 st, u64 hist, int hist_ld) {
    return dnn_argmax_final(CP(part), S, M, IP(out), IP(out2), IP(pos_inc), ST(st), IP(hist), hist_ld);
  });
  m.def("gemm_oneshot_sweep", [](u64 A, int lda, u64 Wsh, u64 sw, u64 C, int ldc, int M, int N, int K, int mt, int ntw,
                                 int steps, int splitk, int w8, u64 ws, long long ws_bytes, u64 st) {
    return dnn_gemm_oneshot_sweep(CP(A), lda, CP(Wsh), CFP(sw), P(C), ldc, M, N, K, mt, ntw, steps, splitk, w8, P(ws),
                                  ws_bytes, ST(st));
  });
  m.def("gemm_skinny_sweep", [](u64 A, int lda, u64 W, int ldw, u64 sw, u64 C, int ldc, int M, int N, int K, int nt,
                                int u, int ks, int pipe, int w8, u64 st) {
    return dnn_gemm_skinny_sweep(CP(A), lda, CP(W), ldw, CFP(sw), P(C), ldc, M, N, K, nt, u, ks, pipe, w8, ST(st));
  });
  m.def("gemm_set_tile", [](int tile) { return dnn_gemm_set_tile(tile); });
  m.def("gemm_set_anatomy", [](int bits) { return dnn_gemm_set_anatomy(bits); });
  m.def("gemm_set_skinny_pin", [](int id, int ks, int n, int k) { return dnn_gemm_set_skinny_pin(id, ks, n, k); });
  m.def("gemm_set_half_cost", [](float c) { return dnn_gemm_set_half_cost(c); });
  m.def("gemm_bf16_qkv_scatter", [](u64 A, int lda, u64 W, int ldw, u64 bias, u64 rowstat, u64 colsum, u64 q, u64 kc,
                                    u64 vc, u64 pos, int B, int T, int H, int Hkv, int hd, int S, int K, u64 st) {
    return dnn_gemm_bf16_qkv_scatter(CP(A), lda, CP(W), ldw, CFP(bias), CFP(rowstat), CFP(colsum), P(q), P(kc), P(vc),
                                     CIP(pos), B, T, H, Hkv, hd, S, K, ST(st));
  });
  m.def("gemm_fp8_qkv_scatter", [](u64 A8, u64 sa, u64 W8, u64 sw, u64 bias, u64 q, u64 kc, u64 vc, u64 pos, int B,
                                   int T, int H, int Hkv, int hd, int S, int Kb, u64 st) {
    return dnn_gemm_fp8_qkv_scatter(CP(A8), CFP(sa), CP(W8), CFP(sw), CFP(bias), P(q), P(kc), P(vc), CIP(pos), B, T, H,
                                    Hkv, hd, S, Kb, ST(st));
  });
  m.def("gemm_set_res_prefetch", [](int on) { return dnn_gemm_set_res_prefetch(on); });
  m.def("gemm_set_skinny_max_m", [](int m) { return dnn_gemm_set_skinny_max_m(m); });
  m.def("gemm_fp8_set_tile", [](int tile) { return dnn_gemm_fp8_set_tile(tile); });
  m.def("silu_mul_packed", [](u64 gu, int ld_in, u64 out, int ld_out, int M, int F, u64 st) {
    return dnn_silu_mul_packed(CP(gu), ld_in, P(out), ld_out, M, F, ST(st));
  });
  m.def("cifar_stage0_v4", [](u64 x, u64 out, u64 w1p, u64 b1, u64 w2p, u64 b2, int B, int grid, u64 st) {
    return dnn_cifar_stage0_v4(CFP(x), P(out), CP(w1p), CFP(b1), CP(w2p), CFP(b2), B, grid, ST(st));
  });
  m.def("cifar_set_v4_pt", [](int pt) { return dnn_cifar_set_v4_pt(pt); });
  m.def("cifar_stage0_x3", [](u64 x, u64 out, u64 w1h, u64 w1l, u64 b1, u64 w2h, u64 w2l, u64 b2, int B, int grid,
                              u64 st, int split_out) {
    return dnn_cifar_stage0_x3(CFP(x), FP(out), CP(w1h), CP(w1l), CFP(b1), CP(w2h), CP(w2l), CFP(b2), B, grid,
                               ST(st), split_out);
  }, py::arg("x"), py::arg("out"), py::arg("w1h"), py::arg("w1l"), py::arg("b1"), py::arg("w2h"), py::arg("w2l"),
        py::arg("b2"), py::arg("B"), py::arg("grid"), py::arg("st"), py::arg("split_out") = 0);
  m.def("cifar_s0_set_wide_store", [](int on) { return dnn_cifar_s0_set_wide_store(on); });
  m.def("cifar_split3", [](u64 a, int lda, u64 o, int ldo, int M, int K, u64 st, int blocked) {
    return dnn_cifar_split3(CFP(a), lda, P(o), ldo, M, K, ST(st), blocked);
  }, py::arg("a"), py::arg("lda"), py::arg("o"), py::arg("ldo"), py::arg("M"), py::arg("K"), py::arg("st"),
        py::arg("blocked") = 0);
  m.def("cifar_fc1_x3", [](u64 a, int lda, u64 wh, u64 wl, int ldw, u64 bias, u64 c, int ldc, int M, int N, int K,
                           u64 st, int a_split) {
    return dnn_cifar_fc1_x3(CFP(a), lda, CP(wh), CP(wl), ldw, CFP(bias), FP(c), ldc, M, N, K, ST(st), a_split);
  }, py::arg("a"), py::arg("lda"), py::arg("wh"), py::arg("wl"), py::arg("ldw"), py::arg("bias"), py::arg("c"),
        py::arg("ldc"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("st"), py::arg("a_split") = 0);
  m.def("cifar_split_blocked", [](u64 a, u64 o, int M, int K, int dir, u64 st) {
    return dnn_cifar_split_blocked(CFP(a), FP(o), M, K, dir, ST(st));
  });
  m.def("cifar_head_tail_x3", [](u64 hid, u64 w2h, u64 w2l, u64 b2, u64 probs, u64 pred, int B, u64 st) {
    return dnn_cifar_head_tail_x3(CFP(hid), CP(w2h), CP(w2l), CFP(b2), FP(probs), IP(pred), B, ST(st));
  });
  m.def("cifar_head_tail", [](u64 hid, u64 w2p, u64 b2, u64 probs, u64 pred, int B, u64 st) {
    return dnn_cifar_head_tail(CP(hid), CP(w2p), CFP(b2), FP(probs), IP(pred), B, ST(st));
  });
#ifdef DNN_HAVE_TRANSFORMER
  m.def("row_stats", [](u64 x, int ldx, u64 stats, int M, int N, float eps, int rms, u64 st) {
    return dnn_row_stats(CP(x), ldx, FP(stats), M, N, eps, rms, ST(st));
  });
  m.def("layernorm", [](u64 x, int ldx, u64 w, u64 b, u64 y, int ldy, int M, int N, float eps, int rms, u64 st) {
    return dnn_layernorm(CP(x), ldx, CFP(w), CFP(b), P(y), ldy, M, N, eps, rms, ST(st));
  });
  m.def("layernorm_q8", [](u64 x, int ldx, u64 w, u64 b, u64 q, int ldq, u64 sq, int M, int N, int kpad, float eps,
                           int rms, u64 st, int split) {
    return dnn_layernorm_q8(CP(x), ldx, CFP(w), CFP(b), P(q), ldq, FP(sq), M, N, kpad, eps, rms, ST(st), split);
  }, py::arg("x"), py::arg("ldx"), py::arg("w"), py::arg("b"), py::arg("q"), py::arg("ldq"), py::arg("sq"), py::arg("M"),
     py::arg("N"), py::arg("kpad"), py::arg("eps"), py::arg("rms"), py::arg("st"), py::arg("split") = 0);
  m.def("embed_gpt2", [](u64 idx, u64 wte, u64 wpe, u64 out, int B, int T, int d, u64 pos, int V, int Pn, u64 st) {
    return dnn_embed_gpt2(CIP(idx), CP(wte), CP(wpe), P(out), B, T, d, CIP(pos), V, Pn, ST(st));
  });
  m.def("qkv_split", [](u64 qkv, u64 q, u64 kc, u64 vc, int B, int T, int H, int Hkv, int hd, int S, u64 pos,
                        u64 cos, u64 sin, int rope, u64 st, int kv8) {
    return dnn_qkv_split(CP(qkv), P(q), P(kc), P(vc), B, T, H, Hkv, hd, S, CIP(pos), CFP(cos), CFP(sin), rope,
                         ST(st), kv8);
  }, py::arg("qkv"), py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("B"), py::arg("T"), py::arg("H"),
     py::arg("Hkv"), py::arg("hd"), py::arg("S"), py::arg("pos"), py::arg("cos"), py::arg("sin"), py::arg("rope"),
     py::arg("st"), py::arg("kv8") = 0);
  m.def("flash_attn_qkv", [](u64 qkv, int ldqkv, u64 kc, u64 vc, u64 o, int B, int T, int H, int Hkv, int hd, int S,
                             u64 pos, float scale, u64 st, int kv8) {
    return dnn_flash_attn_qkv(CP(qkv), ldqkv, P(kc), P(vc), P(o), B, T, H, Hkv, hd, S, CIP(pos), scale, ST(st), kv8);
  }, py::arg("qkv"), py::arg("ldqkv"), py::arg("kc"), py::arg("vc"), py::arg("o"), py::arg("B"), py::arg("T"),
     py::arg("H"), py::arg("Hkv"), py::arg("hd"), py::arg("S"), py::arg("pos"), py::arg("scale"), py::arg("st"),
     py::arg("kv8") = 0);
  m.def("flash_attn", [](u64 q, u64 kc, u64 vc, u64 o, int B, int T, int H, int Hkv, int hd, int S, u64 pos,
                         float scale, u64 st, int kv8) {
    return dnn_flash_attn(CP(q), CP(kc), CP(vc), P(o), B, T, H, Hkv, hd, S, CIP(pos), scale, ST(st), kv8);
  }, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("o"), py::arg("B"), py::arg("T"), py::arg("H"),
     py::arg("Hkv"), py::arg("hd"), py::arg("S"), py::arg("pos"), py::arg("scale"), py::arg("st"), py::arg("kv8") = 0);
  m.def("attn_decode", [](u64 q, u64 kc, u64 vc, u64 o, int B, int H, int Hkv, int hd, int S, u64 lens,
                          float scale, int splits, u64 ws, u64 st, int kv8) {
    return dnn_attn_decode(CP(q), CP(kc), CP(vc), P(o), B, H, Hkv, hd, S, CIP(lens), scale, splits, FP(ws), ST(st),
                           kv8);
  }, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("o"), py::arg("B"), py::arg("H"), py::arg("Hkv"),
     py::arg("hd"), py::arg("S"), py::arg("lens"), py::arg("scale"), py::arg("splits"), py::arg("ws"), py::arg("st"),
     py::arg("kv8") = 0);
  m.def("attn_decode_qkv", [](u64 qkv, int ldqkv, u64 kc, u64 vc, u64 o, int B, int H, int Hkv, int hd, int S,
                              u64 pos, u64 cos, u64 sin, float scale, int splits, u64 ws, u64 st, int kv8) {
    return dnn_attn_decode_qkv(CP(qkv), ldqkv, P(kc), P(vc), P(o), B, H, Hkv, hd, S, CIP(pos), CFP(cos), CFP(sin),
                               scale, splits, FP(ws), ST(st), kv8);
  }, py::arg("qkv"), py::arg("ldqkv"), py::arg("kc"), py::arg("vc"), py::arg("o"), py::arg("B"), py::arg("H"),
     py::arg("Hkv"), py::arg("hd"), py::arg("S"), py::arg("pos"), py::arg("cos"), py::arg("sin"), py::arg("scale"),
     py::arg("splits"), py::arg("ws"), py::arg("st"), py::arg("kv8") = 0);
  m.def("sample_topk", [](u64 x, int ld, int M, int N, u64 out, float temperature, int topk, unsigned seed, u64 step,
                          u64 st) {
    return dnn_sample_topk(CP(x), ld, M, N, reinterpret_cast<int*>(out), temperature, topk, seed,
                           reinterpret_cast<const int*>(step), ST(st));
  });
  m.def("argmax_rows", [](u64 x, int ld, int M, int N, u64 out, int f32in, u64 st, u64 out2, u64 pos_inc, u64 part,
                          u64 hist, int hist_ld) {
    return dnn_argmax_rows(CP(x), ld, M, N, IP(out), f32in, ST(st), IP(out2), IP(pos_inc),
                           reinterpret_cast<void*>(static_cast<uintptr_t>(part)), IP(hist), hist_ld);
  }, py::arg("x"), py::arg("ld"), py::arg("M"), py::arg("N"), py::arg("out"), py::arg("f32in"), py::arg("st"),
     py::arg("out2") = 0, py::arg("pos_inc") = 0, py::arg("part") = 0, py::arg("hist") = 0, py::arg("hist_ld") = 0);
  m.def("quant_fp8_rows", [](u64 x, int ldx, u64 q, u64 scale, int M, int K, int kpad, u64 st, int split) {
    return dnn_quant_fp8_rows(CP(x), ldx, P(q), FP(scale), M, K, kpad, ST(st), split);
  }, py::arg("x"), py::arg("ldx"), py::arg("q"), py::arg("scale"), py::arg("M"), py::arg("K"), py::arg("kpad"),
     py::arg("st"), py::arg("split") = 0);
  m.def("gemm_fp8", [](u64 A, u64 sa, u64 W, u64 sw, u64 C, int ldc, u64 bias, u64 R, int ldr, int M, int N, int K,
                       int act, u64 st) {
    return dnn_gemm_fp8(CP(A), CFP(sa), CP(W), CFP(sw), P(C), ldc, CFP(bias), CP(R), ldr, M, N, K, act, ST(st));
  });
#endif

  // ---- native RCCL data plane (csrc/comm/p2p.cpp) ----
  m.def("comm_available", []() { return dnn_comm_available(); });
  m.def("comm_last_error", []() { return std::string(dnn_comm_last_error()); });
  m.def("comm_unique_id", []() {
    char id[128];
    if (dnn_comm_unique_id(id) != 0) throw std::runtime_error(dnn_comm_last_error());
    return py::bytes(id, 128);
  });
  m.def("comm_create", [](py::bytes id, int nranks, int rank, int device, int async) {
    std::string s = id;
    if (s.size() != 128) throw std::runtime_error("comm_create: the unique id must be 128 bytes");
    long long h;
    {
      py::gil_scoped_release nogil;
      h = dnn_comm_create(s.data(), nranks, rank, device, async);
    }
    if (h == 0) throw std::runtime_error(dnn_comm_last_error());
    return h;
  });
  m.def("comm_wait_ready", [](long long h, int timeout_ms) { return dnn_comm_wait_ready(h, timeout_ms); },
        py::call_guard<py::gil_scoped_release>());
  // posts release the GIL: one waiting on a completed ring slot must never
  // keep the watchdog thread from running abort_all
  m.def("comm_post", [](long long h, int kind, u64 ptr, long long bytes, int peer, u64 st, int on_stream) {
    return dnn_comm_post(h, kind, P(ptr), bytes, peer, ST(st), on_stream);
  }, py::call_guard<py::gil_scoped_release>());
  m.def("comm_group", [](long long h, std::vector<int> kinds, std::vector<u64> ptrs, std::vector<long long> bytes,
                         std::vector<int> peers, u64 st, int on_stream) {
    const size_t n = kinds.size();
    if (ptrs.size() != n || bytes.size() != n || peers.size() != n) throw std::runtime_error("comm_group: ragged op lists");
    std::vector<void*> p(n);
    for (size_t i = 0; i < n; ++i) p[i] = P(ptrs[i]);
    py::gil_scoped_release nogil;
    return dnn_comm_group(h, (int)n, kinds.data(), p.data(), bytes.data(), peers.data(), ST(st), on_stream);
  });
  m.def("comm_wait", [](long long h, long long tok, u64 st) { return dnn_comm_wait(h, tok, ST(st)); });
  m.def("comm_query", [](long long h, long long tok) { return dnn_comm_query(h, tok); });
  m.def("comm_sync", [](long long h, long long tok, int timeout_ms) { return dnn_comm_sync(h, tok, timeout_ms); },
        py::call_guard<py::gil_scoped_release>());
  m.def("comm_async_error", [](long long h) { return dnn_comm_async_error(h); });
  m.def("comm_abort", [](long long h) { return dnn_comm_abort(h); }, py::call_guard<py::gil_scoped_release>());
  m.def("comm_destroy", [](long long h) { return dnn_comm_destroy(h); }, py::call_guard<py::gil_scoped_release>());
  m.def("comm_stats", [](long long h) {
    long long o[4] = {0, 0, 0, 0};
    dnn_comm_stats(h, o);
    return py::make_tuple(o[0], o[1], o[2], o[3]);
  });
}
