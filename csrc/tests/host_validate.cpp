// Host-side validation of the kernel C ABI under AddressSanitizer / UBSan
// (tests/test_host_sanitizer.py builds this with `-Xarch_host -fsanitize=...`:
// the GPU sanitizer is not available on this pool, so the host half of every
// entry point — shape checks, config tables, the guards that keep a kernel
// from being launched with operands its grid does not cover — is what runs
// instrumented).  Every call below must be REJECTED before any launch, so the
// program needs no GPU.  Prints "host_validate ok" and exits 0 on success.
#include <cstdio>

#include "../kernels/api.h"

static int g_fail = 0;

// Rejections are negative; 0 or a positive hipError_t means a launch was
// attempted (with no GPU it fails), i.e. the guard did not catch the shape.
static void expect_reject(int rc, const char* what) {
  if (rc >= 0) {
    std::printf("NOT REJECTED: %s (rc=%d)\n", what, rc);
    ++g_fail;
  }
}

static void expect_noop(int rc, const char* what) {
  if (rc != 0) {
    std::printf("empty problem should be a no-op: %s (rc=%d)\n", what, rc);
    ++g_fail;
  }
}

int main() {
  char buf[64] = {0};
  void* p = buf;
  float* f = reinterpret_cast<float*>(buf);
  int* ip = reinterpret_cast<int*>(buf);
  hipStream_t st = nullptr;
  // GEMMs
  expect_reject(dnn_gemm_bf16(p, 96, p, 96, p, 8, nullptr, nullptr, 0, 128, 128, 96, 0, 0, st), "gemm K%64");
  expect_reject(dnn_gemm_bf16(p, 64, p, 64, p, 8, nullptr, nullptr, 0, 0, 128, 64, 0, 0, st), "gemm M=0");
  expect_reject(dnn_gemm_set_tile(64), "gemm tile 64");
  expect_reject(dnn_gemm_skinny(p, 64, nullptr, p, 64, nullptr, p, 8, nullptr, nullptr, 0, 257, 16, 64, 0, 0, 0, st),
                "skinny M>256");
  expect_reject(dnn_gemm_skinny(p, 64, f, p, 64, f, p, 8, nullptr, nullptr, 0, 65, 16, 64, 0, 0, 1, st),
                "skinny fp8 M>64");
  expect_reject(dnn_gemm_skinny(p, 64, nullptr, p, 64, nullptr, p, 8, nullptr, nullptr, 0, 4, 16, 64, 0, 0, 1, st),
                "skinny fp8 without scales");
  expect_reject(dnn_gemm_skinny(p, 48, nullptr, p, 48, nullptr, p, 8, nullptr, nullptr, 0, 4, 24, 48, 3, 0, 0, st),
                "skinny silu N%16");
  expect_reject(dnn_gemm_skinny_norm(p, 64, p, 64, p, 8, nullptr, nullptr, 0, 4, 16, 64, 0, 2, nullptr, 1e-5f, st),
                "skinny LN without colsum");
  expect_reject(dnn_gemm_skinny_norm(p, 64, p, 64, p, 8, nullptr, nullptr, 0, 4, 16, 64, 2, 1, nullptr, 1e-5f, st),
                "skinny norm unsupported act");
  expect_reject(dnn_gemm_skinny_w8(p, 96, p, 96, f, p, 8, nullptr, nullptr, 0, 4, 16, 96, 0, 0, nullptr, 0.f, st),
                "w8 K%64");
  expect_reject(dnn_gemm_skinny_w8(p, 64, p, 32, f, p, 8, nullptr, nullptr, 0, 4, 16, 64, 0, 0, nullptr, 0.f, st),
                "w8 ldw < K");
  expect_reject(dnn_gemm_skinny_w8(p, 64, p, 64, nullptr, p, 8, nullptr, nullptr, 0, 4, 16, 64, 0, 0, nullptr, 0.f,
                                   st), "w8 without scales");
  expect_reject(dnn_gemm_skinny_sweep(p, 64, p, 64, nullptr, p, 8, 4, 16, 64, 1, 2, 16, 0, 0, st), "sweep ks>8");
  expect_reject(dnn_gemm_fp8(p, f, p, f, p, 8, nullptr, nullptr, 0, 128, 128, 96, 0, st), "fp8 K%128");
  expect_reject(dnn_gemm_fp8(p, f, p, f, p, 8, nullptr, nullptr, 0, 128, 24, 128, 3, st), "fp8 silu N%16");
  expect_reject(dnn_quant_fp8_rows(p, 12, p, f, 4, 12, 128, st), "quant K%8");
  expect_reject(dnn_quant_fp8_rows(p, 256, p, f, 4, 256, 128, st), "quant kpad<K");
  // norms / embedding
  expect_reject(dnn_layernorm(p, 12, f, f, p, 12, 4, 12, 1e-5f, 0, st), "layernorm N%8");
  expect_reject(dnn_layernorm(p, 16384, f, f, p, 16384, 4, 16384, 1e-5f, 1, st), "layernorm N>8192");
  expect_reject(dnn_embed_gpt2(ip, p, p, p, 1, 1, 12, ip, 8, 8, st), "embed d%8");
  expect_reject(dnn_embed_gpt2(ip, p, p, p, 1, 1, 16, ip, 0, 8, st), "embed empty vocab");
  // attention
  expect_reject(dnn_qkv_split(p, p, p, p, 1, 1, 4, 4, 24, 16, ip, nullptr, nullptr, 0, st), "qkv_split hd%16");
  expect_reject(dnn_qkv_split(p, p, p, p, 1, 1, 6, 4, 64, 16, ip, nullptr, nullptr, 0, st), "qkv_split H%Hkv");
  expect_reject(dnn_flash_attn(p, p, p, p, 1, 8, 6, 4, 64, 16, ip, 0.1f, st), "flash H%Hkv");
  expect_reject(dnn_flash_attn(p, p, p, p, 1, 8, 4, 4, 96, 16, ip, 0.1f, st), "flash hd=96");
  expect_reject(dnn_attn_decode(p, p, p, p, 1, 4, 4, 64, 16, ip, 0.1f, 0, f, st), "decode splits=0");
  expect_reject(dnn_attn_decode(p, p, p, p, 1, 32, 2, 64, 16, ip, 0.1f, 1, f, st), "decode G>8");
  expect_reject(dnn_attn_decode(p, p, p, p, 1, 4, 4, 96, 16, ip, 0.1f, 1, f, st), "decode hd=96");
  expect_reject(dnn_attn_decode(p, p, p, p, 1, 8, 2, 64, 16, ip, 0.1f, 1, f, st, 1), "decode fp8 KV, GQA at hd 64");
  expect_reject(dnn_attn_decode_qkv(p, 100, p, p, p, 1, 4, 4, 64, 16, ip, nullptr, nullptr, 0.1f, 1, f, st),
                "decode_qkv ldqkv too small");
  // sampling
  expect_reject(dnn_sample_topk(p, 16, 2, 16, ip, 0.f, 0, 1u, nullptr, st), "sample temperature 0");
  expect_reject(dnn_sample_topk(p, 12, 2, 12, ip, 1.f, 0, 1u, nullptr, st), "sample ld%8");
  expect_reject(dnn_argmax_rows(p, 12, 2, 12, ip, 0, st), "argmax bf16 ld%8");
  expect_noop(dnn_argmax_rows(p, 16, 0, 16, ip, 0, st), "argmax M=0");
  // CIFAR
  expect_reject(dnn_cifar_set_v4_pt(3), "v4 pt%4");
  expect_reject(dnn_cifar_set_v4_pt(36), "v4 pt>32");
  expect_noop(dnn_cifar_stage0_v4(f, p, p, f, p, f, 0, 0, st), "stage0 B=0");
  expect_noop(dnn_cifar_head_tail(p, p, f, f, ip, 0, st), "head B=0");
  if (g_fail) {
    std::printf("host_validate FAILED (%d)\n", g_fail);
    return 1;
  }
  std::printf("host_validate ok\n");
  return 0;
}
