"""In-process A/B of the 256^2 GEMM against another build of gemm_bf16.hip
(``bench/libgemm_old.so``, called through ctypes with the same C entry point)
on the prefill epilogues (folded norm, GELU, residual) of the GPT-2 shapes.
One JSON line per shape.  Build the comparison library from any commit:

    git show <rev>:csrc/kernels/gemm_bf16.hip > /tmp/g.hip
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Icsrc/kernels /tmp/g.hip \
        csrc/kernels/gemm_skinny.hip -o bench/libgemm_old.so

(profiles/archive/r2_gemm_persist_vs_prior_ab.jsonl: the persistent-grid rewrite vs
the kernel before it — 8-21 % slower, reverted.)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SHAPES = [(32768, 2304, 768, "norm"), (32768, 3072, 768, "gelu+norm"), (32768, 2304, 768, "none"),
          (32768, 3072, 768, "gelu"), (32768, 768, 768, "res"), (32768, 768, 3072, "res")]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    from distributed_neural_networks_amd.ops.gemm import linear
    old = ctypes.CDLL(os.path.join(ROOT, "bench", "libgemm_old.so"))
    f = old.dnn_gemm_bf16
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    acts = {"none": 0, "relu": 1, "gelu": 2}
    for (M, N, K, epi) in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).bfloat16() if epi == "res" else None
        a = epi.split("+")[0]
        act = acts.get(a, 0)
        rs = cs = None
        if epi.endswith("norm"):
            mean, rstd = torch.randn(M, device=dev), torch.rand(M, device=dev) + 0.5
            rs, cs = torch.stack([rstd, -mean * rstd], 1).contiguous(), torch.randn(N, device=dev)
        o_new = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        o_old = torch.empty_like(o_new)

        def run_new():
            linear(x, w, bias, act=act, residual=r, out=o_new, rowstat=rs, colsum=cs)

        def run_old():
            rc = f(x.data_ptr(), K, w.data_ptr(), K, o_old.data_ptr(), N, bias.data_ptr(),
                   r.data_ptr() if r is not None else None, N if r is not None else 0, M, N, K, act, 0,
                   torch.cuda.current_stream().cuda_stream, None, rs.data_ptr() if rs is not None else None,
                   cs.data_ptr() if cs is not None else None)
            if rc != 0:
                raise RuntimeError(f"old gemm rc {rc}")
        t = {"new": [], "old": []}
        for _ in range(3):
            t["new"].append(timeit(run_new))
            t["old"].append(timeit(run_old))
        res = {"M": M, "N": N, "K": K, "epilogue": epi, "bit_identical": bool(torch.equal(o_new, o_old))}
        for k in ("old", "new"):
            ms = sorted(t[k])[1]
            res[f"{k}_ms"] = round(ms, 4)
            res[f"{k}_tflops"] = round(2.0 * M * N * K / ms / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
