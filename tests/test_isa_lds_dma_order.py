"""Static race check of the decode GEMMs' LDS-DMA images (CPU only:
hipcc cross-compiles gfx950 device assembly, nothing runs on a GPU).

gemm_oneshot.h issues each wave's activation image by LDS-DMA and then every
weight load, and retires the image with a *counted* wait: ``vmcnt(N)`` with N
the number of weight loads issued after it.  That wait covers the image only
if no other vector-memory load is issued between the first and the last
image DMA, and at least N loads follow the last one before the first LDS read
(a load sunk past the DMA by the compiler let the image be read before it
landed: the round-5 race fixed with ``sched_barrier``).  The check reads the
assembly of the product instantiations (the planned GPT-2 / GPT-2 XL decode
configurations and the forced test shapes) and asserts both, so a schedule
change that breaks the count fails here, on the CPU, rather than as rare
wrong tiles on the GPU.  (MI355X_MICROARCH.md item 7: nothing but the
issuing wave's covering vmcnt orders a ds_read behind a pending LDS-DMA.)
The fused LM head (gemm_head.h) stages its activation image the same way,
one image per K pass: every LDS read must come after a wait that retires
the pass's last DMA.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# <MT, NTW, W8, NORM, ACT, SPLIT, STEPS>: gemm_skinny.hip os_plan (planned
# shapes and the forced "every eligible shape" mode the GPU tests use)
CONFIGS = [
    (2, 2, "false", 2, "ACT_NONE", "false", 1),   # GPT-2 c_attn (folded LN)
    (2, 2, "false", 2, "ACT_GELU", "false", 1),   # GPT-2 c_fc (folded LN + GELU)
    (1, 1, "false", 0, "ACT_NONE", "false", 1),   # GPT-2 O (+ residual)
    (2, 1, "false", 2, "ACT_GELU", "false", 1),   # forced mode, N = 2304 / K = 768
    (2, 4, "true", 2, "ACT_NONE", "false", 2),    # GPT-2 XL c_attn (W8, two steps)
    (2, 4, "true", 2, "ACT_GELU", "false", 2),    # GPT-2 XL c_fc
    (1, 2, "true", 0, "ACT_NONE", "false", 2),    # GPT-2 XL O
    (2, 4, "true", 0, "ACT_NONE", "true", 2),     # split-K slab variant
]

# <W8, NORM, NCH, CPP, GS>: the GPT-2 and GPT-2 XL fp8 heads of the decode step
HEADS = [("false", 2, 24, 24, 12), ("true", 2, 25, 14, 5)]

SRC = """#include "kernels/gemm_oneshot.h"
#include "kernels/gemm_head.h"
namespace dnn {{
void* isa_keep[] = {{ {items} }};
}}
"""


def _asm():
    items = ", ".join([f"(void*)&gemm_oneshot_kernel<{mt}, {ntw}, {w8}, {norm}, {act}, {split}, {steps}>"
                       for mt, ntw, w8, norm, act, split, steps in CONFIGS] +
                      [f"(void*)&gemm_head_kernel<{w8}, {norm}, {nch}, {cpp}, {gs}>" for w8, norm, nch, cpp, gs in HEADS])
    d = tempfile.mkdtemp(prefix="dnn_isa_")
    src, out = os.path.join(d, "oneshot_isa.hip"), os.path.join(d, "oneshot_isa.s")
    with open(src, "w") as f:
        f.write(SRC.format(items=items))
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "csrc"), "-Wno-unused-result", "-Wno-pass-failed", "-o", out, src],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(out) as f:
        text = f.read()
    shutil.rmtree(d, ignore_errors=True)
    return text


def _kernels(text, kernel="gemm_oneshot_kernel"):
    """{mangled name: [memory / wait instructions in program order]}"""
    out, name = {}, None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S*" + kernel + r"\S*):", line)
        if m:
            name = m.group(1)
            out[name] = []
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            name = None
            continue
        t = line.strip()
        if re.match(r"(global_load|buffer_load|ds_read|s_waitcnt)", t):
            out[name].append(t)
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_oneshot_image_dma_retired_by_counted_wait():
    ks = _kernels(_asm())
    assert len(ks) == len(CONFIGS), sorted(ks)
    for name, seq in ks.items():
        dma = [i for i, t in enumerate(seq) if "global_load_lds" in t]
        assert dma, name
        first, last = dma[0], dma[-1]
        between = [t for t in seq[first:last] if t.startswith(("global_load", "buffer_load")) and "lds" not in t]
        assert not between, f"{name}: loads interleaved with the image DMA: {between[:4]}"
        # the first LDS read after the image: the vmcnt in force must be <= the
        # loads issued after the last DMA
        issued, wait = 0, None
        for t in seq[last + 1:]:
            if t.startswith(("global_load", "buffer_load")):
                issued += 1
            elif t.startswith("s_waitcnt") and "vmcnt" in t:
                wait = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            elif t.startswith("ds_read"):
                break
        assert wait is not None, f"{name}: no vmcnt wait before the first image read"
        assert wait <= issued, f"{name}: vmcnt({wait}) with only {issued} loads after the image DMA"


def _unretired_reads(seq):
    """Linear scan (the kernels' DMA phases are fully unrolled): LDS reads
    issued while an LDS-DMA may still be pending, i.e. before a vmcnt wait
    that leaves at most as many loads outstanding as were issued after the
    most recent DMA."""
    pending, after, bad = False, 0, []
    for t in seq:
        if "global_load_lds" in t or (t.startswith("buffer_load") and " lds" in t):
            pending, after = True, 0
        elif t.startswith(("global_load", "buffer_load")):
            after += 1
        elif t.startswith("s_waitcnt") and "vmcnt" in t:
            if pending and int(re.search(r"vmcnt\((\d+)\)", t).group(1)) <= after:
                pending = False
        elif t.startswith("ds_read") and pending:
            bad.append(t)
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_lds_dma_images_retired_before_reads():
    text = _asm()
    for kernel, n in (("gemm_oneshot_kernel", len(CONFIGS)), ("gemm_head_kernel", len(HEADS))):
        ks = _kernels(text, kernel)
        assert len(ks) == n, (kernel, sorted(ks))
        for name, seq in ks.items():
            assert any("global_load_lds" in t for t in seq), name
            bad = _unretired_reads(seq)
            assert not bad, f"{name}: {len(bad)} LDS reads before the image DMA is retired: {bad[:3]}"
