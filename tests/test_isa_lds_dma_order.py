"""Static race check of the decode GEMMs' LDS-DMA images (CPU only:
hipcc cross-compiles gfx950 device assembly, nothing runs on a GPU).

gemm_oneshot.h issues each wave's activation image by LDS-DMA and then every
weight load.  The kernel reads an image only after composable_kernel's
direct-load sequence (vmcnt(0), lgkmcnt(0), s_barrier; gemm_oneshot.h
"Retiring the image"), not after a count of the weights issued behind it:
an LDS-DMA is not ordered with the plain loads that follow it.  This check
reads the assembly of the product instantiations (the planned GPT-2 / GPT-2
XL decode configurations and the forced test shapes) and of the fused LM head
(gemm_head.h, one image per K pass) and asserts, on every control-flow path,
that no LDS read follows an LDS-DMA without a vmcnt(0) and then an s_barrier
in between.  The round-4/5 counted-wait variant (probe bit ABL 128) is
compiled too and must be flagged, so the check is known to see what it
guards.

The same assembly (built with the library's own flags, ops/build.py) must hold
no cross-half packed FP32 op (v_pk_*_f32 ... op_sel:[...]): the SLP
vectoriser's packed subtracts in the row statistics were the rounds-5/6 "race"
(gemm_oneshot.h "The race of rounds 5-6", profiles/r6_oneshot_race_root_cause.md);
an SLP build of the same kernels must show them, so that check also sees what
it guards.  (The GPU-side screens: bench/probes/oneshot_race_probe.py and
tests/test_stream_gemm_gpu.py::test_oneshot_coresident_race_screen.)
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
RACY = [(2, 1, "false", 2, "ACT_GELU", "false", 1, 128), (1, 2, "true", 0, "ACT_NONE", "false", 2, 128)]
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


def _lib_flags():
    import sys
    sys.path.insert(0, ROOT)
    from distributed_neural_networks_amd.ops.build import PER_FILE_FLAGS
    return PER_FILE_FLAGS["gemm_skinny.hip"]


_ASM = {}


def _asm(extra=None):
    extra = _lib_flags() if extra is None else extra
    key = " ".join(extra)
    if key not in _ASM:
        _ASM[key] = _asm_build(extra)
    return _ASM[key]


def _asm_build(extra):
    items = ", ".join([f"(void*)&gemm_oneshot_kernel<{mt}, {ntw}, {w8}, {norm}, {act}, {split}, {steps}>"
                       for mt, ntw, w8, norm, act, split, steps in CONFIGS] +
                      [f"(void*)&gemm_oneshot_kernel<{mt}, {ntw}, {w8}, {norm}, {act}, {split}, {steps}, {abl}>"
                       for mt, ntw, w8, norm, act, split, steps, abl in RACY] +
                      [f"(void*)&gemm_head_kernel<{w8}, {norm}, {nch}, {cpp}, {gs}>" for w8, norm, nch, cpp, gs in HEADS])
    d = tempfile.mkdtemp(prefix="dnn_isa_")
    src, out = os.path.join(d, "oneshot_isa.hip"), os.path.join(d, "oneshot_isa.s")
    with open(src, "w") as f:
        f.write(SRC.format(items=items))
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "csrc"), "-Wno-unused-result", "-Wno-pass-failed"] + list(extra) +
                       ["-o", out, src],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(out) as f:
        text = f.read()
    shutil.rmtree(d, ignore_errors=True)
    return text


def _kernels(text, kernel="gemm_oneshot_kernel", raw=False):
    """{mangled name: [memory / wait instructions in program order]} (raw:
    every label and instruction, for the control-flow scan)"""
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
        t = line.split(";")[0].strip()
        if raw:
            if t and not t.startswith("."):
                out[name].append(t)
            elif re.match(r"^\.LBB\w+:", t):
                out[name].append(t)
        elif re.match(r"(global_load|buffer_load|ds_read|s_waitcnt)", t):
            out[name].append(t)
    return out


def _product(ks):
    """Drop the probe instantiations (ABL != 0: a ninth template argument)."""
    return {n: q for n, q in ks.items() if not re.search(r"ELi128EE", n)}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_oneshot_image_dma_issued_first():
    """The image DMAs form one run (no load in between): every weight load is
    issued after the whole image, as the kernel's issue order intends."""
    ks = _product(_kernels(_asm()))
    assert len(ks) == len(CONFIGS), sorted(ks)
    for name, seq in ks.items():
        dma = [i for i, t in enumerate(seq) if "global_load_lds" in t]
        assert dma, name
        between = [t for t in seq[dma[0]:dma[-1]] if t.startswith(("global_load", "buffer_load")) and "lds" not in t]
        assert not between, f"{name}: loads interleaved with the image DMA: {between[:4]}"


def _unretired_reads(lines, barriers: int = 1):
    """LDS reads that some path reaches after an LDS-DMA without vmcnt(0) and
    then s_barrier in between: a forward may-analysis over the kernel's
    basic blocks (labels, s_branch / s_cbranch_*, s_endpgm)."""
    blocks, labels, cur = [], {}, []
    for t in lines:  # split into basic blocks
        if t.endswith(":"):
            if cur:
                blocks.append(cur)
            cur = []
            labels[t[:-1]] = len(blocks)
            continue
        cur.append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm")):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    # labels index the block that starts after them
    succ = []
    for i, b in enumerate(blocks):
        last = b[-1] if b else ""
        nxt = [i + 1] if i + 1 < len(blocks) else []
        m = re.match(r"s_(c?)branch\w*\s+(\.LBB\w+)", last)
        if last.startswith("s_endpgm"):
            succ.append([])
        elif m:
            tgt = labels.get(m.group(2))
            succ.append(([tgt] if tgt is not None else []) + (nxt if m.group(1) else []))
        else:
            succ.append(nxt)
    # a block's entry state is the worst over its predecessors;
    # encoded state: 0 clear, 2 + barriers pending, or 1 .. barriers (barriers still needed
    # after the wait); a higher value is worse
    top = barriers + 1
    entry = [0] * len(blocks)
    bad, work = set(), list(range(len(blocks)))
    while work:
        i = work.pop(0)
        st = entry[i]
        for j, t in enumerate(blocks[i]):
            if "global_load_lds" in t or (t.startswith("buffer_load") and " lds" in t):
                st = top
            elif t.startswith("s_waitcnt") and re.search(r"vmcnt\(0\)", t):
                st = min(st, barriers)
            elif t.startswith("s_barrier") and 0 < st < top:
                st -= 1
            elif t.startswith("ds_read") and st:
                bad.add((i, j, t))
        for k in succ[i]:
            if st > entry[k]:
                entry[k] = st
                work.append(k)
    return sorted(bad)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_lds_dma_images_retired_before_reads():
    text = _asm()
    for kernel, n in (("gemm_oneshot_kernel", len(CONFIGS)), ("gemm_head_kernel", len(HEADS))):
        ks = _product(_kernels(text, kernel, raw=True))
        assert len(ks) == n, (kernel, sorted(ks))
        for name, seq in ks.items():
            assert any("global_load_lds" in t for t in seq), name
            bad = _unretired_reads(seq, 1)
            assert not bad, f"{name}: {len(bad)} LDS reads before the image DMA is retired: {bad[:3]}"
    # the racy variants must be flagged (the check sees the bug): the counted
    # wait (ABL 128)
    racy = {n: q for n, q in _kernels(text, raw=True).items() if n not in _product({n: q})}
    assert len(racy) == len(RACY), sorted(racy)
    for name, seq in racy.items():
        assert _unretired_reads(seq, 1), f"{name}: counted-wait variant not flagged"

PK_CROSS = re.compile(r"^v_pk_\w+_f32\b.*\bop_sel:\[")


def _cross_half(text):
    return {n: [t for t in seq if PK_CROSS.match(t)] for n, seq in _product(_kernels(text, raw=True)).items()}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_oneshot_no_cross_half_packed_fp32():
    """The one-shot kernels as the library builds them hold no cross-half
    packed FP32 op; the same source with the SLP vectoriser on does (the
    row-statistics subtracts), so the check sees what it guards."""
    assert "-fno-slp-vectorize" in _lib_flags()
    got = _cross_half(_asm())
    assert len(got) == len(CONFIGS), sorted(got)
    bad = {n: v[:2] for n, v in got.items() if v}
    assert not bad, bad
    slp = _cross_half(_asm(["-fslp-vectorize"]))
    assert sum(bool(v) for v in slp.values()) >= 1, "the SLP control build shows no cross-half packed op"
