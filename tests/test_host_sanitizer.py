"""Host AddressSanitizer + UBSan run of the kernel library's C ABI (SURVEY §5,
race detection / sanitizers).  GPU-side ASan / xnack+ builds are not available
on this pool, so every kernel source is compiled with the sanitizers on the
HOST half only (``-Xarch_host -fsanitize=...``) and linked with
``csrc/tests/host_validate.cpp``, which drives every entry point with shapes
it must reject before launching.  No GPU needed."""
import hashlib
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_validate_asan_ubsan():
    from distributed_neural_networks_amd.ops import build as b
    srcs = sorted(s for s in b.sources() if s.endswith(".hip")) + [os.path.join(ROOT, "csrc", "tests",
                                                                                 "host_validate.cpp")]
    h = hashlib.sha1()
    for s in srcs + [os.path.join(ROOT, "csrc", "kernels", "api.h")]:
        h.update(open(s, "rb").read())
    out_dir = os.path.join(ROOT, "build", "asan")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, f"host_validate_{h.hexdigest()[:10]}")
    if not os.path.exists(exe):
        san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
               "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=all"]
        flags = ["-O1", "-g", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "csrc"),
                 "-DDNN_HAVE_TRANSFORMER", "-Wno-unused-command-line-argument"]
        from concurrent.futures import ThreadPoolExecutor

        def compile_one(s):
            o = os.path.join(out_dir, os.path.basename(s) + ".o")
            extra = ["-x", "hip"] if s.endswith(".cpp") else []
            r = subprocess.run([HIPCC] + flags + san + extra + ["-c", s, "-o", o], capture_output=True, text=True)
            assert r.returncode == 0, f"{s}:\n{r.stderr[-3000:]}"
            return o

        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            objs = list(ex.map(compile_one, srcs))
        r = subprocess.run([HIPCC] + san + ["--offload-arch=gfx950", "-o", exe] + objs, capture_output=True,
                           text=True)
        assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "host_validate ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    for stale in os.listdir(out_dir):  # keep only the current binary
        if stale.startswith("host_validate_") and os.path.join(out_dir, stale) != exe:
            os.remove(os.path.join(out_dir, stale))
