"""Host-code sanitizer tier: the native library's host entry
points (multi-threaded LIBSVM parser, TD-PPR / local clustering, host RNG)
built with AddressSanitizer + UndefinedBehaviorSanitizer and, separately,
ThreadSanitizer (hipcc, sanitizers on the host side only: -Xarch_host), then
driven by tests/native/sanitize_host.cpp.  GPU kernels are covered by the
gpu tier (device sanitizers are not available on the GPU pool)."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "libskylark_amd", "_native")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
VARIANTS = {
    "asan_ubsan": (["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"],
                   ["-fsanitize=address,undefined"]),
    "tsan": (["-Xarch_host", "-fsanitize=thread"], ["-fsanitize=thread"]),
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_host_code_under_sanitizers(tmp_path, variant):
    from libskylark_amd.ml.graph import _setup
    N, D, _, Cc = _setup(0.85, 5.0, 1e-3, 4)
    op = tmp_path / "op.bin"
    with open(op, "wb") as f:
        f.write(struct.pack("<ii", N, 4) + struct.pack("<d", Cc) + np.ascontiguousarray(D, np.float64).tobytes())
    cflags, lflags = VARIANTS[variant]
    exe = tmp_path / f"san_{variant}"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *cflags, "-Xarch_host",
           "-fno-omit-frame-pointer", "-I", os.path.join(SRC, "include"), "-x", "hip",
           os.path.join(ROOT, "tests", "native", "sanitize_host.cpp"),
           os.path.join(SRC, "src", "libsvm_io.cpp"), os.path.join(SRC, "src", "graph_local.cpp"),
           os.path.join(SRC, "src", "rng_kernels.hip"), "-o", str(exe), *lflags, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    for args in ([str(op)], []):          # real collocation operator, then a deliberately bad one
        run = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=180, env=env)
        assert run.returncode == 0, run.stdout[-2000:] + run.stderr[-4000:]
        assert "sanitize_host ok" in run.stdout
        assert "Sanitizer" not in run.stderr, run.stderr[-4000:]
