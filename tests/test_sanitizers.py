"""Host-code sanitizers: the C++ low-bit library (quantizers,
dequantizers, device-layout repack, CPU GEMMs) rebuilt with AddressSanitizer +
UndefinedBehaviorSanitizer and driven over randomised shapes by
csrc/selftest/host_selftest.cpp.  Host only: GPU kernels are covered by their
numerics tests (device-side sanitizers are not used on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ipex_llm_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_library_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_selftest")
    srcs = [os.path.join(CSRC, "selftest", "host_selftest.cpp"), os.path.join(CSRC, "cpu", "quant.cpp"),
            os.path.join(CSRC, "cpu", "gemm_q4.cpp")]
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-march=x86-64-v3", *san, "-I", CSRC, *srcs, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "33"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "0 failures" in r.stdout, r.stdout[-2000:] + r.stderr[-6000:]
