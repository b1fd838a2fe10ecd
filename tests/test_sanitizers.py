"""Host-code sanitizers (race detection / sanitizers): the product's host symbolic analysis
(uno_amd/csrc/analysis.cpp), the multi-threaded CPU baseline and the oracle built with
-fsanitize=address,undefined (oracle/Makefile `asan`) and run on known-answer, random and arrowband
systems (oracle/sanitize_main.cpp).  Device code is not sanitized (GPU ASan is not available on the pool)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="4")
    out = subprocess.run([os.path.join(ROOT, "oracle", "_asan", "sanitize_main")], capture_output=True, text=True,
                         env=env, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "runtime error" not in out.stderr and "ERROR: AddressSanitizer" not in out.stderr, out.stderr[-4000:]
    assert out.stdout.count(" ok") >= 8, out.stdout
