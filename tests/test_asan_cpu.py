"""SURVEY §5 sanitizers: the C ABI's host-side argument checks built with
AddressSanitizer (`make asan`: the library's host code and tests/abi_check.c
with -fsanitize=address; device code unchanged, no GPU sanitizer) and driven
without a GPU: every invalid call is rejected with an error code and message
before any HIP call, zero-work calls succeed, and ASan reports nothing."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "adaptive-volume-rendering_amd")


def test_abi_argument_checks_under_asan():
    b = subprocess.run(["make", "-C", PKG, "asan", "-j8"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([os.path.join(PKG, "build", "abi_check_asan")], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "abi_check: 0 failure(s)" in r.stdout
    assert "AddressSanitizer" not in r.stderr
