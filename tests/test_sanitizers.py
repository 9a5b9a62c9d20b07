"""The host C++ of libart under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5,
tools/asan/): the batched tree driver (art_forest.cpp) on the oracle's CPU segments --
forward trees, Monte-Carlo branches, the backtrace, saveMode 3 data, determinism and the
error paths -- and the C boundary (art_capi.cpp): its host entry points and every argument
check. Any sanitizer report fails the run (UBSan without recovery, LeakSanitizer on for
the driver with third-party runtimes suppressed)."""
import os
import shutil
import subprocess

import pytest

ASAN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "asan")
pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None,
                                reason="needs hipcc and make")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-C", ASAN, "-j4"], check=True, capture_output=True)
    return ASAN


@pytest.mark.parametrize("exe,leaks,ok", [("forest_asan", 1, "forest OK"), ("capi_asan", 0, "capi OK")])
def test_host_code_is_sanitizer_clean(built, exe, leaks, ok):
    env = dict(os.environ, ASAN_OPTIONS=f"detect_leaks={leaks}:abort_on_error=0",
               LSAN_OPTIONS=f"suppressions={os.path.join(built, 'lsan.supp')}",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(built, "build", exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and ok in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr
