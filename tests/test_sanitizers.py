"""Host code under ASan + UBSan: the instrumented builds
(libsbo_asan.so: frontier.cpp, polygeom.cpp and the host paths of sbo_api.cpp;
liboracle_asan.so) are loaded with clang's ASan runtime preloaded, the CPU
tests of those libraries run clean, and an out-of-bounds read is caught (so
the instrumentation is live).  tools/asan_check.sh runs the whole CPU suite
the same way."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
pytestmark = pytest.mark.skipif(not RT or not os.path.exists("/opt/rocm/bin/hipcc"), reason="no clang ASan runtime")


@pytest.fixture(scope="module")
def san_env():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "safe_bayesian_optimization_amd"), "asan"],
                   check=True, capture_output=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=RT[-1], ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:exitcode=97",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=98",
               SBO_LIB=os.path.join(ROOT, "safe_bayesian_optimization_amd", "lib", "libsbo_asan.so"),
               ORC_LIB=os.path.join(ROOT, "oracle", "liboracle_asan.so"))
    return env


def test_host_code_clean_under_asan_ubsan(san_env):
    tests = [os.path.join(ROOT, "tests", t) for t in
             ("test_frontier.py", "test_polygeom.py", "test_oracle_golden.py", "test_abi.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider", *tests],
                       cwd=ROOT, env=san_env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_instrumentation_is_live(san_env):
    code = ("import numpy as np\n"
            "from safe_bayesian_optimization_amd import _native as N\n"
            "assert N.LIB_PATH.endswith('libsbo_asan.so')\n"
            "x = np.zeros(4); s = np.ones(4, np.uint8)\n"
            "N.lib().sbo_next_subgoal(x.ctypes.data, x.ctypes.data, x.ctypes.data, x.ctypes.data, s.ctypes.data,"
            " 64, 8, 8, 0.0, 0.0)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=san_env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode in (97, 98) and "heap-buffer-overflow" in r.stderr, r.stderr[-2000:]
