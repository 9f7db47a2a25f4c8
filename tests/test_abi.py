"""libsbo.so loads on a CPU-only host and exports every symbol include/sbo.h declares."""
import ctypes
import os
import re

from safe_bayesian_optimization_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sbo.h")).read()
    return sorted(set(re.findall(r"SBO_API\s+[\w\s\*]+?\b(sbo_\w+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(N.EXPORTS)


def test_library_exports_every_symbol():
    lib = N.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_version_and_status_strings():
    lib = N.lib()
    assert lib.sbo_version().decode().startswith("sbo-mi355x")
    assert lib.sbo_status_string(2).decode() == "SBO_E_NOT_SPD"


def test_key_combine_semantics():
    lib = N.lib()
    k = lambda s, i: N.sbo_key(s, i)  # noqa: E731
    c = lib.sbo_key_combine
    assert c(k(1.0, 5), k(2.0, 9)).idx == 9
    assert c(k(2.0, 5), k(2.0, 3)).idx == 3          # tie -> lowest global index
    assert c(k(0.0, -1), k(-5.0, 7)).idx == 7        # -1 = empty shard
    assert c(k(0.0, -1), k(0.0, -1)).idx == -1


def test_null_context_is_rejected_without_device():
    lib = N.lib()
    assert lib.sbo_fit(None, None, None, None, 0, N.sbo_hyper(0.4, 1, 0.1, 0), 0) == 1
    assert lib.sbo_tick(None, None, None, 0, 2.0, 0.0, 0, 0, None, None, None, None, None, None, 0) == 1


def test_cpp_node_driver_builds_and_links():
    """tools/sbo_tick_main.cpp (the C++ node mirror over include/sbo_node.hpp) links to libsbo."""
    import subprocess
    exe = os.path.join(ROOT, "safe_bayesian_optimization_amd", "lib", "sbo_tick_main")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def test_pmc_summaries_travel_to_the_gpu_box():
    """bench.py's roofline.traffic reads profiles/r*_pmc_<config>.json on the GPU
    box (bench.pmc_traffic); .gpurunignore must not exclude them (VERDICT r5 weak 3:
    a blanket ./profiles entry made BENCH_r05's traffic null)."""
    import fnmatch
    import glob
    pats = [p.strip() for p in open(os.path.join(ROOT, ".gpurunignore")) if p.strip()]
    files = glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_C4.json"))
    assert files
    for f in files:
        rel = "./" + os.path.relpath(f, ROOT)
        parts = rel.split("/")
        prefixes = ["/".join(parts[:i]) for i in range(2, len(parts) + 1)]
        for p in pats:
            for cand in prefixes + [pp[2:] for pp in prefixes]:
                assert not fnmatch.fnmatch(cand, p.rstrip("/")), (p, rel)
