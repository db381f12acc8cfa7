"""Sanitizer build of the host-side C++ (SURVEY.md §5 "race detection /
sanitizers"): the native runtime (cfd_runtime.cpp, Model::run's worker and
queues), the slab plan (slab_plan.h) and the mesher's host code
(cfd_mesh.hip: polygons, predicates, tesselation) compiled with
-fsanitize=address,undefined and driven on the CPU by tests/asan/asan_host.cpp
(the runtime over a stub model, from several threads at once).  A sanitizer
report or a failed check fails the test.  No GPU needed."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or not shutil.which("make"),
                    reason="needs hipcc (host-side sanitizer build)")
def test_host_code_under_asan_ubsan():
    b = subprocess.run(["make", "-s", "-j4", "-C", ASAN], capture_output=True, text=True,
                       timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    # verify_asan_link_order=0: a preloaded library ahead of the sanitizer
    # runtime (if the environment has one) is tolerated, not removed
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ASAN, "_build", "asan_host")], capture_output=True,
                       text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "asan_host ok" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
