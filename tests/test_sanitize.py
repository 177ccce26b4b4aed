"""The host C/C++ layer under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md section 4
item 6): tests/c/sanitize.c built by `make -C tests/c sanitize` from host/*.c,
csrc/jpgx_plan.cpp and oracle/cpu_ref.c (no GPU), run on hostile BMP headers, every quality's
planning, the oracle's hot path with the modelled x0 = -8 underflow read (preprocess.c:159-160),
the Block/JpgData/dpcm/JFIF host API.  Any sanitizer report aborts the run."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None,
                    reason="needs gcc/g++ with libasan/libubsan")
def test_host_layer_under_asan_ubsan(tmp_path):
    b = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "c"), "sanitize"],
                       capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(REPO, "tests", "c", "_build", "sanitize"), str(tmp_path),
                        os.path.join(REPO, "tests", "golden", "images")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "sanitize: clean" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
