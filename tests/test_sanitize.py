"""ASan + UBSan run of the host C++ (csrc/graph.cpp, csrc/cpu_backend.cpp) and of the
oracle's C restatement: tests/sanitize/san_main.cpp builds graphs, runs the
_cpu message passing against the oracle and the oracle's ECC / perturbation loops; any
sanitizer report fails the process."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="4")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(HERE, "build", "san_main")], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
