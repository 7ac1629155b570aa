"""CPU sanitizer builds of the C++ host runtime: ASan+UBSan and TSan builds of a
threaded stress driver (parallel safetensors copy_many, tree-parallel BLAKE3 from several threads,
the shared BPE cache under concurrent encodes). Any sanitizer report aborts the binary."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("kinds", ["address,undefined", "thread"])
def test_runtime_stress_under_sanitizer(kinds, tmp_path):
    import build_native
    exe = build_native.build_sanitized(kinds)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), "8"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "stress ok" in r.stdout
