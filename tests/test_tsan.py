"""Host code under ThreadSanitizer: `make tsan` builds the product's code
model and the oracle with -fsanitize=thread, and tests/tsan/tsan_check.cpp drives them from 8
threads over shared code objects (the reference's one-decoder-per-thread structure,
QEC_LDPC/DecoderCPU.h:419-438).  No report, and every thread agrees with a serial run."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tsan_bin():
    r = subprocess.run(["make", "-s", "tsan"], cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0 and "fsanitize" in r.stderr and "not" in r.stderr:
        pytest.skip("no ThreadSanitizer runtime: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return os.path.join(ROOT, "build", "tsan", "tsan_check")


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_host_code_is_race_free(tsan_bin, code_paths, key):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([tsan_bin, code_paths[key]], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "tsan ok" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr
