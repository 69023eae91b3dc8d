"""CPU: the oracle and the workload generator under ASan + UBSan.

Host code only (GPU sanitizers are not available on the pool).  oracle/sanitize_driver.c
encodes a sweep of random streams (every subframe type, stereo mode, RICE2/escapes, wasted
bits, variable blocksizes, 8..24 bits, 1..8 channels), decodes them through the oracle's
state machine in both C# driving patterns, replays the FLACDecoder / FLACFileReader surfaces
and decodes corrupted and truncated copies.  A sanitizer report aborts the driver.
"""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_and_generator_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "build", "sanitize_driver"), "120"], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
