"""GPU: the C ABI from a C/C++ caller with no Python in the process (examples/capi_check,
hipcc + include/ina.h + libina.so): quantise -> 8-way sum-reduce -> NGA-256 pack ->
unpack -> dequantise, checked against host arithmetic inside the binary, plus the
error-code path."""
import os
import subprocess

import pytest

from tests.conftest import REPO

pytestmark = pytest.mark.gpu

BIN = os.path.join(REPO, "examples", "capi_check")


def test_c_caller_end_to_end():
    assert os.path.exists(BIN), "examples/capi_check not built (make -C examples / __graft_entry__.build())"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
