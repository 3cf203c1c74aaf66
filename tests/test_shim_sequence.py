"""The cgo shim's call sequence made from C through the
C-ABI (tests/harness/shim_sequence.c): per-object Encrypt/Decrypt, per-block
calls through the aggregator with descriptors in C memory and data in the
pinned pool (the cgo pointer rule), the same over the multi-device context,
checksum() and the ReadAt verify -- all checked against the oracle."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "harness", "shim_sequence")


def test_shim_harness_is_built_and_links():
    """Built by __graft_entry__.build() (tests/harness/Makefile); every C-ABI
    symbol it calls resolves against the in-tree libjfsx.so."""
    assert os.path.exists(EXE), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", "-r", EXE], capture_output=True, text=True)
    assert "undefined symbol" not in out.stdout + out.stderr
    assert "libjfsx.so" in out.stdout


@pytest.mark.gpu
def test_shim_sequence_on_gpu():
    out = subprocess.run([EXE], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "shim sequence ok" in out.stdout
