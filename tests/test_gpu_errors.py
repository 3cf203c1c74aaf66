"""Batch-level failures are diagnosable (What's weak 8): the engine
keeps the HIP error and call site behind a JFSX_EIO / JFSX_ENOMEM
(jfsx_last_error), EngineError carries it, and the LZ4 compressor input that
once faulted the device (a match candidate in a block's first bytes) is
covered."""
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc  # checker only

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def test_failed_allocation_names_the_hip_error(eng):
    with pytest.raises(E.EngineError) as ei:
        eng.alloc(1 << 52)  # 4 PiB: hipMalloc fails
    err = ei.value
    assert err.code == E.ENOMEM
    assert err.hip_error != 0 and "hipMalloc" in err.detail and "jfsx_api.cpp" in err.detail
    assert eng.last_error() == (err.hip_error, err.detail)
    # the context stays usable after a failed allocation, and the handled
    # failure does not resurface as the next batch's launch error (a stale
    # hipGetLastError() once turned it into JFSX_EIO)
    buf = eng.alloc(1 << 20)
    buf.free()
    assert eng.lz4_compress([b"abcd" * 100]) == [orc.lz4_compress(b"abcd" * 100)]
    assert eng.zstd_compress([b"zstd" * 100])[0][:4] == b"\x28\xb5\x2f\xfd"


def test_lz4_match_in_first_bytes():
    # jfsx_lz4.hip count_and_back: with the 4-byte test and the count in one
    # round of loads (skip = 0), a match candidate at block positions 0..2
    # puts lane 0's match dword before byte 0; 84c5bd5 guards it (mps < 0).
    # The r2 JFSX_EIO (gpurun_out/lz4cab_c2, an uncommitted build between
    # 31a22e9 and 84c5bd5) came back cleanly in 1.3 s, with no memory-access
    # fault abort, so it was an API-level error; this covers the
    # inputs that guard is for.  Blocks that open with repeats of period 1..4,
    # across the small-table boundary.
    e = E.Engine(0)
    try:
        srcs = []
        for period in (1, 2, 3, 4):
            unit = bytes(range(97, 97 + period))
            for n in (13, 14, 20, 64, 65, 300, 4096, 65546, 65547, 70000):
                srcs.append((unit * (n // period + 1))[:n])
                srcs.append(((unit * 8)[:period * 2] + bytes((i * 7) & 255 for i in range(n)))[:n])
        outs = e.lz4_compress(srcs)
        for s, o in zip(srcs, outs):
            assert o == orc.lz4_compress(s), len(s)
    finally:
        e.close()
