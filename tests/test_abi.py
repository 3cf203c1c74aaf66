"""The C-ABI library loads and exports every symbol include/jfsx.h declares
(no compute calls: those need a GPU)."""
import ctypes
import os
import re

from juicefs_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "jfsx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(jfsx_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _declared() == sorted(engine.EXPORTS)


def test_library_exports_every_symbol():
    L = engine.load_library()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.jfsx_abi_version() == 9


def test_struct_layout_matches_header():
    # jfsx_blk: key[32] nonce[12] u32 | src dst len | tag[16] | crc | status bad got expect
    assert ctypes.sizeof(engine.jfsx_blk) == 112
    assert engine.jfsx_blk.src.offset == 48 and engine.jfsx_blk.tag.offset == 72
    assert engine.jfsx_blk.crc.offset == 88 and engine.jfsx_blk.status.offset == 96
    assert ctypes.sizeof(engine.jfsx_range) == 40


def test_no_device_is_an_error_not_a_fallback(monkeypatch):
    # without a HIP device the engine must refuse to construct
    if engine.device_count() > 0:
        return
    import pytest
    with pytest.raises(RuntimeError):
        engine.Engine(0)


def test_gen_key_matches_oracle_stream():
    from oracle import oracle as orc
    for b in (0, 1, 77, 123456):
        assert engine.gen_key(0x4A465321, b) == orc.gen_key(0x4A465321, b)


def test_parse_header():
    L = engine.load_library()
    obj = bytes([1, 0, 12]) + bytes(256) + bytes(12) + bytes(21)
    kl, nl = ctypes.c_int(), ctypes.c_int()
    assert L.jfsx_parse_header(obj, len(obj), ctypes.byref(kl), ctypes.byref(nl)) == 0
    assert (kl.value, nl.value) == (256, 12)
    assert L.jfsx_parse_header(obj[:271], 271, ctypes.byref(kl), ctypes.byref(nl)) == engine.EMISFORMED


def test_last_error_is_empty_without_a_failure():
    # jfsx_last_error(NULL, ...): the calling thread's record; nothing failed here
    assert engine.last_error(None) == (0, "")


def test_metrics_struct_layout():
    # jfsx_metrics: 26 uint64 counters, double kernel_ms, uint64 kernel_launches
    assert ctypes.sizeof(engine.jfsx_metrics) == 28 * 8
    assert engine.jfsx_metrics.kernel_ms.offset == 26 * 8
    src = open(os.path.join(ROOT, "include", "jfsx.h")).read()
    body = src[src.index("typedef struct jfsx_metrics"):src.index("} jfsx_metrics;")]
    names = re.findall(r"\b([a-z0-9_]+)\b(?=[,;])", body)
    assert names == [f for f, _ in engine.jfsx_metrics._fields_]
