"""GPU parity of the LZ4 stage (jfsx_lz4_compress_batch /
jfsx_lz4_decompress_batch) against the oracle (oracle/jfs_lz4.c, itself pinned
against the LZ4 C library in tests/test_lz4_oracle.py) and the golden
fixtures.  Bit-exact compressed bytes; decoded bytes and accept/reject of
malformed blocks as LZ4_decompress_safe."""
import hashlib
import json
import os

import numpy as np
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc
from tests import lz4_data

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "lz4_golden.json")


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def test_golden_batch_host(eng):
    g = json.load(open(GOLD))["cases"]
    srcs = [lz4_data.sample(c["kind"], c["n"], c["seed"]) for c in g]
    outs = eng.lz4_compress(srcs)
    for c, src, out in zip(g, srcs, outs):
        assert len(out) == c["out_len"], (c["kind"], c["n"])
        assert hashlib.sha256(out).hexdigest() == c["out_sha256"], (c["kind"], c["n"])
    back = eng.lz4_decompress(outs, [c["n"] for c in g])
    for c, src, (st, d) in zip(g, srcs, back):
        assert st == E.OK and d == src, (c["kind"], c["n"])


@pytest.mark.parametrize("n", [8 << 20, (16 << 20) - 5])
def test_large_blocks(eng, n):
    for kind in ("text", "random", "runs"):
        src = lz4_data.sample(kind, n, seed=3)
        out = eng.lz4_compress([src])[0]
        assert out == orc.lz4_compress(src), kind
        st, d = eng.lz4_decompress([out], [n])[0]
        assert st == E.OK and d == src


def _stale_entry_block(n, seed):
    """Random bytes with 16-byte phrases repeated at distances around the
    LZ4 window (65535 / 65536) and the LDS table's 2^17 / 2^18 position
    aliases, plus zero runs longer than 64 KiB (the parse jumps past several
    sweep points at once)."""
    rng = np.random.default_rng(seed)
    b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    pos = 4096
    for d in (65531, 65532, 65535, 65536, 65537, 131071, 131072, 131073, 196608, 262143, 262144, 262145,
              262144 + 65535, 327680):
        ph = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        if pos + d + 16 < n:
            b[pos:pos + 16] = ph
            b[pos + d:pos + d + 16] = ph
        pos += 1031
    for z0, zl in ((n // 3, 200000), (n // 2 + 7, 70001), (n - 140000, 131073)):
        if z0 + zl < n:
            b[z0:z0 + zl] = bytes(zl)
    return bytes(b)


@pytest.mark.parametrize("table", ["lds", "global"])
def test_table_kinds_match_oracle(eng, table, monkeypatch):
    """Both compressor tables (JFSX_LZ4_TABLE: the 18-bit LDS table with its
    64 KiB sweeps, the u32 global table) give the library's bytes: phrases
    repeated across the 64 KiB window and the LDS table's position aliases,
    long zero runs, and 4 MiB text / random / runs blocks."""
    monkeypatch.setenv("JFSX_LZ4_TABLE", table)
    srcs = [_stale_entry_block(1 << 20, 11), _stale_entry_block((3 << 20) + 77, 12)]
    srcs += [lz4_data.sample(k, 4 << 20, seed=21) for k in ("text", "random", "runs")]
    srcs += [lz4_data.sample("text", 70000, seed=22), lz4_data.sample("text", 65546, seed=23)]
    outs = eng.lz4_compress(srcs)
    for i, (src, out) in enumerate(zip(srcs, outs)):
        assert out == orc.lz4_compress(src), (table, i, len(src))


def test_device_batch_ragged_unaligned(eng):
    """Device-resident batch: ragged lengths, src/dst at odd offsets."""
    rng = np.random.default_rng(5)
    n = 40
    lens = [int(x) for x in rng.integers(0, 300000, n)]
    srcs = [lz4_data.sample(lz4_data.KINDS[i % len(lz4_data.KINDS)], lens[i], seed=100 + i) for i in range(n)]
    bounds = [int(E.lz4_bound(L)) for L in lens]
    inb = eng.alloc(sum(L + 8 for L in lens))
    outb = eng.alloc(sum(b + 8 for b in bounds))
    specs, io, oo = [], 0, 0
    for i in range(n):
        a, b = io + (i % 4), oo + (i % 3)
        inb.upload(np.frombuffer(srcs[i], np.uint8) if lens[i] else np.zeros(0, np.uint8), a)
        specs.append((inb.ptr + a, lens[i], outb.ptr + b, bounds[i]))
        io += lens[i] + 8
        oo += bounds[i] + 8
    arr, m = eng.make_zblocks(specs)
    eng.lz4_compress_batch(arr, m, E.MEM_DEVICE)
    comp = []
    for i in range(n):
        assert arr[i].status == E.OK
        got = outb.download(arr[i].out_len, specs[i][2] - outb.ptr).tobytes()
        assert got == orc.lz4_compress(srcs[i]), (i, lens[i])
        comp.append(got)
    # decode the compressed images back into the input buffer's slots (device mode)
    cb = eng.alloc(sum(len(c) + 8 for c in comp))
    dspecs, co = [], 0
    for i, c in enumerate(comp):
        cb.upload(np.frombuffer(c, np.uint8), co + 1)
        dspecs.append((cb.ptr + co + 1, len(c), specs[i][0], lens[i]))
        co += len(c) + 8
    darr, m = eng.make_zblocks(dspecs)
    eng.lz4_decompress_batch(darr, m, E.MEM_DEVICE)
    for i in range(n):
        assert darr[i].status == E.OK and darr[i].out_len == lens[i]
        assert inb.download(lens[i], specs[i][0] - inb.ptr).tobytes() == srcs[i]


def test_decompress_malformed_matches_oracle(eng):
    rng = np.random.default_rng(9)
    blobs, caps, exp = [], [], []
    for trial in range(400):
        kind = lz4_data.KINDS[trial % len(lz4_data.KINDS)]
        n = int(rng.choice([20, 300, 5000, 70000]))
        c = bytearray(orc.lz4_compress(lz4_data.sample(kind, n, seed=trial)))
        m = trial % 4
        if m == 0 and len(c) > 1:
            c = c[:int(rng.integers(0, len(c)))]
        elif m == 1:
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, len(c)))
                c[i] ^= 1 << int(rng.integers(0, 8))
        elif m == 2:
            c[int(rng.integers(0, len(c)))] = int(rng.integers(0, 256))
        cap = n if rng.random() < 0.7 else int(rng.integers(0, n + 50))
        blobs.append(bytes(c))
        caps.append(cap)
        exp.append(orc.lz4_decompress(bytes(c), cap))
    got = eng.lz4_decompress(blobs, caps)
    bad = 0
    for (st, d), (rc, ref) in zip(got, exp):
        if rc < 0:
            assert st == E.EFORMAT
            bad += 1
        else:
            assert st == E.OK and d == ref
    assert bad > 50  # the corpus does exercise the reject paths


def test_edge_statuses(eng):
    # empty input with capacity: malformed; "\x00" into zero capacity: ok, 0 bytes
    assert eng.lz4_decompress([b"", b"\x00"], [10, 0]) == [(E.EFORMAT, b""), (E.OK, b"")]
    # a destination one byte short
    c = orc.lz4_compress(bytes(1000))
    assert eng.lz4_decompress([c], [999])[0][0] == E.EFORMAT
    # compress needs a CompressBound-sized destination
    src = np.zeros(1000, np.uint8)
    dst = np.zeros(1000, np.uint8)
    arr, n = eng.make_zblocks([(src.ctypes.data, 1000, dst.ctypes.data, 1000)])
    with pytest.raises(E.EngineError) as ei:
        eng.lz4_compress_batch(arr, n, E.MEM_HOST)
    assert ei.value.code == E.EINVAL


def test_match_in_the_first_bytes(eng):
    """Periodic inputs whose first match starts at byte 1..8 of the block.  The
    compressor's combined 4-byte test and match count reads the match side at
    a lane-0 position below byte 0 here; before that read was clamped the
    position wrapped to 2^32 - k and the load faulted (the round-2 EIO of
    gpurun_out/lz4cab_c2).  Every block equals the oracle's, in
    blocks placed at every alignment of a 4-byte word."""
    srcs = []
    for period in range(1, 9):
        for n in (13, 14, 17, 31, 64, 100, 300, 4096):
            pat = bytes((0x61 + 7 * k) & 0xff for k in range(period))
            srcs.append((pat * (n // period + 1))[:n])
    outs = eng.lz4_compress(srcs)
    for s, o in zip(srcs, outs):
        assert o == orc.lz4_compress(s), (len(s), s[:8])
    inb = eng.alloc(sum(len(s) + 3 for s in srcs) + 64)
    caps = [int(E.lz4_bound(len(s))) for s in srcs]
    outb = eng.alloc(sum(caps) + 64)
    specs, io, oo = [], 1, 0
    for s, c in zip(srcs, caps):
        inb.upload(np.frombuffer(s, np.uint8), io)
        specs.append((inb.ptr + io, len(s), outb.ptr + oo, c))
        io += len(s) + 3
        oo += c
    arr, k = eng.make_zblocks(specs)
    eng.lz4_compress_batch(arr, k, E.MEM_DEVICE)
    for i, (s, (_, _, dp, _)) in enumerate(zip(srcs, specs)):
        assert arr[i].status == E.OK
        assert outb.download(arr[i].out_len, dp - outb.ptr).tobytes() == orc.lz4_compress(s), i
