"""Scheduling logic of the aggregator and the async queue
(juicefs_amd/csrc/jfsx_agg.cpp), compiled for the host over stub batch entry
points (tests/harness/agg_host.cpp): many threads making the reference's
one-block synchronous calls (dataEncryptor.Encrypt/Decrypt,
pkg/object/encrypt.go:164-216; the cache-read verify, disk_cache.go:1315-1327)
must come out as few, well-formed batches, each caller getting exactly its own
result.  The GPU behaviour of the same code is in tests/test_gpu_agg.py."""
import ctypes
import os
import subprocess
import threading

import numpy as np
import pytest

from juicefs_amd import engine as E

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FAKE_CTX = ctypes.c_void_p(0x1000)


@pytest.fixture(scope="module")
def H(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("agg") / "agg_host.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-I", os.path.join(ROOT, "include"),
                           "-o", out, os.path.join(HERE, "harness", "agg_host.cpp"), "-lpthread"])
    L = ctypes.CDLL(out)
    P, I, U64, U32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32
    BP = ctypes.POINTER(E.jfsx_blk)
    for name, res, args in [
        ("jfsx_agg_new", I, [P, I, U64, U32, ctypes.POINTER(P)]),
        ("jfsx_agg_free", I, [P]),
        ("jfsx_agg_seal", I, [P, I, BP, I, I]),
        ("jfsx_agg_open", I, [P, I, BP, I, I]),
        ("jfsx_agg_crc32c", I, [P, ctypes.POINTER(E.jfsx_range), I, I]),
        ("jfsx_agg_stats", I, [P, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        ("jfsx_seal_batch_async", I, [P, I, I, BP, I, I, ctypes.POINTER(U64)]),
        ("jfsx_open_batch_async", I, [P, I, I, BP, I, I, ctypes.POINTER(U64)]),
        ("jfsx_wait", I, [P, U64, I]),
        ("harness_reset", None, [I]),
        ("harness_batches", I, [P, P, P, I]),
        ("harness_close", None, [P]),
        ("harness_set_ndev", None, [I]),
        ("harness_open_ctx", I, []),
        ("harness_batch_devs", I, [P, P, I]),
        ("harness_batch_srcs", I, [I, P, I]),
        ("jfsx_mctx_open", I, [U64, U32, ctypes.POINTER(P)]),
        ("jfsx_mctx_close", I, [P]),
        ("jfsx_mctx_ndev", I, [P]),
        ("jfsx_mctx_ctx", P, [P, I]),
        ("jfsx_mctx_seal_batch", I, [P, I, I, BP, I, I]),
        ("jfsx_mctx_open_batch", I, [P, I, I, BP, I, I]),
        ("jfsx_mctx_crc32c_segments", I, [P, I, ctypes.POINTER(E.jfsx_range), I, I]),
        ("jfsx_agg_new_mctx", I, [P, I, U64, U32, ctypes.POINTER(P)]),
        ("jfsx_agg_dev_batches", I, [P, I, ctypes.POINTER(U64)]),
        ("jfsx_agg_lz4_compress", I, [P, ctypes.POINTER(E.jfsx_zblk), I]),
        ("jfsx_agg_lz4_decompress", I, [P, ctypes.POINTER(E.jfsx_zblk), I]),
        ("jfsx_mctx_lz4_compress_batch", I, [P, I, ctypes.POINTER(E.jfsx_zblk), I]),
        ("harness_pageable", None, [ctypes.c_size_t, ctypes.c_size_t]),
        ("harness_bounces", I, []),
    ]:
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def batches(H):
    cap = 100000
    s, o, m = (ctypes.c_int * cap)(), (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    n = H.harness_batches(s, o, m, cap)
    return [(s[i], o[i], m[i]) for i in range(n)]


def fake_tag(key, length, algo):
    return bytes(key[k] ^ ((length >> (8 * (k & 7))) & 255) ^ algo for k in range(16))


def mkblk(i, length):
    b = E.jfsx_blk()
    key = bytes((i * 31 + k) & 255 for k in range(32))
    ctypes.memmove(b.key, key, 32)
    b.len = length
    return b, key


def new_agg(H, max_blocks=0, max_bytes=0, window_us=2000):
    h = ctypes.c_void_p()
    assert H.jfsx_agg_new(FAKE_CTX, max_blocks, max_bytes, window_us, ctypes.byref(h)) == 0
    return h


def stats(H, h):
    v = [ctypes.c_uint64() for _ in range(3)]
    assert H.jfsx_agg_stats(h, *[ctypes.byref(x) for x in v]) == 0
    return tuple(x.value for x in v)


def run_threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: B902 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def test_concurrent_seals_coalesce_and_return_own_results(H):
    H.harness_reset(3000)
    h = new_agg(H, window_us=5000)
    N, PER = 32, 8
    got = {}

    def worker(t):
        for j in range(PER):
            i = t * PER + j
            b, key = mkblk(i, 1000 + i)
            assert H.jfsx_agg_seal(h, E.AES256GCM, ctypes.byref(b), E.CRC_GEN, E.MEM_HOST) == 0
            assert b.status == E.OK
            got[i] = (bytes(b.tag), fake_tag(key, 1000 + i, E.AES256GCM))

    run_threads(N, worker)
    assert all(a == e for a, e in got.values()) and len(got) == N * PER
    calls, nb, blocks = stats(H, h)
    assert calls == blocks == N * PER
    # coalesced, not one batch per call (about 8 per batch with 32 callers over
    # 4 dispatchers; a loaded host trickles requests in, so the bound is loose)
    assert nb < calls // 3, (calls, nb)
    bs = batches(H)
    assert sum(s for s, _, _ in bs) == N * PER and all(op == 0 and m == E.CRC_GEN for _, op, m in bs)
    assert H.jfsx_agg_free(h) == 0


def test_groups_never_mix_ops_or_modes(H):
    H.harness_reset(1000)
    h = new_agg(H, window_us=3000)
    res = {}

    def worker(i):
        b, key = mkblk(i, 4096 + i)
        kind = i % 3
        if kind == 0:
            rc = H.jfsx_agg_seal(h, E.CHACHA20P1305, ctypes.byref(b), E.CRC_NONE, E.MEM_HOST)
        elif kind == 1:
            ctypes.memmove(b.tag, fake_tag(key, 4096 + i, E.AES256GCM) if i % 2 else bytes(16), 16)
            rc = H.jfsx_agg_open(h, E.AES256GCM, ctypes.byref(b), E.CRC_VERIFY, E.MEM_HOST)
        else:
            r = E.jfsx_range()
            r.len = i
            rc = H.jfsx_agg_crc32c(h, ctypes.byref(r), E.CRC_VERIFY, E.MEM_HOST)
            res[i] = (rc, r.status)
            return
        res[i] = (rc, b.status)

    run_threads(60, worker)
    for i, (rc, st) in res.items():
        assert rc == 0
        if i % 3 == 1:
            assert st == (E.OK if i % 2 else E.ETAG), i
        elif i % 3 == 2:
            assert st == (E.ECRC if i % 7 == 3 else E.OK), i
    ops = {op for _, op, _ in batches(H)}
    assert ops == {0, 1, 2}
    calls, nb, blocks = stats(H, h)
    assert calls == blocks == 60 and nb >= 3
    H.jfsx_agg_free(h)


def test_max_blocks_and_max_bytes_cap_batches(H):
    H.harness_reset(2000)
    h = new_agg(H, max_blocks=5, window_us=20000)
    run_threads(40, lambda i: H.jfsx_agg_seal(h, 0, ctypes.byref(mkblk(i, 100)[0]), 0, E.MEM_HOST))
    assert max(s for s, _, _ in batches(H)) <= 5
    H.jfsx_agg_free(h)
    H.harness_reset(2000)
    h = new_agg(H, max_bytes=3000, window_us=20000)
    run_threads(40, lambda i: H.jfsx_agg_seal(h, 0, ctypes.byref(mkblk(i, 1000)[0]), 0, E.MEM_HOST))
    assert max(s for s, _, _ in batches(H)) <= 3
    H.jfsx_agg_free(h)


def test_lone_request_leaves_after_window(H):
    H.harness_reset(0)
    h = new_agg(H, window_us=1000)
    b, key = mkblk(7, 77)
    assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), 0, E.MEM_HOST) == 0
    assert bytes(b.tag) == fake_tag(key, 77, 0)
    assert stats(H, h) == (1, 1, 1)
    H.jfsx_agg_free(h)


def test_invalid_request_fails_alone(H):
    H.harness_reset(1000)
    h = new_agg(H, window_us=5000)
    rcs = {}

    def worker(i):
        b, _ = mkblk(i, 500)
        b.reserved = 1 if i == 5 else 0  # the stub engine rejects this block
        rcs[i] = H.jfsx_agg_seal(h, 0, ctypes.byref(b), 0, E.MEM_HOST)

    run_threads(16, worker)
    assert rcs[5] == E.EINVAL
    assert all(rc == 0 for i, rc in rcs.items() if i != 5)
    # argument errors the aggregator sees itself never reach the engine
    b, _ = mkblk(0, 1)
    assert H.jfsx_agg_seal(h, 9, ctypes.byref(b), 0, E.MEM_HOST) == E.EINVAL
    assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), 0, 5) == E.EINVAL
    H.jfsx_agg_free(h)


def test_async_tickets_order_poll_and_close(H):
    H.harness_reset(20000)
    ctx = ctypes.c_void_p(0x2000)
    arrs, tickets = [], []
    for k in range(4):
        arr = (E.jfsx_blk * 3)()
        for i in range(3):
            ctypes.memmove(arr[i].key, bytes([k * 3 + i]) * 32, 32)
            arr[i].len = 10 * k + i
        t = ctypes.c_uint64()
        assert H.jfsx_seal_batch_async(ctx, 1, 3, arr, 0, E.MEM_DEVICE, ctypes.byref(t)) == 0
        arrs.append(arr)
        tickets.append(t.value)
    assert len(set(tickets)) == 4
    assert H.jfsx_wait(ctx, tickets[3], 0) == E.EAGAIN  # 4 x 20 ms queued: not done yet
    assert H.jfsx_wait(ctx, tickets[3], -1) == 0
    for t in tickets[:3]:
        assert H.jfsx_wait(ctx, t, -1) == 0  # earlier batches finished first (FIFO)
    assert H.jfsx_wait(ctx, tickets[0], 0) == E.EINVAL  # retired
    for k, arr in enumerate(arrs):
        for i in range(3):
            assert bytes(arr[i].tag) == fake_tag(bytes([k * 3 + i]) * 32, 10 * k + i, 1)
    # a batch the engine rejects reports through jfsx_wait
    bad = (E.jfsx_blk * 1)()
    bad[0].reserved = 1
    t = ctypes.c_uint64()
    assert H.jfsx_open_batch_async(ctx, 0, 1, bad, 0, E.MEM_DEVICE, ctypes.byref(t)) == 0
    assert H.jfsx_wait(ctx, t.value, -1) == E.EINVAL
    # close runs what is still queued
    arr = (E.jfsx_blk * 1)()
    arr[0].len = 5
    assert H.jfsx_seal_batch_async(ctx, 0, 1, arr, 0, E.MEM_DEVICE, ctypes.byref(t)) == 0
    H.harness_close(ctx)
    assert bytes(arr[0].tag) == fake_tag(bytes(32), 5, 0)
    assert H.jfsx_wait(ctx, t.value, 0) == E.EINVAL


# ---------------------------------------------------------------------------
# multi-device context (jfsx_mctx) and the per-device dispatchers


def batch_devs(H):
    cap = 100000
    d, f = (ctypes.c_int * cap)(), (ctypes.c_uint64 * cap)()
    n = H.harness_batch_devs(d, f, cap)
    return [(d[i], f[i]) for i in range(n)]


def mctx(H, mask=0, ndev=4):
    H.harness_set_ndev(ndev)
    m = ctypes.c_void_p()
    assert H.jfsx_mctx_open(mask, 0, ctypes.byref(m)) == 0
    return m


def test_mctx_open_mask_and_close(H):
    m = mctx(H, 0)
    assert H.jfsx_mctx_ndev(m) == 4
    assert [H.jfsx_mctx_ctx(m, i) for i in range(4)] == [0x1000, 0x1100, 0x1200, 0x1300]
    assert H.jfsx_mctx_ctx(m, 4) is None
    assert H.jfsx_mctx_close(m) == 0
    m = mctx(H, 0b1010)
    assert H.jfsx_mctx_ndev(m) == 2 and H.jfsx_mctx_ctx(m, 1) == 0x1300
    H.jfsx_mctx_close(m)
    assert H.harness_open_ctx() == 0  # every context closed again
    x = ctypes.c_void_p()
    assert H.jfsx_mctx_open(1 << 4, 0, ctypes.byref(x)) == E.ENODEV  # device 4 not visible
    H.harness_set_ndev(0)
    assert H.jfsx_mctx_open(0, 0, ctypes.byref(x)) == E.ENODEV
    H.harness_set_ndev(4)


@pytest.mark.parametrize("ndev", [4, 8])
@pytest.mark.parametrize("lens", [[4 << 20] * 64, [1000 * (i % 7 + 1) for i in range(37)], [5, 0, 0, 9], [1 << 30]])
def test_mctx_batch_splits_runs_by_bytes(H, lens, ndev):
    """A host batch is cut into contiguous per-device runs balanced by bytes;
    every block is processed exactly once, by one device, and gets its own
    result (4 and 8 fake devices: the 8-GPU node's split)."""
    H.harness_reset(0)
    m = mctx(H, ndev=ndev)
    n = len(lens)
    arr = (E.jfsx_blk * n)()
    keys = []
    for i, ln in enumerate(lens):
        key = bytes([(i * 7 + k) & 255 for k in range(32)])
        ctypes.memmove(arr[i].key, key, 32)
        arr[i].len = ln
        keys.append(key)
    assert H.jfsx_mctx_seal_batch(m, 1, n, arr, E.CRC_GEN, E.MEM_HOST) == 0
    for i, ln in enumerate(lens):
        assert bytes(arr[i].tag) == fake_tag(keys[i], ln, 1), i
    bd = batch_devs(H)
    sizes = [s for s, _, _ in batches(H)]
    assert sum(sizes) == n and len(bd) == min(ndev, n) and len({d for d, _ in bd}) == len(bd)
    if len(set(lens)) == 1 and n % ndev == 0:
        assert sizes == [n // ndev] * ndev  # equal blocks: equal runs
    # runs are contiguous and in order: device d's first block follows device d-1's run
    order = sorted(zip([d for d, _ in bd], sizes))
    start = 0
    for d, sz in order:
        start += sz
    assert start == n
    total = sum(lens) + n
    for (d, _), sz in zip(bd, sizes):
        assert sz >= 1
    if n >= 8 and len(set(lens)) > 1:
        # balanced: no run exceeds its fair share by more than one block
        per = {}
        i = 0
        for d, sz in order:
            per[d] = sum(lens[i:i + sz]) + sz
            i += sz
        assert max(per.values()) <= total / ndev + max(lens) + 1
    H.jfsx_mctx_close(m)
    H.harness_set_ndev(4)


def test_mctx_errors(H):
    H.harness_reset(0)
    m = mctx(H)
    arr = (E.jfsx_blk * 8)()
    for i in range(8):
        arr[i].len = 100
    # device batches route by ownership: host pointers (here null) have no device
    assert H.jfsx_mctx_seal_batch(m, 0, 8, arr, 0, E.MEM_DEVICE) == E.EINVAL
    assert batches(H) == []
    assert H.jfsx_mctx_seal_batch(m, 0, 0, arr, 0, E.MEM_HOST) == 0
    # an engine error on one device reaches the caller
    arr[5].reserved = 1
    assert H.jfsx_mctx_seal_batch(m, 0, 8, arr, 0, E.MEM_HOST) == E.EINVAL
    H.jfsx_mctx_close(m)
    # a one-device context passes device batches through; the stub device 3 fails them
    m = mctx(H, 0b1000)
    arr[5].reserved = 0
    assert H.jfsx_mctx_seal_batch(m, 0, 8, arr, 0, E.MEM_DEVICE) == E.EIO
    r = (E.jfsx_range * 3)()
    assert H.jfsx_mctx_crc32c_segments(m, 3, r, E.CRC_GEN, E.MEM_HOST) == 0
    H.jfsx_mctx_close(m)


def test_agg_over_devices_spreads_batches(H):
    """One dispatcher per device: with slow batches, concurrent per-block calls
    run on every device at once, and each caller still gets its own result."""
    H.harness_reset(20000)
    m = mctx(H)
    h = ctypes.c_void_p()
    assert H.jfsx_agg_new_mctx(m, 8, 0, 2000, ctypes.byref(h)) == 0
    res = {}

    def worker(i):
        b, key = mkblk(i, 1000 + i)
        rc = H.jfsx_agg_seal(h, 0, ctypes.byref(b), E.CRC_GEN, E.MEM_HOST)
        res[i] = rc == 0 and bytes(b.tag) == fake_tag(key, 1000 + i, 0)

    run_threads(96, worker)
    assert all(res.values()) and len(res) == 96
    per = []
    for i in range(4):
        v = ctypes.c_uint64()
        assert H.jfsx_agg_dev_batches(h, i, ctypes.byref(v)) == 0
        per.append(v.value)
    assert H.jfsx_agg_dev_batches(h, 4, ctypes.byref(ctypes.c_uint64())) == E.EINVAL
    assert all(p >= 1 for p in per), per  # every device took work
    calls, nb, blocks = stats(H, h)
    assert calls == blocks == 96 and nb == sum(per)
    assert max(s for s, _, _ in batches(H)) <= 8
    assert {d for d, _ in batch_devs(H)} == {0, 1, 2, 3}
    H.jfsx_agg_free(h)
    H.jfsx_mctx_close(m)


def test_lz4_calls_from_many_threads_batch_and_isolate_errors(H):
    """Per-block Compress / Decompress calls (cachedStore.upload / load,
    cached_store.go:387, :738) from many goroutines come out as few lz4
    batches, never mixed with AEAD or the other direction; a request the
    engine rejects (EINVAL) fails alone, a malformed block only flags itself."""
    H.harness_reset(3000)
    agg = ctypes.c_void_p()
    assert H.jfsx_agg_new(FAKE_CTX, 0, 0, 2000, ctypes.byref(agg)) == 0
    T = 48
    zs = [E.jfsx_zblk() for _ in range(T)]
    rcs = [None] * T
    for i, z in enumerate(zs):
        z.src_len = 1000 + i if i != 13 else 7
        z.dst_cap = 5000 if i not in (28, 29) else 1  # 28: a compress the engine rejects

    def worker(i):
        f = H.jfsx_agg_lz4_compress if i % 2 == 0 else H.jfsx_agg_lz4_decompress
        rcs[i] = f(agg, ctypes.byref(zs[i]), E.MEM_HOST)
    th = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i, z in enumerate(zs):
        if i % 2 == 0:
            assert rcs[i] == (E.EINVAL if i == 28 else 0)
            if i != 28:
                assert z.out_len == z.src_len // 2 + 1 and z.status == E.OK
        else:
            assert rcs[i] == 0, i  # a decompress with dst_cap 1 is no argument error
            assert z.status == (E.EFORMAT if i == 13 else E.OK)
    sizes, ops, modes = (ctypes.c_int * 256)(), (ctypes.c_int * 256)(), (ctypes.c_int * 256)()
    nb = H.harness_batches(sizes, ops, modes, 256)
    assert set(ops[:nb]) == {3, 4}
    # coalesced (the rejected request's batch is re-run one request at a time)
    assert nb < T * 2 // 3
    assert H.jfsx_agg_free(agg) == 0


def test_mctx_lz4_split_over_devices(H):
    H.harness_reset(0)
    H.harness_set_ndev(4)
    m = ctypes.c_void_p()
    assert H.jfsx_mctx_open(0, 0, ctypes.byref(m)) == 0
    n = 10
    zs = (E.jfsx_zblk * n)()
    for i in range(n):
        zs[i].src_len, zs[i].dst_cap = 4096 * (i + 1), 9000 * (i + 1)
    assert H.jfsx_mctx_lz4_compress_batch(m, n, zs, E.MEM_HOST) == 0
    assert all(zs[i].out_len == zs[i].src_len // 2 + 1 for i in range(n))
    dev, first = (ctypes.c_int * 16)(), (ctypes.c_uint64 * 16)()
    nb = H.harness_batch_devs(dev, first, 16)
    assert sorted(dev[:nb]) == [0, 1, 2, 3]
    assert H.jfsx_mctx_close(m) == 0


def test_agg_over_devices_rejects_device_memory(H):
    """device pointers belong to one GPU, and any dispatcher of a
    multi-device aggregator may take a group, so JFSX_MEM_DEVICE requests are
    rejected there (as jfsx_mctx_*_batch do); a one-device aggregator keeps
    accepting them."""
    H.harness_reset(0)
    m = mctx(H)
    h = ctypes.c_void_p()
    assert H.jfsx_agg_new_mctx(m, 8, 0, 100, ctypes.byref(h)) == 0
    b, _ = mkblk(0, 4096)
    r = E.jfsx_range()
    z = E.jfsx_zblk()
    assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), E.CRC_GEN, E.MEM_DEVICE) == E.EINVAL
    assert H.jfsx_agg_open(h, 0, ctypes.byref(b), E.CRC_NONE, E.MEM_DEVICE) == E.EINVAL
    assert H.jfsx_agg_crc32c(h, ctypes.byref(r), E.CRC_GEN, E.MEM_DEVICE) == E.EINVAL
    for f in (H.jfsx_agg_lz4_compress, H.jfsx_agg_lz4_decompress, H.jfsx_agg_zstd_decompress):
        assert f(h, ctypes.byref(z), E.MEM_DEVICE) == E.EINVAL
    assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), E.CRC_GEN, E.MEM_HOST) == 0
    assert stats(H, h)[0] == 1  # the rejected calls never reached the queue
    H.jfsx_agg_free(h)
    H.jfsx_mctx_close(m)
    one = mctx(H, 0b0001)
    assert H.jfsx_agg_new_mctx(one, 8, 0, 100, ctypes.byref(h)) == 0
    assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), E.CRC_GEN, E.MEM_DEVICE) == 0
    H.jfsx_agg_free(h)
    H.jfsx_mctx_close(one)


def dev_ptr(d, off):
    """A fake device pointer of device d (tests/harness/agg_host.cpp device_of)."""
    return ((d + 1) << 40) + off


@pytest.mark.parametrize("order", ["grouped", "interleaved"])
def test_mctx_device_batch_routes_by_owner(H, order):
    """A device-memory batch on an 8-device context: every block runs on the
    GPU that owns its buffers (BASELINE configs[1] at 8 GPUs from one process),
    each device's blocks in the caller's order, in place when they are one run
    of the array and gathered otherwise; every block gets its own result."""
    H.harness_reset(0)
    m = mctx(H, ndev=8)
    per = 6
    n = 8 * per
    arr = (E.jfsx_blk * n)()
    owner = {}
    for i in range(n):
        d = i // per if order == "grouped" else i % 8
        j = i % per if order == "grouped" else i // 8
        ctypes.memmove(arr[i].key, bytes([(i * 5 + k) & 255 for k in range(32)]), 32)
        arr[i].len = 4096 + i
        arr[i].src = dev_ptr(d, j << 23)
        arr[i].dst = dev_ptr(d, (j << 23) + (1 << 22))
        arr[i].crc = dev_ptr(d, (1 << 34) + 512 * j)
        owner[arr[i].src] = (d, i)
    assert H.jfsx_mctx_seal_batch(m, 0, n, arr, E.CRC_GEN, E.MEM_DEVICE) == 0
    for i in range(n):
        assert bytes(arr[i].tag) == fake_tag(bytes([(i * 5 + k) & 255 for k in range(32)]), 4096 + i, 0), i
        assert arr[i].src == owner[arr[i].src][1] * 0 + arr[i].src  # the caller's records stay in place
    bd = batch_devs(H)
    assert sorted(d for d, _ in bd) == list(range(8))  # one batch per device
    buf = (ctypes.c_uint64 * 64)()
    for b, (d, _) in enumerate(bd):
        k = H.harness_batch_srcs(b, buf, 64)
        srcs = list(buf[:k])
        assert k == per and all(owner[p][0] == d for p in srcs)
        assert [owner[p][1] for p in srcs] == sorted(owner[p][1] for p in srcs)  # caller's order kept
    H.jfsx_mctx_close(m)
    H.harness_set_ndev(4)


def test_mctx_device_batch_rejects_mixed_or_foreign_buffers(H):
    H.harness_reset(0)
    m = mctx(H, mask=0b0110, ndev=8)  # devices 1 and 2
    arr = (E.jfsx_blk * 2)()
    for i in range(2):
        arr[i].len = 64
        arr[i].src = arr[i].dst = dev_ptr(1 + i, 0)
    assert H.jfsx_mctx_seal_batch(m, 0, 2, arr, 0, E.MEM_DEVICE) == 0
    assert sorted(d for d, _ in batch_devs(H)) == [1, 2]
    arr[1].dst = dev_ptr(1, 4096)  # src on device 2, dst on device 1
    assert H.jfsx_mctx_seal_batch(m, 0, 2, arr, 0, E.MEM_DEVICE) == E.EINVAL
    arr[1].dst = arr[1].src = dev_ptr(5, 0)  # device 5 is not in the context
    assert H.jfsx_mctx_seal_batch(m, 0, 2, arr, 0, E.MEM_DEVICE) == E.EINVAL
    arr[1].src = arr[1].dst = dev_ptr(2, 0)
    arr[1].crc = 0x1000  # a host CRC array beside device data
    assert H.jfsx_mctx_seal_batch(m, 0, 2, arr, E.CRC_GEN, E.MEM_DEVICE) == E.EINVAL
    # a zero-length block with no buffers runs on the first device
    H.harness_reset(0)
    z = (E.jfsx_blk * 1)()
    assert H.jfsx_mctx_seal_batch(m, 0, 1, z, 0, E.MEM_DEVICE) == 0
    assert [d for d, _ in batch_devs(H)] == [1]
    # device ranges route the same way
    r = (E.jfsx_range * 3)()
    for i, d in enumerate((2, 1, 2)):
        r[i].data, r[i].len, r[i].crc = dev_ptr(d, 65536 * i), 32768, dev_ptr(d, 1 << 30)
    H.harness_reset(0)
    assert H.jfsx_mctx_crc32c_segments(m, 3, r, E.CRC_GEN, E.MEM_DEVICE) == 0
    assert sorted(d for d, _ in batch_devs(H)) == [1, 2]
    H.jfsx_mctx_close(m)
    H.harness_set_ndev(4)


def test_pipelined_seals_run_several_batches_at_once(H):
    """Host-memory Seal requests pipeline (jfsx_seal_batch keeps several
    batches in flight): with the engine busy, free dispatchers take what is
    queued at once, so a 20-caller closed loop (max-uploads,
    cmd/flags.go:124-128) has several batches running together instead of one
    batch all callers wait for."""
    H.harness_reset(5000)
    h = new_agg(H, max_bytes=4 * 4096, window_us=2000)
    live, peak = [0], [0]
    lock = threading.Lock()

    def worker(t):
        for j in range(6):
            b, key = mkblk(t * 6 + j, 4096)
            with lock:
                live[0] += 1
            assert H.jfsx_agg_seal(h, 0, ctypes.byref(b), E.CRC_GEN, E.MEM_HOST) == 0
            with lock:
                live[0] -= 1
            assert bytes(b.tag) == fake_tag(key, 4096, 0)

    import time
    t0 = time.perf_counter()
    run_threads(20, worker)
    el = time.perf_counter() - t0
    calls, nb, blocks = stats(H, h)
    assert calls == blocks == 120
    assert max(s for s, _, _ in batches(H)) <= 4
    # 120 blocks in batches of <= 4 at 5 ms each: >= 30 batches, 150 ms one at a
    # time; several dispatchers overlap them
    assert nb >= 30 and el < 0.6 * nb * 0.005, (nb, el)
    H.jfsx_agg_free(h)


def test_serial_ops_keep_one_batch_per_device(H):
    """Codec and CRC requests hold their context for the whole call, so a
    device runs one such batch at a time and the requests that arrive
    meanwhile join the next batch (one wave per object: bigger batches)."""
    H.harness_reset(20000)
    h = new_agg(H, window_us=1000)
    zs = [E.jfsx_zblk() for _ in range(40)]
    for z in zs:
        z.src_len, z.dst_cap = 1000, 5000

    def worker(i):
        if i >= 8:
            import time
            time.sleep(0.005)  # arrive while the first batch runs
        assert H.jfsx_agg_lz4_compress(h, ctypes.byref(zs[i]), E.MEM_HOST) == 0

    run_threads(40, worker)
    sizes = [s for s, _, _ in batches(H)]
    assert sum(sizes) == 40 and len(sizes) <= 3, sizes
    H.jfsx_agg_free(h)


def fake_bytes(src, key):
    """The stub engine's bytes (agg_host.cpp fake_bytes): src ^ key ^ 0x5A."""
    return src ^ np.resize(np.frombuffer(key, np.uint8), len(src)) ^ np.uint8(0x5A)


def test_pageable_per_object_calls_stage_through_shared_arenas(H):
    """Per-object calls on pageable memory (a Go-heap slice: io.ReadAll's
    result and Encrypt's fresh object, encrypt.go:183, :258) are staged by the
    aggregator on the calling thread: the block is copied into a slice of a
    shared pinned arena, the batch runs on the staged copies, and the output
    comes back into the caller's own buffer.  20 callers, Seal then Open of
    each block (every 5th in place), every 7th Open with a bad tag (nothing
    released: the caller's buffer is zeroed); all callers' blocks share a few
    arenas (jfsx_agg.cpp arena_reserve); a block larger than a quarter of an
    arena takes a bounce buffer of its own."""
    H.harness_reset(300)
    N, PER, L = 20, 6, 65536 + 100
    buf = np.zeros((3, N * PER, L), np.uint8)
    src, obj, back = buf[0], buf[1], buf[2]
    src[:] = np.random.default_rng(5).integers(0, 256, src.shape, np.uint8)
    H.harness_pageable(buf.ctypes.data, buf.ctypes.data + buf.nbytes)
    b0 = H.harness_bounces()
    h = new_agg(H, window_us=2000)
    errs = []

    def worker(t):
        for j in range(PER):
            i = t * PER + j
            b, key = mkblk(i, L)
            b.src, b.dst = src[i].ctypes.data, obj[i].ctypes.data
            assert H.jfsx_agg_seal(h, E.AES256GCM, ctypes.byref(b), E.CRC_NONE, E.MEM_HOST) == 0
            assert b.status == E.OK and bytes(b.tag) == fake_tag(key, L, E.AES256GCM)
            assert b.src == src[i].ctypes.data and b.dst == obj[i].ctypes.data  # the caller's pointers kept
            if not np.array_equal(obj[i], fake_bytes(src[i], key)):
                errs.append(("seal", i))
            o, _ = mkblk(i, L)
            ctypes.memmove(o.tag, b.tag, 16)
            if i % 7 == 3:
                o.tag[0] ^= 1
            if i % 5 == 0:  # in place: the object buffer becomes the plaintext
                o.src = o.dst = obj[i].ctypes.data
                want_buf = obj[i]
            else:
                back[i] = 0xEE
                o.src, o.dst = obj[i].ctypes.data, back[i].ctypes.data
                want_buf = back[i]
            assert H.jfsx_agg_open(h, E.AES256GCM, ctypes.byref(o), E.CRC_NONE, E.MEM_HOST) == 0
            if i % 7 == 3:
                if o.status != E.ETAG or want_buf.any():
                    errs.append(("etag", i))
            elif o.status != E.OK or not np.array_equal(want_buf, src[i]):
                errs.append(("open", i))

    run_threads(N, worker)
    assert not errs, errs[:5]
    assert H.harness_bounces() - b0 <= 4  # a few shared arenas, not one buffer per call
    # a block over a quarter of an arena: a bounce buffer of its own
    big = np.zeros(2 * ((16 << 20) + 4096), np.uint8)
    big[: len(big) // 2] = 7
    H.harness_pageable(big.ctypes.data, big.ctypes.data + big.nbytes)
    b, key = mkblk(999, len(big) // 2)
    b.src, b.dst = big.ctypes.data, big.ctypes.data + len(big) // 2
    n0 = H.harness_bounces()
    assert H.jfsx_agg_seal(h, E.AES256GCM, ctypes.byref(b), E.CRC_NONE, E.MEM_HOST) == 0 and b.status == E.OK
    assert H.harness_bounces() == n0 + 1
    assert np.array_equal(big[len(big) // 2:], fake_bytes(big[: len(big) // 2], key))
    H.harness_pageable(0, 0)
    assert H.jfsx_agg_free(h) == 0
