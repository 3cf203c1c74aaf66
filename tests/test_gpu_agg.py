"""GPU parity of the asynchronous batches (jfsx_*_async + jfsx_wait) and of
the aggregator (jfsx_agg): many threads making one-block synchronous calls,
as dataEncryptor.Encrypt/Decrypt (pkg/object/encrypt.go:164-216) and the
cache-read verify (pkg/chunk/disk_cache.go:1315-1327) are made, get results
bit-identical to the oracle while the engine sees a few large batches."""
import ctypes
import os
import threading

import numpy as np
import pytest

from juicefs_amd import encrypt as enc
from juicefs_amd import engine as E
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ORC = {E.AES256GCM: orc.AES256GCM, E.CHACHA20P1305: orc.CHACHA20P1305}


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def run_threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: B902 -- re-raised below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_async_batches_match_oracle(eng, algo):
    lens = [[0, 17, 32768], [4 << 20, 100003], [65536 + 5, 1, 2 << 20]]
    jobs = []
    for bi, group in enumerate(lens):
        specs, keep = [], []
        for i, n in enumerate(group):
            p = orc.gen_block(31, 10 * bi + i, n)
            src, dst = eng.alloc(max(n, 16)), eng.alloc(max(n, 16))
            if n:
                src.upload(p)
            crc = eng.alloc(4 * max(1, -(-n // E.SEG)))
            key, nonce = orc.gen_key(31, 10 * bi + i)
            specs.append({"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": n, "crc": crc.ptr})
            keep.append((p, key, nonce, src, dst, crc))
        arr, cnt = eng.make_blocks(specs)
        t = eng.seal_batch_async(algo, arr, cnt, E.CRC_GEN, E.MEM_DEVICE)
        jobs.append((t, arr, keep))
    for t, arr, keep in reversed(jobs):  # any wait order
        assert eng.wait(t) is True
        for i, (p, key, nonce, src, dst, crc) in enumerate(keep):
            c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
            assert bytes(arr[i].tag) == tag and arr[i].status == E.OK
            if p.size:
                assert dst.download(p.size).tobytes() == c
            want = orc.checksum(p)
            assert crc.download(len(want)).tobytes() == want
    with pytest.raises(E.EngineError):
        eng.wait(jobs[0][0])  # retired ticket


def test_async_poll_and_batch_error(eng):
    n = 64 << 20
    src, dst = eng.alloc(n), eng.alloc(n)
    arr, cnt = eng.make_blocks([{"key": bytes(32), "nonce": bytes(12), "src": src.ptr, "dst": dst.ptr, "len": n}])
    t = eng.seal_batch_async(E.AES256GCM, arr, cnt, E.CRC_NONE, E.MEM_DEVICE)
    first = eng.wait(t, 0)
    assert first in (True, False)
    if first is False:
        assert eng.wait(t) is True
    bad, cnt = eng.make_blocks([{"key": bytes(32), "nonce": bytes(12), "src": src.ptr + 1, "dst": dst.ptr,
                                 "len": 64}])  # unaligned device pointer -> EINVAL at run time
    t = eng.open_batch_async(E.AES256GCM, bad, cnt, E.CRC_NONE, E.MEM_DEVICE)
    with pytest.raises(E.EngineError) as ei:
        eng.wait(t)
    assert ei.value.code == E.EINVAL


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_aggregator_concurrent_encrypt_decrypt(eng, algo):
    rng = np.random.default_rng(algo + 3)
    lens = [int(x) for x in rng.integers(0, 1 << 20, 96)] + [4 << 20, 0, 1, 32768]
    N = len(lens)
    plains = [orc.gen_block(41, i, n) for i, n in enumerate(lens)]
    keys = [orc.gen_key(41, i) for i in range(N)]
    out = [None] * N
    with E.Aggregator(eng, window_us=2000) as agg:
        def seal(i):
            p = plains[i]
            c = np.empty(max(p.size, 1), np.uint8)
            cs = np.zeros(4 * max(1, -(-p.size // E.SEG)), np.uint8)
            arr, _ = eng.make_blocks([{"key": keys[i][0], "nonce": keys[i][1], "src": p.ctypes.data if p.size else None,
                                       "dst": c.ctypes.data, "len": p.size, "crc": cs.ctypes.data}])
            agg.seal(algo, arr[0], E.CRC_GEN, E.MEM_HOST)
            assert arr[0].status == E.OK
            out[i] = (c[:p.size].copy(), bytes(arr[0].tag), cs.tobytes())

        run_threads(N, seal)
        calls, batches, blocks = agg.stats()
        assert calls == blocks == N and batches < N
        for i in range(N):
            c, tag = orc.seal(ORC[algo], keys[i][0], keys[i][1], plains[i], fast=True)
            assert out[i][0].tobytes() == c and out[i][1] == tag, i
            assert out[i][2][:len(orc.checksum(plains[i]))] == orc.checksum(plains[i])

        # Decrypt side: in place, one block tampered -> only it fails
        res = [None] * N

        def open_(i):
            c, tag, cs = out[i]
            if i == 7:
                tag = bytes([tag[0] ^ 1]) + tag[1:]
            buf = c.copy()
            arr, _ = eng.make_blocks([{"key": keys[i][0], "nonce": keys[i][1], "src": buf.ctypes.data if buf.size else None,
                                       "dst": buf.ctypes.data if buf.size else None, "len": buf.size, "tag": tag,
                                       "crc": np.frombuffer(cs, np.uint8).ctypes.data}])
            agg.open(algo, arr[0], E.CRC_VERIFY, E.MEM_HOST)
            res[i] = (arr[0].status, buf)

        run_threads(N, open_)
        for i in range(N):
            st, buf = res[i]
            if i == 7:
                assert st == E.ETAG
            else:
                assert st == E.OK and buf[:lens[i]].tobytes() == plains[i].tobytes(), i


def test_aggregator_crc_verify(eng):
    lens = [32768 * 3 + 5, 1 << 20, 7, 0]
    datas = [orc.gen_block(51, i, n) for i, n in enumerate(lens)]
    sums = [bytearray(orc.checksum(d)) for d in datas]
    sums[1][9] ^= 0x10  # segment 2 of range 1 has a wrong expected CRC
    res = {}
    with E.Aggregator(eng, window_us=1000) as agg:
        def verify(i):
            r = E.jfsx_range()
            d = datas[i]
            cs = (ctypes.c_uint8 * len(sums[i])).from_buffer(sums[i])
            r.data, r.len, r.crc = d.ctypes.data if d.size else None, d.size, ctypes.addressof(cs)
            agg.crc32c(r, E.CRC_VERIFY, E.MEM_HOST)
            res[i] = (r.status, r.bad_seg)

        run_threads(len(lens), verify)
    assert res[1] == (E.ECRC, 2)
    assert all(res[i][0] == E.OK for i in (0, 2, 3))


def test_data_encryptor_through_aggregator(eng):
    """dataEncryptor.Encrypt/Decrypt called per object from 24 threads, the
    way cachedStore's upload and read goroutines call them, round-trip and
    reach the engine as a few batches."""
    rsae = enc.NewRSAEncryptor(enc.GenerateRsaKey(2048))
    plains = [orc.gen_block(61, i, (i * 77777) % (1 << 20)).tobytes() for i in range(48)]
    objs, back = [None] * 48, [None] * 48
    with E.Aggregator(eng, window_us=3000) as agg:
        de = enc.NewDataEncryptor(rsae, "aes256gcm-rsa", eng, agg=agg)
        run_threads(48, lambda i: objs.__setitem__(i, de.Encrypt(plains[i])))
        run_threads(48, lambda i: back.__setitem__(i, de.Decrypt(objs[i])))
        calls, batches, blocks = agg.stats()
    assert back == plains
    assert calls == 96 and batches < 96
    plain_de = enc.NewDataEncryptor(rsae, "aes256gcm-rsa", eng)
    assert [plain_de.Decrypt(o) for o in objs[:4]] == plains[:4]


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_multi_device_context_host_batch(algo):
    """jfsx_mctx over every visible GPU (one on the test box): a host batch
    split into per-device runs gives the oracle's bytes, tags and CRCs; the
    aggregator over the same context serves per-block callers."""
    m = E.MultiEngine(0)
    try:
        assert m.ndev == E.device_count()
        lens = [0, 5, 32769, 1 << 20, 777777, 4 << 20, 3, 65536]
        ps, outs, crcs, specs = [], [], [], []
        for i, n in enumerate(lens):
            key, nonce = orc.gen_key(123, i)
            p = orc.gen_block(123, i, n)
            o = np.zeros(max(n, 1), np.uint8)
            cb = np.zeros(4 * max(1, -(-n // E.SEG)), np.uint8)
            ps.append(p), outs.append(o), crcs.append(cb)
            specs.append({"key": key, "nonce": nonce, "src": p.ctypes.data if n else None, "dst": o.ctypes.data,
                          "len": n, "crc": cb.ctypes.data})
        arr, nb = E.Engine.make_blocks(specs)
        m.seal_batch(algo, arr, nb, E.CRC_GEN, E.MEM_HOST)
        for i, n in enumerate(lens):
            key, nonce = orc.gen_key(123, i)
            c, tag = orc.seal(ORC[algo], key, nonce, ps[i], fast=True)
            assert bytes(arr[i].tag) == tag and outs[i][:n].tobytes() == c, i
            assert crcs[i].tobytes() == orc.checksum(ps[i], hw=True), i
        with E.Aggregator(m, window_us=2000) as agg:
            res = {}

            def worker(i):
                key, nonce = orc.gen_key(123, i)
                p = ps[i]
                c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
                q = np.zeros(max(p.size, 1), np.uint8)
                a, _ = E.Engine.make_blocks([{"key": key, "nonce": nonce, "src": outs[i].ctypes.data,
                                              "dst": q.ctypes.data, "len": p.size, "tag": tag,
                                              "crc": crcs[i].ctypes.data}])
                agg.open(algo, a[0], E.CRC_VERIFY, E.MEM_HOST)
                res[i] = (a[0].status, q[:p.size].tobytes() == p.tobytes())

            run_threads(len(lens), worker)
            assert all(v == (E.OK, True) for v in res.values()), res
            assert sum(agg.dev_batches()) >= 1
    finally:
        m.close()


def test_lz4_per_block_calls_through_the_aggregator():
    """cachedStore.upload / load call Compress / Decompress once per block
    from many goroutines: through jfsx_agg they become batches, each caller
    gets its own bytes (bit-exact to the oracle)."""
    import threading
    from tests import lz4_data
    eng = E.Engine(0)
    try:
        T = 24
        srcs = [np.frombuffer(lz4_data.sample(lz4_data.KINDS[i % 6], 50000 + 997 * i, seed=i), np.uint8)
                for i in range(T)]
        outs = [np.zeros(int(E.lz4_bound(s.size)), np.uint8) for s in srcs]
        backs = [np.zeros(s.size, np.uint8) for s in srcs]
        zc = [E.jfsx_zblk() for _ in range(T)]
        zd = [E.jfsx_zblk() for _ in range(T)]
        with E.Aggregator(eng, window_us=3000) as agg:
            def worker(i):
                z = zc[i]
                z.src, z.src_len, z.dst, z.dst_cap = srcs[i].ctypes.data, srcs[i].size, outs[i].ctypes.data, outs[i].size
                agg.lz4_compress(z)
                d = zd[i]
                d.src, d.src_len, d.dst, d.dst_cap = outs[i].ctypes.data, z.out_len, backs[i].ctypes.data, backs[i].size
                agg.lz4_decompress(d)
            th = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            calls, batches, blocks = agg.stats()
        for i in range(T):
            assert zc[i].status == E.OK and zd[i].status == E.OK
            assert outs[i][:zc[i].out_len].tobytes() == orc.lz4_compress(srcs[i])
            assert zd[i].out_len == srcs[i].size and backs[i].tobytes() == srcs[i].tobytes()
        assert calls == 2 * T and batches < calls
    finally:
        eng.close()


def _host_block(seed, i, n):
    p = orc.gen_block(seed, i, n)
    key, nonce = orc.gen_key(seed, i)
    c = np.zeros(max(n, 1), np.uint8)
    cs = np.zeros(4 * max(1, -(-n // E.SEG)), np.uint8)
    return p, key, nonce, c, cs


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_host_pipeline_shared_by_concurrent_callers(algo):
    """jfsx_seal_batch / jfsx_open_batch on host memory share one pipeline of
    staging slots per context and wait only for their own groups: two callers
    whose batches each span more groups than there are slots (2 MiB slots),
    plus 16 one-block callers, all at once, every block bit-exact to the oracle
    and every CRC array right; then the same through Open."""
    eng = E.Engine(0)
    try:
        eng.set_slot_bytes(2 << 20)
        rng = np.random.default_rng(algo + 11)
        big = [[int(x) for x in rng.integers(1, 3 << 20, 24)] for _ in range(2)]
        small = [int(x) for x in rng.integers(0, 5 << 20, 16)]
        jobs = [(0, ln) for ln in big] + [(1, [ln]) for ln in small]
        res = [None] * len(jobs)

        def work(j):
            _, lens = jobs[j]
            blocks = [_host_block(900 + j, i, n) for i, n in enumerate(lens)]
            arr, nb = eng.make_blocks([{"key": k, "nonce": nn, "src": p.ctypes.data if p.size else None,
                                        "dst": c.ctypes.data, "len": p.size, "crc": cs.ctypes.data}
                                       for p, k, nn, c, cs in blocks])
            eng.seal_batch(algo, arr, nb, E.CRC_GEN, E.MEM_HOST)
            tags = [bytes(arr[i].tag) for i in range(nb)]
            # and back through Open, in place, verifying the CRCs
            for i, (p, k, nn, c, cs) in enumerate(blocks):
                arr[i].src = arr[i].dst = c.ctypes.data
                ctypes.memmove(arr[i].tag, tags[i], 16)
            eng.open_batch(algo, arr, nb, E.CRC_VERIFY, E.MEM_HOST)
            res[j] = (blocks, tags, [arr[i].status for i in range(nb)])

        run_threads(len(jobs), work)
        for blocks, tags, st in res:
            for (p, k, nn, c, cs), tag, s in zip(blocks, tags, st):
                ct, etag = orc.seal(ORC[algo], k, nn, p, fast=True)
                assert tag == etag and s == E.OK
                assert c[:p.size].tobytes() == p.tobytes()  # opened in place: the plaintext again
                assert cs.tobytes() == orc.checksum(p, hw=True)
    finally:
        eng.close()


_META_COPY_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from juicefs_amd import engine as E
from oracle import oracle as orc
eng = E.Engine(0)
eng.set_slot_bytes(2 << 20)
rng = np.random.default_rng(5)
lens = [int(x) for x in rng.integers(0, 3 << 20, 12)] + [0, 17]
specs, keep = [], []
for i, n in enumerate(lens):
    p = orc.gen_block(77, i, n)
    k, nn = orc.gen_key(77, i)
    c = np.zeros(max(n, 1), np.uint8)
    cs = np.zeros(4 * max(1, -(-n // E.SEG)), np.uint8)
    keep.append((p, k, nn, c, cs))
    specs.append({"key": k, "nonce": nn, "src": p.ctypes.data if n else None, "dst": c.ctypes.data, "len": n,
                  "crc": cs.ctypes.data})
arr, nb = eng.make_blocks(specs)
eng.seal_batch(E.AES256GCM, arr, nb, E.CRC_GEN, E.MEM_HOST)
for i, (p, k, nn, c, cs) in enumerate(keep):
    ct, tag = orc.seal(orc.AES256GCM, k, nn, p, fast=True)
    assert bytes(arr[i].tag) == tag and c[:p.size].tobytes() == ct, i
    assert cs.tobytes() == orc.checksum(p, hw=True), i
    arr[i].src = arr[i].dst = c.ctypes.data
eng.open_batch(E.AES256GCM, arr, nb, E.CRC_VERIFY, E.MEM_HOST)
assert all(arr[i].status == E.OK for i in range(nb))
assert all(c[:p.size].tobytes() == p.tobytes() for p, k, nn, c, cs in keep)
eng.close()
print("meta copy ok")
"""


def test_host_pipeline_metadata_copy_mode():
    """JFSX_PIPE_META=copy (descriptors and results as copies on the copy
    streams instead of the default pull kernel and pinned-mirror results), in
    a child process since the mode is read once: a host batch across several
    slots seals and opens bit-exact to the oracle, CRC arrays included."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, JFSX_PIPE_META="copy")
    out = subprocess.run([sys.executable, "-c", _META_COPY_SCRIPT % root], env=env, capture_output=True, text=True,
                         timeout=110)
    assert out.returncode == 0 and "meta copy ok" in out.stdout, out.stderr[-2000:]


def test_agg_data_encrypt_equals_data_encrypt(eng):
    """jfsx_agg_data_encrypt / _decrypt (dataEncryptor.Encrypt / Decrypt through
    the aggregator, encrypt.go:164-216) write the same object bytes and object
    checksum as the one-call form, from 20 threads."""
    wrapped = bytes(range(256))
    lens = [0, 1, 4 << 20, 100003, 32768] + [(i * 98765) % (1 << 20) for i in range(15)]
    got = [None] * len(lens)
    with E.Aggregator(eng, window_us=500, max_bytes=16 << 20) as agg:
        def work(i):
            p = orc.gen_block(71, i, lens[i]).tobytes()
            key, nonce = orc.gen_key(71, i)
            obj, crc = agg.data_encrypt(E.AES256GCM, key, nonce, wrapped, p, obj_crc=True)
            back = agg.data_decrypt(E.AES256GCM, key, obj)
            got[i] = (p, key, nonce, obj, crc, back)
        run_threads(len(lens), work)
    for p, key, nonce, obj, crc, back in got:
        assert (obj, crc) == eng.data_encrypt(E.AES256GCM, key, nonce, wrapped, p, obj_crc=True)
        assert back == p


def test_multi_device_context_device_batch():
    """A device-memory batch on a multi-device context runs each block on the
    GPU that owns its buffers (here every visible GPU's own blocks), bit-exact
    to the oracle; device memory of another process-local context routes too."""
    m = E.MultiEngine(0)
    try:
        specs, keep = [], []
        for d in range(m.ndev):
            mem = m.member(d)
            for i, n in enumerate([4 << 20, 12345, 0, 65536]):
                gi = 10 * d + i
                p = orc.gen_block(77, gi, n)
                src, dst = mem.alloc(max(n, 16)), mem.alloc(max(n, 16))
                if n:
                    src.upload(p)
                crc = mem.alloc(4 * max(1, -(-n // E.SEG)))
                key, nonce = orc.gen_key(77, gi)
                specs.append({"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": n, "crc": crc.ptr})
                keep.append((p, key, nonce, src, dst, crc, mem))
        arr, nb = E.Engine.make_blocks(specs)
        m.seal_batch(E.AES256GCM, arr, nb, E.CRC_GEN, E.MEM_DEVICE)
        for i, (p, key, nonce, src, dst, crc, mem) in enumerate(keep):
            c, tag = orc.seal(orc.AES256GCM, key, nonce, p, fast=True)
            assert bytes(arr[i].tag) == tag and dst.download(p.size).tobytes() == c, i
            assert crc.download().tobytes()[:len(orc.checksum(p))] == orc.checksum(p)
        for k in keep:
            for b in k[3:6]:
                b.free()
    finally:
        m.close()


def test_pinned_staging_on_the_gpu_numa_node(eng):
    """jfsx_alloc_pinned_node places the staging pages on the GPU's NUMA node
    (when the process may use that node), and the placement is reported."""
    node = eng.numa_node()
    nbytes = 256 << 20
    p = eng.alloc_pinned_node(nbytes)
    try:
        got = E.host_numa_node(p, nbytes)
        assert got != -2  # one node for the whole pool
        allowed = ""
        for line in open("/proc/self/status"):
            if line.startswith("Mems_allowed_list"):
                allowed = line.split(":", 1)[1].strip()
        nodes = set()
        for part in allowed.split(","):
            if "-" in part:
                a, b = part.split("-")
                nodes |= set(range(int(a), int(b) + 1))
            elif part:
                nodes.add(int(part))
        if node >= 0 and node in nodes and got >= 0:
            assert got == node, (got, node, allowed)
    finally:
        eng.free_pinned(p)
