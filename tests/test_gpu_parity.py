"""GPU parity: the HIP kernels (through the C-ABI) against the oracle and the
golden vectors.  Bit-exact: ciphertext, tags, CRC32C arrays, statuses."""
import hashlib
import json
import os

import numpy as np
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ALGOS = {"aes256gcm": E.AES256GCM, "chacha20poly1305": E.CHACHA20P1305}
ORC = {E.AES256GCM: orc.AES256GCM, E.CHACHA20P1305: orc.CHACHA20P1305}


@pytest.fixture(scope="module", params=["ttable", "bitslice"])
def eng(request):
    """Every parity case runs on both AES-GCM keystream kernels (T-table in LDS
    and the bitsliced VALU AES; the ChaCha path ignores the flag)."""
    e = E.Engine(0, E.CTX_BITSLICE if request.param == "bitslice" else 0)
    yield e
    e.close()


def _gold():
    with open(os.path.join(GOLD, "aead_vectors.json")) as f:
        return json.load(f)["vectors"]


def _seal_device(eng, algo, items, crc_mode=E.CRC_GEN):
    """items: list of (key, nonce, plaintext uint8 array). Returns (C list, tags, crc list, blks)."""
    bufs, specs, crcs = [], [], []
    for key, nonce, p in items:
        src = eng.alloc(max(p.size, 16))
        dst = eng.alloc(max(p.size, 16))
        src.upload(p)
        nseg = max(1, -(-p.size // E.SEG))
        cb = eng.alloc(4 * nseg)
        bufs += [src, dst, cb]
        crcs.append((cb, nseg))
        specs.append({"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": p.size, "crc": cb.ptr})
    arr, n = eng.make_blocks(specs)
    eng.seal_batch(algo, arr, n, crc_mode, E.MEM_DEVICE)
    outs = []
    for i, (key, nonce, p) in enumerate(items):
        c = bufs[3 * i + 1].download(p.size).tobytes()
        cb, nseg = crcs[i]
        outs.append((c, bytes(arr[i].tag), cb.download(4 * nseg).tobytes(), arr[i].status))
    return outs


@pytest.mark.parametrize("v", _gold(), ids=lambda v: "%s-%d" % (v["algo"], v["len"]))
def test_seal_golden_device(eng, v):
    algo = ALGOS[v["algo"]]
    p = orc.gen_block(v["seed"], v["block"], v["len"])
    key, nonce = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
    (c, tag, crc, st), = _seal_device(eng, algo, [(key, nonce, p)])
    assert st == E.OK
    assert tag.hex() == v["tag"]
    assert hashlib.sha256(c).hexdigest() == v["c_sha256"]
    assert crc.hex() == v["crc"]


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_seal_ragged_batch_vs_oracle(eng, algo):
    rng = np.random.default_rng(1 + algo)
    lens = [0, 1, 15, 16, 17, 1023, 1024, 1025, 32767, 32768, 32769, 65536 + 7, 524288, 524288 + 16,
            (1 << 20) + 3] + [int(x) for x in rng.integers(1, 3 << 20, 17)]
    items = []
    for i, n in enumerate(lens):
        key, nonce = orc.gen_key(11, i)
        items.append((key, nonce, orc.gen_block(11, i, n)))
    outs = _seal_device(eng, algo, items)
    for (key, nonce, p), (c, tag, crc, st) in zip(items, outs):
        c2, t2 = orc.seal(ORC[algo], key, nonce, p, fast=True)
        assert st == E.OK
        assert tag == t2, "len %d" % p.size
        assert c == c2, "len %d" % p.size
        assert crc == orc.checksum(p, hw=True), "len %d" % p.size


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_open_verify_roundtrip_and_failures(eng, algo):
    lens = [0, 5, 4096, 100000, 1 << 20, (4 << 20) - 5]
    bufs = []
    specs = []
    exp = []
    for i, n in enumerate(lens):
        key, nonce = orc.gen_key(21, i)
        p = orc.gen_block(21, i, n)
        c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
        crc = bytearray(orc.checksum(p, hw=True))
        if i == 3:
            tag = bytes([tag[0] ^ 1]) + tag[1:]            # tag corruption -> ETAG
        if i == 4:
            crc[4 * 7 + 2] ^= 0x10                          # CRC corruption of segment 7 -> ECRC
        src = eng.alloc(max(n, 16))
        dst = eng.alloc(max(n, 16))
        cb = eng.alloc(len(crc))
        src.upload(np.frombuffer(c, np.uint8))
        cb.upload(np.frombuffer(bytes(crc), np.uint8))
        bufs += [src, dst, cb]
        specs.append({"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": n, "tag": tag,
                      "crc": cb.ptr})
        exp.append((p, bytes(crc)))
    arr, nb = eng.make_blocks(specs)
    eng.open_batch(algo, arr, nb, E.CRC_VERIFY, E.MEM_DEVICE)
    for i, (p, crc) in enumerate(exp):
        b = arr[i]
        if i == 3:
            assert b.status == E.ETAG
            continue
        if i == 4:
            assert b.status == E.ECRC and b.crc_bad_seg == 7
            good = orc.crc32c(p[7 * E.SEG:8 * E.SEG].tobytes())
            assert b.crc_got == good
            assert b.crc_expect == int.from_bytes(crc[28:32], "big")
            continue
        assert b.status == E.OK, i
        assert bufs[3 * i + 1].download(p.size).tobytes() == p.tobytes()


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_host_mode_seal_open(eng, algo):
    key, nonce = orc.gen_key(3, 3)
    for n in (0, 1, 77, 32768 * 3 + 11, 1 << 20):
        p = orc.gen_block(3, n, n)
        c, tag, crc = eng.seal(algo, key, nonce, p, crc=True)
        c2, t2 = orc.seal(ORC[algo], key, nonce, p, fast=True)
        assert (c, tag) == (c2, t2)
        assert crc == orc.checksum(p)
        assert eng.open(algo, key, nonce, c, tag, crc=crc) == p.tobytes()
        bad = bytes([tag[0] ^ 0x80]) + tag[1:]
        assert eng.open(algo, key, nonce, c, bad) is None


@pytest.mark.parametrize("n", [0, 1, 16, 1000, 32767, 32768, 32769, 98309, 102400, 1 << 20, (4 << 20) - 1])
def test_checksum_matches_reference_semantics(eng, n):
    d = orc.gen_block(8, n, n)
    assert eng.checksum(d) == orc.checksum(d)


def test_crc_segments_device_gen_verify(eng):
    lens = [1, 32768, 65536, 100000, 4 << 20]
    bufs, rs = [], []
    for i, n in enumerate(lens):
        d = orc.gen_block(9, i, n)
        db = eng.alloc(n)
        db.upload(d)
        cb = eng.alloc(4 * max(1, -(-n // E.SEG)))
        bufs.append((d, db, cb))
    arr = (E.jfsx_range * len(lens))()
    for i, (d, db, cb) in enumerate(bufs):
        arr[i].data, arr[i].len, arr[i].crc = db.ptr, d.size, cb.ptr
    eng.crc32c_segments(arr, len(lens), E.CRC_GEN, E.MEM_DEVICE)
    for i, (d, db, cb) in enumerate(bufs):
        assert cb.download().tobytes()[:len(orc.checksum(d))] == orc.checksum(d)
    # corrupt one data byte of range 3 in segment 2 -> verify reports it
    d, db, cb = bufs[3]
    bad = d.copy()
    bad[2 * E.SEG + 5] ^= 1
    db.upload(bad)
    eng.crc32c_segments(arr, len(lens), E.CRC_VERIFY, E.MEM_DEVICE)
    for i in range(len(lens)):
        if i == 3:
            assert arr[i].status == E.ECRC and arr[i].bad_seg == 2
            assert arr[i].got == orc.crc32c(bad[2 * E.SEG:3 * E.SEG].tobytes())
        else:
            assert arr[i].status == E.OK


def test_crc_segments_ragged_many_tasks(eng):
    """crc_segments_k: ragged tails (byte-serial path), short segments, and
    ranges split over several 16-wave tasks (0.5-4 MiB each)."""
    rng = np.random.default_rng(5)
    lens = [0, 15, 16, 17, 1023, 1024, 1025, 32767, 32769, (512 << 10) + 3, (3 << 20) + 1, (9 << 20) + 13,
            (16 << 20)] + [int(x) for x in rng.integers(1, 1 << 21, 20)]
    bufs = []
    for i, n in enumerate(lens):
        d = orc.gen_block(21, i, n)
        db = eng.alloc(max(n, 16))
        if n:
            db.upload(d)
        cb = eng.alloc(4 * max(1, -(-n // E.SEG)))
        bufs.append((d, db, cb))
    arr = (E.jfsx_range * len(lens))()
    for i, (d, db, cb) in enumerate(bufs):
        arr[i].data, arr[i].len, arr[i].crc = db.ptr, d.size, cb.ptr
    eng.crc32c_segments(arr, len(lens), E.CRC_GEN, E.MEM_DEVICE)
    for i, (d, db, cb) in enumerate(bufs):
        want = orc.checksum(d)
        assert cb.download().tobytes()[:len(want)] == want, lens[i]
    eng.crc32c_segments(arr, len(lens), E.CRC_VERIFY, E.MEM_DEVICE)
    assert all(arr[i].status == E.OK for i in range(len(lens)))


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_object_format_vs_oracle(eng, algo):
    wrapped = bytes(range(256))
    for n in (0, 5, 4096 + 3):
        key, nonce = orc.gen_key(4, n)
        p = orc.gen_block(4, n, n)
        obj = eng.data_encrypt(algo, key, nonce, wrapped, p)
        assert obj == orc.data_encrypt(ORC[algo], key, nonce, wrapped, p)
        rc, back = eng.data_decrypt(algo, key, obj)
        assert rc == 0 and back == p.tobytes()
        assert eng.data_decrypt(algo, key, obj[:271])[0] == E.EMISFORMED
        bad = bytearray(obj)
        bad[-3] ^= 4
        assert eng.data_decrypt(algo, key, bytes(bad))[0] == E.ETAG


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_large_batch_sample_vs_oracle(eng, algo):
    """64 (GCM) / 16 (ChaCha) x 4 MiB device batch, every block checked against the oracle."""
    nb, L = (64 if algo == E.AES256GCM else 16), 4 << 20
    src = eng.alloc(nb * L)
    dst = eng.alloc(nb * L)
    crc = eng.alloc(nb * 512)
    specs = []
    eng.gen_synthetic_batch(src, L, [L] * nb, 0x4A465321, 0)
    for b in range(nb):
        key, nonce = orc.gen_key(0x4A465321, b)
        specs.append({"key": key, "nonce": nonce, "src": src.ptr + b * L, "dst": dst.ptr + b * L, "len": L,
                      "crc": crc.ptr + 512 * b})
    eng.sync()
    arr, n = eng.make_blocks(specs)
    eng.seal_batch(algo, arr, n, E.CRC_GEN, E.MEM_DEVICE)
    cs = crc.download()
    for b in range(nb):
        p = orc.gen_block(0x4A465321, b, L)
        key, nonce = orc.gen_key(0x4A465321, b)
        c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
        assert bytes(arr[b].tag) == tag, b
        assert dst.download(L, offset=b * L).tobytes() == c, b
        assert cs[512 * b:512 * (b + 1)].tobytes() == orc.checksum(p, hw=True), b


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_large_tasks_few_slots_vs_oracle(eng, algo):
    """A batch big enough that each 2 MiB block is cut into only 3 tasks: the
    finalize kernel then runs 64 threads per block while the slots' lifts
    reach H^(2^17) (the 64 GiB bench shape; a 64-thread finalize once staged
    only the first 16 powers).  Every tag and CRC array against the oracle,
    then Open of every block."""
    nb, L, seed = 200, 2 << 20, 0x4A465322
    src, dst, crc = eng.alloc(nb * L), eng.alloc(nb * L), eng.alloc(nb * 256)
    eng.gen_synthetic_batch(src, L, [L] * nb, seed, 0)
    specs = []
    for b in range(nb):
        key, nonce = orc.gen_key(seed, b)
        specs.append({"key": key, "nonce": nonce, "src": src.ptr + b * L, "dst": dst.ptr + b * L, "len": L,
                      "crc": crc.ptr + 256 * b})
    eng.sync()
    arr, n = eng.make_blocks(specs)
    eng.seal_batch(algo, arr, n, E.CRC_GEN, E.MEM_DEVICE)
    tags, crcs, _ = orc.expect_batch(ORC[algo], 8, [L] * nb, seed, 0, 256)
    got = np.frombuffer(b"".join(bytes(arr[b].tag) for b in range(nb)), np.uint8).reshape(nb, 16)
    assert (got == tags).all(axis=1).all(), np.nonzero(~(got == tags).all(axis=1))[0][:5]
    assert (crc.download().reshape(nb, 256) == crcs).all()
    for b in (0, nb - 1):
        key, nonce = orc.gen_key(seed, b)
        c, _ = orc.seal(ORC[algo], key, nonce, orc.gen_block(seed, b, L), fast=True)
        assert dst.download(L, offset=b * L).tobytes() == c, b
    ospecs = [dict(s, src=s["dst"], dst=s["src"], tag=bytes(arr[b].tag)) for b, s in enumerate(specs)]
    oarr, n = eng.make_blocks(ospecs)
    eng.open_batch(algo, oarr, n, E.CRC_VERIFY, E.MEM_DEVICE)
    assert all(oarr[b].status == E.OK for b in range(nb))


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_host_ingest_pipeline_ring(eng, algo):
    """MEM_HOST batches streamed through the context's persistent 8-slot host
    pipeline (kPipe slots shared by every caller; descriptors pulled into the
    slot by a kernel, results in its pinned mirror), with 1 MiB slots so one
    call is many groups that wrap the ring: seal + CRC and open + verify, one
    tag failure wiped on Open."""
    eng.set_slot_bytes(1 << 20)
    try:
        lens = [300000, 1 << 20, 5, 0, 777777, 2 << 20, 65536, 123457, 1 << 19, 4097]
        ps, keys, outs, crcs = [], [], [], []
        specs = []
        for i, n in enumerate(lens):
            key, nonce = orc.gen_key(31, i)
            p = orc.gen_block(31, i, n)
            o = np.zeros(max(n, 1), np.uint8)
            cb = np.zeros(4 * max(1, -(-n // E.SEG)), np.uint8)
            ps.append(p), keys.append((key, nonce)), outs.append(o), crcs.append(cb)
            specs.append({"key": key, "nonce": nonce, "src": p.ctypes.data if n else None, "dst": o.ctypes.data,
                          "len": n, "crc": cb.ctypes.data})
        arr, nb = eng.make_blocks(specs)
        eng.seal_batch(algo, arr, nb, E.CRC_GEN, E.MEM_HOST)
        ospecs = []
        plain = []
        for i, n in enumerate(lens):
            key, nonce = keys[i]
            c, tag = orc.seal(ORC[algo], key, nonce, ps[i], fast=True)
            assert bytes(arr[i].tag) == tag and outs[i][:n].tobytes() == c, i
            assert crcs[i].tobytes() == orc.checksum(ps[i], hw=True), i
            if i == 4:
                tag = bytes([tag[0] ^ 2]) + tag[1:]
            q = np.full(max(n, 1), 0xAB, np.uint8)
            plain.append(q)
            ospecs.append({"key": key, "nonce": nonce, "src": outs[i].ctypes.data, "dst": q.ctypes.data, "len": n,
                           "tag": tag, "crc": crcs[i].ctypes.data})
        oarr, nb = eng.make_blocks(ospecs)
        eng.open_batch(algo, oarr, nb, E.CRC_VERIFY, E.MEM_HOST)
        for i, n in enumerate(lens):
            if i == 4:
                assert oarr[i].status == E.ETAG
                assert not plain[i][:n].any()  # nothing released
            else:
                assert oarr[i].status == E.OK, i
                assert plain[i][:n].tobytes() == ps[i].tobytes(), i
    finally:
        eng.set_slot_bytes(256 << 20)


def test_gen_synthetic_batch_matches_oracle_stream(eng):
    """The bench's one-launch generator writes block block0+i at i*stride
    with its own (ragged) length: the oracle's gen_block stream."""
    lens = [0, 1, 15, 16, 17, 4095, 100003, 1 << 20, 65536]
    stride = 1 << 20
    buf = eng.alloc(stride * len(lens))
    buf.upload(np.full(stride * len(lens), 0x5A, np.uint8))
    eng.gen_synthetic_batch(buf, stride, lens, 77, 1000)
    for i, n in enumerate(lens):
        got = buf.download(stride, offset=i * stride)
        assert got[:n].tobytes() == orc.gen_block(77, 1000 + i, n).tobytes(), n
        assert (got[n:] == 0x5A).all(), n  # nothing past the block
