"""ctypes binding of libjfsx.so (include/jfsx.h).

This is the host side of the drop-in boundary.  Every compute call goes
through the HIP library; there is no CPU fallback: if libjfsx.so is missing
or no GPU is visible, constructing an Engine raises.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JFSX_LIB") or os.path.join(_HERE, "libjfsx.so")

AES256GCM = 0
CHACHA20P1305 = 1
CRC_NONE, CRC_GEN, CRC_VERIFY = 0, 1, 2
CRC_CT = 4  # flag: segment CRCs over the ciphertext (object checksum)
CRC_BOTH = 8  # flag (with CRC_GEN): plaintext CRCs, then ciphertext CRCs, in one array
CTX_BITSLICE = 1  # context flag: AES-GCM keystream from the bitsliced AES (VALU)
MEM_DEVICE, MEM_HOST = 0, 1
OK, ETAG, ECRC = 0, 1, 2
EOF = 3  # jfsx_cache_verify: short read
EFORMAT = 4  # malformed LZ4 block / zstd frame (the library's error)
EDSTSIZE = 5  # zstd: the output does not fit in dst_cap
EINVAL, ENODEV, EIO, ENOMEM, EMISFORMED, EAGAIN = -22, -19, -5, -12, -74, -11
SEG = 32 << 10

# every symbol include/jfsx.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "jfsx_abi_version", "jfsx_device_count", "jfsx_ctx_open", "jfsx_ctx_close", "jfsx_ctx_sync",
    "jfsx_ctx_stream", "jfsx_ctx_set_timing", "jfsx_ctx_set_slot_bytes", "jfsx_ctx_kernel_time", "jfsx_alloc_pinned",
    "jfsx_free_pinned", "jfsx_alloc_device", "jfsx_free_device", "jfsx_memcpy_h2d", "jfsx_memcpy_d2h",
    "jfsx_seal_batch", "jfsx_open_batch", "jfsx_crc32c_segments", "jfsx_checksum", "jfsx_cache_verify",
    "jfsx_data_encrypt", "jfsx_data_decrypt", "jfsx_parse_header", "jfsx_gen_synthetic", "jfsx_gen_key",
    "jfsx_debug_tables", "jfsx_crc32c_update", "jfsx_crc32c_combine", "jfsx_object_crc32c",
    "jfsx_rsa_key_new", "jfsx_rsa_key_free", "jfsx_rsa_oaep_decrypt_batch",
    "jfsx_seal_batch_async", "jfsx_open_batch_async", "jfsx_crc32c_segments_async", "jfsx_wait",
    "jfsx_agg_new", "jfsx_agg_free", "jfsx_agg_seal", "jfsx_agg_open", "jfsx_agg_crc32c", "jfsx_agg_stats",
    "jfsx_gen_synthetic_batch", "jfsx_mctx_open", "jfsx_mctx_close", "jfsx_mctx_ndev", "jfsx_mctx_ctx",
    "jfsx_mctx_seal_batch", "jfsx_mctx_open_batch", "jfsx_mctx_crc32c_segments", "jfsx_agg_new_mctx",
    "jfsx_agg_dev_batches", "jfsx_lz4_bound", "jfsx_lz4_compress_batch", "jfsx_lz4_decompress_batch",
    "jfsx_agg_lz4_compress", "jfsx_agg_lz4_decompress", "jfsx_mctx_lz4_compress_batch", "jfsx_mctx_lz4_decompress_batch",
    "jfsx_zstd_decompress_batch", "jfsx_agg_zstd_decompress", "jfsx_mctx_zstd_decompress_batch",
    "jfsx_last_error", "jfsx_zstd_bound", "jfsx_zstd_compress_batch", "jfsx_agg_zstd_compress",
    "jfsx_mctx_zstd_compress_batch", "jfsx_ctx_metrics", "jfsx_pcie_probe",
    "jfsx_device_numa_node", "jfsx_alloc_pinned_node", "jfsx_host_numa_node",
    "jfsx_agg_data_encrypt", "jfsx_agg_data_decrypt",
    "jfsx_data_encrypt_ex", "jfsx_data_decrypt_ex", "jfsx_agg_data_encrypt_ex", "jfsx_agg_data_decrypt_ex",
]


class EngineError(RuntimeError):
    """A batch-level failure; for JFSX_EIO / JFSX_ENOMEM the message carries
    the HIP error and call site the engine recorded (jfsx_last_error)."""

    def __init__(self, code, what, hip_error=0, detail=""):
        msg = "%s failed: jfsx error %d" % (what, code)
        if detail:
            msg += " [%s]" % detail
        super().__init__(msg)
        self.code = code
        self.hip_error = hip_error
        self.detail = detail


def last_error(ctx=None):
    """(hipError_t value, text) of the last HIP failure on ctx (None: this thread)."""
    e = ctypes.c_int()
    buf = ctypes.create_string_buffer(320)
    load_library().jfsx_last_error(ctx, ctypes.byref(e), buf, len(buf))
    return e.value, buf.value.decode(errors="replace")


def _raise(ctx, rc, what):
    he, txt = last_error(ctx) if rc in (EIO, ENOMEM) else (0, "")
    raise EngineError(rc, what, he, txt)


class jfsx_blk(ctypes.Structure):
    _fields_ = [
        ("key", ctypes.c_uint8 * 32), ("nonce", ctypes.c_uint8 * 12), ("reserved", ctypes.c_uint32),
        ("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("len", ctypes.c_uint64),
        ("tag", ctypes.c_uint8 * 16), ("crc", ctypes.c_void_p), ("status", ctypes.c_int32),
        ("crc_bad_seg", ctypes.c_int32), ("crc_got", ctypes.c_uint32), ("crc_expect", ctypes.c_uint32),
    ]


class jfsx_range(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("crc", ctypes.c_void_p),
        ("status", ctypes.c_int32), ("bad_seg", ctypes.c_int32), ("got", ctypes.c_uint32),
        ("expect", ctypes.c_uint32),
    ]


class jfsx_zblk(ctypes.Structure):
    _fields_ = [
        ("src", ctypes.c_void_p), ("src_len", ctypes.c_uint64), ("dst", ctypes.c_void_p),
        ("dst_cap", ctypes.c_uint64), ("out_len", ctypes.c_uint64), ("status", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


_METRIC_FIELDS = [
    "seal_batches", "seal_blocks", "seal_bytes", "open_batches", "open_blocks", "open_bytes", "open_fail",
    "crc_batches", "crc_ranges", "crc_bytes", "crc_fail", "lz4c_blocks", "lz4c_in", "lz4c_out",
    "lz4d_blocks", "lz4d_in", "lz4d_out", "lz4d_fail", "zstdc_blocks", "zstdc_in", "zstdc_out",
    "zstdd_blocks", "zstdd_in", "zstdd_out", "zstdd_fail", "zstd_serial",
]


class jfsx_metrics(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in _METRIC_FIELDS] + [
        ("kernel_ms", ctypes.c_double), ("kernel_launches", ctypes.c_uint64)]


_lib = None
_lib_lock = threading.Lock()


def load_library(path=LIB_PATH):
    """Load libjfsx.so and declare its signatures.  Raises if it is absent."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise ImportError("libjfsx.so not built (%s); run __graft_entry__.build()" % path)
        L = ctypes.CDLL(path)
        P, I, U64, U32, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t
        PP = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "jfsx_abi_version": (I, []),
            "jfsx_last_error": (I, [P, ctypes.POINTER(I), ctypes.c_char_p, SZ]),
            "jfsx_device_count": (I, [ctypes.POINTER(I)]),
            "jfsx_ctx_open": (I, [I, U32, PP]),
            "jfsx_ctx_close": (I, [P]),
            "jfsx_ctx_sync": (I, [P]),
            "jfsx_ctx_stream": (P, [P]),
            "jfsx_ctx_set_timing": (I, [P, I]),
            "jfsx_ctx_set_slot_bytes": (I, [P, U64]),
            "jfsx_ctx_kernel_time": (I, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64), I]),
            "jfsx_ctx_metrics": (I, [P, ctypes.POINTER(jfsx_metrics), I]),
            "jfsx_pcie_probe": (I, [P, U64, ctypes.POINTER(ctypes.c_double)]),
            "jfsx_alloc_pinned": (I, [P, SZ, PP]),
            "jfsx_device_numa_node": (I, [I, ctypes.POINTER(I)]),
            "jfsx_alloc_pinned_node": (I, [P, SZ, I, PP]),
            "jfsx_host_numa_node": (I, [P, SZ, ctypes.POINTER(I)]),
            "jfsx_agg_data_encrypt": (I, [P, I, P, P, P, I, P, U64, P, U64, ctypes.POINTER(U64), P]),
            "jfsx_agg_data_decrypt": (I, [P, I, P, P, U64, P, U64, ctypes.POINTER(U64), P, P]),
            "jfsx_data_encrypt_ex": (I, [P, I, P, P, P, I, P, U64, P, U64, ctypes.POINTER(U64), P, P]),
            "jfsx_data_decrypt_ex": (I, [P, I, P, P, U64, P, U64, ctypes.POINTER(U64), P, P, P]),
            "jfsx_agg_data_encrypt_ex": (I, [P, I, P, P, P, I, P, U64, P, U64, ctypes.POINTER(U64), P, P]),
            "jfsx_agg_data_decrypt_ex": (I, [P, I, P, P, U64, P, U64, ctypes.POINTER(U64), P, P, P]),
            "jfsx_free_pinned": (I, [P, P]),
            "jfsx_alloc_device": (I, [P, SZ, PP]),
            "jfsx_free_device": (I, [P, P]),
            "jfsx_memcpy_h2d": (I, [P, P, P, SZ]),
            "jfsx_memcpy_d2h": (I, [P, P, P, SZ]),
            "jfsx_seal_batch": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_open_batch": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_crc32c_segments": (I, [P, I, ctypes.POINTER(jfsx_range), I, I]),
            "jfsx_checksum": (I, [P, P, U64, P]),
            "jfsx_cache_verify": (I, [P, P, U64, U64, I, U64, U64, P, ctypes.POINTER(U64),
                                      ctypes.POINTER(U32), ctypes.POINTER(U32), ctypes.POINTER(ctypes.c_int64)]),
            "jfsx_data_encrypt": (I, [P, I, P, P, P, I, P, U64, P, U64, ctypes.POINTER(U64), P]),
            "jfsx_data_decrypt": (I, [P, I, P, P, U64, P, U64, ctypes.POINTER(U64), P, P]),
            "jfsx_crc32c_update": (ctypes.c_uint32, [ctypes.c_uint32, P, U64]),
            "jfsx_crc32c_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, U64]),
            "jfsx_object_crc32c": (I, [P, U64, P, U64, P, P]),
            "jfsx_parse_header": (I, [P, U64, ctypes.POINTER(I), ctypes.POINTER(I)]),
            "jfsx_gen_synthetic": (I, [P, P, U64, U64, U64]),
            "jfsx_gen_key": (None, [U64, U64, P, P]),
            "jfsx_debug_tables": (I, [P, P, P]),
            "jfsx_rsa_key_new": (I, [P, P, P, P, P, P, I, P, I, PP]),
            "jfsx_rsa_key_free": (I, [P]),
            "jfsx_rsa_oaep_decrypt_batch": (I, [P, P, I, P, U64, P, P, U64, P]),
            "jfsx_seal_batch_async": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I, ctypes.POINTER(U64)]),
            "jfsx_open_batch_async": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I, ctypes.POINTER(U64)]),
            "jfsx_crc32c_segments_async": (I, [P, I, ctypes.POINTER(jfsx_range), I, I, ctypes.POINTER(U64)]),
            "jfsx_wait": (I, [P, U64, I]),
            "jfsx_agg_new": (I, [P, I, U64, U32, PP]),
            "jfsx_agg_free": (I, [P]),
            "jfsx_agg_seal": (I, [P, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_agg_open": (I, [P, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_agg_crc32c": (I, [P, ctypes.POINTER(jfsx_range), I, I]),
            "jfsx_agg_stats": (I, [P, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
            "jfsx_gen_synthetic_batch": (I, [P, P, U64, I, P, U64, U64]),
            "jfsx_mctx_open": (I, [U64, U32, PP]),
            "jfsx_mctx_close": (I, [P]),
            "jfsx_mctx_ndev": (I, [P]),
            "jfsx_mctx_ctx": (P, [P, I]),
            "jfsx_mctx_seal_batch": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_mctx_open_batch": (I, [P, I, I, ctypes.POINTER(jfsx_blk), I, I]),
            "jfsx_mctx_crc32c_segments": (I, [P, I, ctypes.POINTER(jfsx_range), I, I]),
            "jfsx_agg_new_mctx": (I, [P, I, U64, U32, PP]),
            "jfsx_agg_dev_batches": (I, [P, I, ctypes.POINTER(U64)]),
            "jfsx_lz4_bound": (U64, [U64]),
            "jfsx_lz4_compress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_lz4_decompress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_agg_lz4_compress": (I, [P, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_agg_lz4_decompress": (I, [P, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_mctx_lz4_compress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_mctx_lz4_decompress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_zstd_decompress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_agg_zstd_decompress": (I, [P, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_mctx_zstd_decompress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_zstd_bound": (U64, [U64]),
            "jfsx_zstd_compress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_agg_zstd_compress": (I, [P, ctypes.POINTER(jfsx_zblk), I]),
            "jfsx_mctx_zstd_compress_batch": (I, [P, I, ctypes.POINTER(jfsx_zblk), I]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, DeviceBuffer):
        return a.ptr
    if isinstance(a, int):
        return a
    raise TypeError(type(a))


def _u8(b):
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b.reshape(-1).view(np.uint8))
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def _obj_plain_len(o):
    """plaintext length an encrypted object's header implies (encrypt.go:197-215), 0 if malformed"""
    if o.size < 3:
        return 0
    return max(0, int(o.size) - 3 - ((int(o[0]) << 8) | int(o[1])) - int(o[2]) - 16)


def debug_tables():
    """Host-built lookup tables (no device needed)."""
    L = load_library()
    aes = np.empty(16384, np.uint32)
    crc = np.empty(8192, np.uint32)
    crcx = np.empty(192, np.uint32)
    L.jfsx_debug_tables(aes.ctypes.data, crc.ctypes.data, crcx.ctypes.data)
    return aes, crc, crcx


def gen_key(seed, block):
    key = np.empty(32, np.uint8)
    nonce = np.empty(12, np.uint8)
    load_library().jfsx_gen_key(seed, block, key.ctypes.data, nonce.ctypes.data)
    return key.tobytes(), nonce.tobytes()


def lz4_bound(n):
    """LZ4_compressBound (compress.go:111 CompressBound)."""
    return load_library().jfsx_lz4_bound(n)


def zstd_bound(n):
    """ZSTD_compressBound (compress.go:80 CompressBound)."""
    return load_library().jfsx_zstd_bound(n)


def device_numa_node(device):
    """jfsx_device_numa_node: the host NUMA node closest to a GPU (-1 unknown)."""
    v = ctypes.c_int(-1)
    load_library().jfsx_device_numa_node(device, ctypes.byref(v))
    return v.value


def host_numa_node(ptr, nbytes):
    """jfsx_host_numa_node: NUMA node of host pages (sampled; -1 unknown, -2 mixed)."""
    v = ctypes.c_int(-1)
    load_library().jfsx_host_numa_node(ptr, nbytes, ctypes.byref(v))
    return v.value


def device_count():
    n = ctypes.c_int()
    rc = load_library().jfsx_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class DeviceBuffer:
    """Device memory owned by an Engine (hipMalloc through the C-ABI)."""

    def __init__(self, eng, nbytes):
        self.eng = eng
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        rc = eng.L.jfsx_alloc_device(eng.ctx, max(self.nbytes, 16), ctypes.byref(p))
        if rc:
            _raise(eng.ctx, rc, "jfsx_alloc_device(%d)" % nbytes)
        self.ptr = p.value

    def free(self):
        if self.ptr:
            self.eng.L.jfsx_free_device(self.eng.ctx, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, host, offset=0):
        h = _u8(host)
        if h.size:
            self.eng._check(self.eng.L.jfsx_memcpy_h2d(self.eng.ctx, self.ptr + offset, h.ctypes.data, h.size),
                            "h2d")

    def download(self, nbytes=None, offset=0):
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(max(n, 1), np.uint8)
        if n:
            self.eng._check(self.eng.L.jfsx_memcpy_d2h(self.eng.ctx, out.ctypes.data, self.ptr + offset, n), "d2h")
        return out[:n]


class Engine:
    """One GPU context (device ordinal + HIP stream + workspace)."""

    def __init__(self, device=0, flags=0):
        """flags: 0 or CTX_BITSLICE (AES-GCM keystream from the bitsliced AES)."""
        self.L = load_library()
        if device_count() <= device:
            raise RuntimeError("jfsx: no HIP device %d visible (the engine has no CPU path)" % device)
        ctx = ctypes.c_void_p()
        rc = self.L.jfsx_ctx_open(device, flags, ctypes.byref(ctx))
        if rc:
            raise EngineError(rc, "jfsx_ctx_open(%d)" % device)
        self.ctx = ctx.value
        self.device = device

    def close(self):
        if getattr(self, "ctx", None):
            if not getattr(self, "_borrowed", False):
                self.L.jfsx_ctx_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc:
            _raise(self.ctx, rc, what)

    def last_error(self):
        """(hipError_t, text) of the last HIP failure on this context."""
        return last_error(self.ctx)

    # -- memory ----------------------------------------------------------
    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    def gen_synthetic(self, buf, length, seed, block, offset=0):
        self._check(self.L.jfsx_gen_synthetic(self.ctx, buf.ptr + offset, length, seed, block), "gen_synthetic")

    def gen_synthetic_batch(self, buf, stride, lens, seed, block0, offset=0):
        """Blocks block0 .. block0+len(lens)-1 at buf + offset + i*stride, one launch."""
        ln = np.asarray(lens, dtype=np.uint64)
        self._check(self.L.jfsx_gen_synthetic_batch(self.ctx, buf.ptr + offset, stride, ln.size, ln.ctypes.data,
                                                    seed, block0), "gen_synthetic_batch")

    def sync(self):
        self._check(self.L.jfsx_ctx_sync(self.ctx), "sync")

    def set_slot_bytes(self, nbytes):
        self._check(self.L.jfsx_ctx_set_slot_bytes(self.ctx, nbytes), "set_slot_bytes")

    def alloc_pinned(self, nbytes):
        p = ctypes.c_void_p()
        self._check(self.L.jfsx_alloc_pinned(self.ctx, max(nbytes, 16), ctypes.byref(p)), "alloc_pinned")
        return p.value

    def free_pinned(self, ptr):
        self.L.jfsx_free_pinned(self.ctx, ptr)

    def alloc_pinned_node(self, nbytes, node=-1):
        """Pinned host memory bound to NUMA node `node` (-1: this GPU's node)."""
        p = ctypes.c_void_p()
        self._check(self.L.jfsx_alloc_pinned_node(self.ctx, max(nbytes, 16), node, ctypes.byref(p)),
                    "alloc_pinned_node")
        return p.value

    def numa_node(self):
        """Host NUMA node closest to this GPU (-1 unknown)."""
        return device_numa_node(self.device)

    def set_timing(self, on):
        self.L.jfsx_ctx_set_timing(self.ctx, 1 if on else 0)

    def kernel_time(self, reset=True):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        self.L.jfsx_ctx_kernel_time(self.ctx, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0)
        return ms.value, n.value

    def pcie_probe(self, nbytes=1 << 30):
        """jfsx_pcie_probe: GB/s H2D alone, D2H alone, and each while both run."""
        out = (ctypes.c_double * 4)()
        self._check(self.L.jfsx_pcie_probe(self.ctx, nbytes, out), "jfsx_pcie_probe")
        return {"h2d": round(out[0], 2), "d2h": round(out[1], 2), "duplex_h2d": round(out[2], 2),
                "duplex_d2h": round(out[3], 2)}

    def metrics(self, reset=False):
        """jfsx_ctx_metrics as a dict (counters since open or the last reset)."""
        m = jfsx_metrics()
        self._check(self.L.jfsx_ctx_metrics(self.ctx, ctypes.byref(m), 1 if reset else 0), "jfsx_ctx_metrics")
        return {f: getattr(m, f) for f, _ in jfsx_metrics._fields_}

    # -- batches -----------------------------------------------------------
    @staticmethod
    def make_blocks(specs):
        """specs: iterable of dicts with key, nonce, src, dst, len, [tag], [crc] (pointers as ints)."""
        specs = list(specs)
        arr = (jfsx_blk * max(len(specs), 1))()
        for i, s in enumerate(specs):
            b = arr[i]
            ctypes.memmove(b.key, bytes(s["key"]), 32)
            ctypes.memmove(b.nonce, bytes(s["nonce"]), 12)
            b.src = s.get("src")
            b.dst = s.get("dst")
            b.len = s["len"]
            if s.get("tag") is not None:
                ctypes.memmove(b.tag, bytes(s["tag"]), 16)
            b.crc = s.get("crc")
        return arr, len(specs)

    def seal_batch(self, algo, blks, n, crc_mode=CRC_GEN, mem=MEM_DEVICE):
        self._check(self.L.jfsx_seal_batch(self.ctx, algo, n, blks, crc_mode, mem), "jfsx_seal_batch")

    def open_batch(self, algo, blks, n, crc_mode=CRC_NONE, mem=MEM_DEVICE):
        self._check(self.L.jfsx_open_batch(self.ctx, algo, n, blks, crc_mode, mem), "jfsx_open_batch")

    def crc32c_segments(self, ranges, n, mode=CRC_GEN, mem=MEM_DEVICE):
        self._check(self.L.jfsx_crc32c_segments(self.ctx, n, ranges, mode, mem), "jfsx_crc32c_segments")

    # -- LZ4 stage (jfsx_lz4_*) -------------------------------------------
    @staticmethod
    def make_zblocks(specs):
        """specs: iterable of (src_ptr, src_len, dst_ptr, dst_cap)."""
        specs = list(specs)
        arr = (jfsx_zblk * max(len(specs), 1))()
        for i, (sp, sl, dp, dc) in enumerate(specs):
            arr[i].src, arr[i].src_len, arr[i].dst, arr[i].dst_cap = sp, sl, dp, dc
        return arr, len(specs)

    def lz4_compress_batch(self, zblks, n, mem=MEM_DEVICE):
        self._check(self.L.jfsx_lz4_compress_batch(self.ctx, n, zblks, mem), "jfsx_lz4_compress_batch")

    def lz4_decompress_batch(self, zblks, n, mem=MEM_DEVICE):
        self._check(self.L.jfsx_lz4_decompress_batch(self.ctx, n, zblks, mem), "jfsx_lz4_decompress_batch")

    def lz4_compress(self, datas):
        """Host buffers in, list of compressed bytes out (one GPU batch)."""
        srcs = [_u8(d) for d in datas]
        dsts = [np.empty(max(int(lz4_bound(s.size)), 1), np.uint8) for s in srcs]
        arr, n = self.make_zblocks((s.ctypes.data, s.size, d.ctypes.data, int(lz4_bound(s.size)))
                                   for s, d in zip(srcs, dsts))
        self.lz4_compress_batch(arr, n, MEM_HOST)
        return [d[:arr[i].out_len].tobytes() for i, d in enumerate(dsts)]

    def lz4_decompress(self, datas, caps):
        """Host buffers in; list of (status, bytes) out, decoded into dst of caps[i] bytes."""
        srcs = [_u8(d) for d in datas]
        dsts = [np.empty(max(int(c), 1), np.uint8) for c in caps]
        arr, n = self.make_zblocks((s.ctypes.data, s.size, d.ctypes.data, int(c))
                                   for s, d, c in zip(srcs, dsts, caps))
        self.lz4_decompress_batch(arr, n, MEM_HOST)
        return [(arr[i].status, d[:arr[i].out_len].tobytes()) for i, d in enumerate(dsts)]

    # -- Zstandard decompression (jfsx_zstd_decompress_batch) -------------
    def zstd_decompress_batch(self, zblks, n, mem=MEM_DEVICE):
        self._check(self.L.jfsx_zstd_decompress_batch(self.ctx, n, zblks, mem), "jfsx_zstd_decompress_batch")

    def zstd_compress_batch(self, zblks, n, mem=MEM_DEVICE):
        self._check(self.L.jfsx_zstd_compress_batch(self.ctx, n, zblks, mem), "jfsx_zstd_compress_batch")

    def zstd_compress(self, datas):
        """Host buffers in; list of level-1 zstd frames out (one GPU batch)."""
        srcs = [_u8(d) for d in datas]
        caps = [int(zstd_bound(s.size)) for s in srcs]
        dsts = [np.empty(max(c, 1), np.uint8) for c in caps]
        arr, n = self.make_zblocks((s.ctypes.data, s.size, d.ctypes.data, c) for s, d, c in zip(srcs, dsts, caps))
        self.zstd_compress_batch(arr, n, MEM_HOST)
        return [d[:arr[i].out_len].tobytes() for i, d in enumerate(dsts)]

    def zstd_decompress(self, datas, caps):
        """Host buffers of zstd frames in; list of (status, bytes) out (dst of caps[i] bytes)."""
        srcs = [_u8(d) for d in datas]
        dsts = [np.empty(max(int(c), 1), np.uint8) for c in caps]
        arr, n = self.make_zblocks((s.ctypes.data, s.size, d.ctypes.data, int(c))
                                   for s, d, c in zip(srcs, dsts, caps))
        self.zstd_decompress_batch(arr, n, MEM_HOST)
        # why each object went to the serial decoder (0: it did not; jfsx.h)
        self.zstd_serial_reasons = [arr[i].reserved for i in range(len(dsts))]
        return [(arr[i].status, d[:arr[i].out_len].tobytes()) for i, d in enumerate(dsts)]

    # -- asynchronous batches (jfsx_*_async + jfsx_wait) ------------------
    def _ticket(self, fn, what, *args):
        t = ctypes.c_uint64()
        self._check(fn(self.ctx, *args, ctypes.byref(t)), what)
        return t.value

    def seal_batch_async(self, algo, blks, n, crc_mode=CRC_GEN, mem=MEM_DEVICE):
        """Queue a seal batch; returns a ticket for wait().  blks and the
        buffers must stay alive until wait() returns."""
        return self._ticket(self.L.jfsx_seal_batch_async, "jfsx_seal_batch_async", algo, n, blks, crc_mode, mem)

    def open_batch_async(self, algo, blks, n, crc_mode=CRC_NONE, mem=MEM_DEVICE):
        return self._ticket(self.L.jfsx_open_batch_async, "jfsx_open_batch_async", algo, n, blks, crc_mode, mem)

    def crc32c_segments_async(self, ranges, n, mode=CRC_GEN, mem=MEM_DEVICE):
        return self._ticket(self.L.jfsx_crc32c_segments_async, "jfsx_crc32c_segments_async", n, ranges, mode, mem)

    def wait(self, ticket, timeout_ms=-1):
        """Return code of the batch (raises on a batch-level error); False if
        it has not finished within timeout_ms (the ticket stays live)."""
        rc = self.L.jfsx_wait(self.ctx, ticket, timeout_ms)
        if rc == EAGAIN:
            return False
        self._check(rc, "jfsx_wait")
        return True

    # -- host-memory conveniences -------------------------------------------
    def seal(self, algo, key, nonce, plaintext, crc=False):
        """Seal one host buffer; returns (ciphertext, tag[, crc bytes])."""
        p = _u8(plaintext)
        out = np.empty(max(p.size, 1), np.uint8)
        cbuf = np.zeros(4 * max(1, -(-p.size // SEG)), np.uint8)
        arr, n = self.make_blocks([{"key": key, "nonce": nonce, "src": p.ctypes.data if p.size else None,
                                    "dst": out.ctypes.data, "len": p.size,
                                    "crc": cbuf.ctypes.data if crc else None}])
        self.seal_batch(algo, arr, n, CRC_GEN if crc else CRC_NONE, MEM_HOST)
        c, tag = out[:p.size].tobytes(), bytes(arr[0].tag)
        return (c, tag, cbuf.tobytes()) if crc else (c, tag)

    def open(self, algo, key, nonce, ciphertext, tag, crc=None):
        """Open one host buffer; returns plaintext or None on authentication failure."""
        c = _u8(ciphertext)
        out = np.zeros(max(c.size, 1), np.uint8)
        cb = _u8(crc) if crc is not None else None
        arr, n = self.make_blocks([{"key": key, "nonce": nonce, "src": c.ctypes.data if c.size else None,
                                    "dst": out.ctypes.data, "len": c.size, "tag": tag,
                                    "crc": cb.ctypes.data if cb is not None else None}])
        self.open_batch(algo, arr, n, CRC_VERIFY if cb is not None else CRC_NONE, MEM_HOST)
        b = arr[0]
        if b.status == ETAG:
            return None
        if b.status == ECRC:
            raise ChecksumError(b.crc_got, b.crc_expect, b.crc_bad_seg)
        return out[:c.size].tobytes()

    def checksum(self, data):
        d = _u8(data)
        out = np.empty(4 * max(1, -(-d.size // SEG)), np.uint8)
        self._check(self.L.jfsx_checksum(self.ctx, d.ctypes.data if d.size else None, d.size, out.ctypes.data),
                    "jfsx_checksum")
        return out.tobytes()

    def cache_verify(self, file_img, length, level, off, size):
        """cacheFile.ReadAt on an in-memory cache file image.
        Returns (rc, data, n, got, expect, bad_seg)."""
        f = _u8(file_img)
        out = np.zeros(max(size, 1), np.uint8)
        n = ctypes.c_uint64()
        got = ctypes.c_uint32()
        exp = ctypes.c_uint32()
        seg = ctypes.c_int64()
        rc = self.L.jfsx_cache_verify(self.ctx, f.ctypes.data, f.size, length, level, off, size, out.ctypes.data,
                                      ctypes.byref(n), ctypes.byref(got), ctypes.byref(exp), ctypes.byref(seg))
        if rc < 0:
            raise EngineError(rc, "jfsx_cache_verify")
        return rc, out[:size].tobytes(), n.value, got.value, exp.value, seg.value

    def data_encrypt(self, algo, key, nonce, wrapped, plaintext, obj_crc=False, seg_crc=False):
        """Object bytes (encrypt.go:182-193); with obj_crc=True also the
        object-store checksum of them (checksum.go:31-53); with seg_crc=True
        also checksum() of the plaintext (disk_cache.go:1218-1231), from the
        same call: obj, or a tuple (obj[, crc][, seg_crcs])."""
        p = _u8(plaintext)
        cap = 3 + len(wrapped) + 12 + p.size + 16
        out = np.empty(cap, np.uint8)
        w = _u8(wrapped)
        olen = ctypes.c_uint64()
        crc = ctypes.c_uint32()
        segs = np.zeros(4 * max(1, -(-p.size // SEG)), np.uint8)
        self._check(self.L.jfsx_data_encrypt_ex(self.ctx, algo, bytes(key), bytes(nonce),
                                                w.ctypes.data if w.size else None, w.size,
                                                p.ctypes.data if p.size else None, p.size, out.ctypes.data, cap,
                                                ctypes.byref(olen), ctypes.byref(crc) if obj_crc else None,
                                                segs.ctypes.data if seg_crc else None),
                    "jfsx_data_encrypt_ex")
        obj = out[:olen.value].tobytes()
        res = (obj,) + ((crc.value,) if obj_crc else ()) + ((segs.tobytes(),) if seg_crc else ())
        return res if len(res) > 1 else obj

    def data_decrypt(self, algo, key, obj, expect_crc=None, seg_crc=False):
        """(rc, plaintext) -- rc JFSX_ECRC when expect_crc is given and the
        object checksum differs; then .last_got_crc holds the computed value.
        With seg_crc=True, (rc, plaintext, checksum() of the plaintext)."""
        o = _u8(obj)
        out = np.empty(max(o.size, 1), np.uint8)
        olen = ctypes.c_uint64()
        exp = ctypes.c_uint32(expect_crc or 0)
        got = ctypes.c_uint32()
        segs = np.full(4 * max(1, -(-_obj_plain_len(o) // SEG)), 0xAA, np.uint8)
        rc = self.L.jfsx_data_decrypt_ex(self.ctx, algo, bytes(key), o.ctypes.data, o.size, out.ctypes.data,
                                         out.size, ctypes.byref(olen),
                                         ctypes.byref(exp) if expect_crc is not None else None,
                                         ctypes.byref(got) if expect_crc is not None else None,
                                         segs.ctypes.data if seg_crc else None)
        self.last_got_crc = got.value
        pt = out[:olen.value].tobytes() if rc == 0 else b""
        return (rc, pt, segs.tobytes()) if seg_crc else (rc, pt)

    def rsa_key(self, p, q, dp, dq, qinv, label=b"keys"):
        """Device copy of an RSA-2048 private key from its CRT components
        (big-endian, 128 bytes each) for oaep_decrypt_batch."""
        k = ctypes.c_void_p()
        lab = bytes(label)
        self._check(self.L.jfsx_rsa_key_new(self.ctx, bytes(p), bytes(q), bytes(dp), bytes(dq), bytes(qinv), len(p),
                                            lab if lab else None, len(lab), ctypes.byref(k)), "jfsx_rsa_key_new")
        return k.value

    def rsa_key_free(self, key):
        if key:
            self.L.jfsx_rsa_key_free(key)

    def oaep_decrypt_batch(self, key, ciphertexts):
        """rsa.DecryptOAEP(sha256, priv, c, label) for every c at once: a list
        of plaintexts, None where Go returns the decryption error."""
        n = len(ciphertexts)
        if n == 0:
            return []
        stride = max(1, max(len(c) for c in ciphertexts))
        buf = np.zeros(n * stride, np.uint8)
        lens = np.zeros(n, np.uint32)
        for i, c in enumerate(ciphertexts):
            c = bytes(c)
            buf[i * stride:i * stride + len(c)] = np.frombuffer(c, np.uint8)
            lens[i] = len(c)
        msg = np.zeros(n * 256, np.uint8)
        mlen = np.zeros(n, np.int32)
        self._check(self.L.jfsx_rsa_oaep_decrypt_batch(self.ctx, key, n, buf.ctypes.data, stride, lens.ctypes.data,
                                                       msg.ctypes.data, 256, mlen.ctypes.data),
                    "jfsx_rsa_oaep_decrypt_batch")
        return [None if mlen[i] < 0 else msg[256 * i:256 * i + mlen[i]].tobytes() for i in range(n)]

    def crc32c_update(self, crc, data):
        return crc32c_update(crc, data)

    def crc32c_combine(self, a, b, len_b):
        return crc32c_combine(a, b, len_b)

    def object_crc32c(self, hdr, seg_crcs, clen, tag):
        return object_crc32c(hdr, seg_crcs, clen, tag)


# host-side CRC32C helpers of the C-ABI (no device needed)
def crc32c_update(crc, data):
    """crc32.Update(crc, MakeTable(Castagnoli), data)."""
    d = _u8(data)
    return load_library().jfsx_crc32c_update(crc, d.ctypes.data if d.size else None, d.size)


def crc32c_combine(a, b, len_b):
    return load_library().jfsx_crc32c_combine(a, b, len_b)


def object_crc32c(hdr, seg_crcs, clen, tag):
    """generateChecksum's value of hdr || C || tag from C's BE segment CRCs."""
    h, sc = _u8(hdr), _u8(seg_crcs)
    out = ctypes.c_uint32()
    rc = load_library().jfsx_object_crc32c(h.ctypes.data if h.size else None, h.size,
                                           sc.ctypes.data if sc.size else None, clen, bytes(tag),
                                           ctypes.byref(out))
    if rc:
        raise EngineError(rc, "jfsx_object_crc32c")
    return out.value


class ChecksumError(Exception):
    """"data checksum %d != expect %d" (pkg/chunk/disk_cache.go:1324)."""

    def __init__(self, got, expect, seg=-1):
        super().__init__("data checksum %d != expect %d" % (got, expect))
        self.got, self.expect, self.seg = got, expect, seg


class MultiEngine:
    """jfsx_mctx: one context per selected GPU (dev_mask bit d = device d, 0 =
    all visible).  Host-memory batches are cut into one contiguous run of
    blocks per device, balanced by bytes; device-memory batches run each block
    on the GPU that owns its buffers.  The parts run concurrently on one
    persistent worker per device (independent blocks, no
    collective)."""

    def __init__(self, dev_mask=0, flags=0):
        self.L = load_library()
        m = ctypes.c_void_p()
        rc = self.L.jfsx_mctx_open(dev_mask, flags, ctypes.byref(m))
        if rc:
            raise EngineError(rc, "jfsx_mctx_open(0x%x)" % dev_mask)
        self.m = m.value
        self.devices = [d for d in range(device_count()) if not dev_mask or (dev_mask >> d) & 1]

    @property
    def ndev(self):
        return self.L.jfsx_mctx_ndev(self.m)

    def member(self, i):
        """An Engine view of device slot i's context (owned by the MultiEngine:
        closing the view does not close the context)."""
        e = Engine.__new__(Engine)
        e.L = self.L
        e.ctx = self.L.jfsx_mctx_ctx(self.m, i)
        if not e.ctx:
            raise EngineError(EINVAL, "jfsx_mctx_ctx(%d)" % i)
        e.device = self.devices[i]
        e._borrowed = True
        return e

    def close(self):
        if getattr(self, "m", None):
            self.L.jfsx_mctx_close(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _errs(self):
        return [last_error(self.L.jfsx_mctx_ctx(self.m, i)) for i in range(self.ndev)]

    def _call(self, what, fn, *args):
        """Run one mctx entry point; a failure raises with the HIP error of
        every member context whose record this call changed (each device's
        part runs on its own worker and records on its own context; records
        left by earlier calls are not reported), or the calling thread's
        record when none did."""
        before = self._errs()
        rc = fn(self.m, *args)
        if not rc:
            return
        if rc in (EIO, ENOMEM):
            recs = [(i, he, txt) for i, ((he, txt), old) in enumerate(zip(self._errs(), before))
                    if (he or txt) and (he, txt) != old]
            if recs:
                raise EngineError(rc, what, recs[0][1], "; ".join("device %d: %s" % (i, t) for i, _, t in recs))
        _raise(None, rc, what)

    def _check(self, rc, what):
        """For calls made outside _call (the aggregator's): every member
        context's record."""
        if not rc:
            return
        if rc in (EIO, ENOMEM):
            recs = [(i, he, txt) for i, (he, txt) in enumerate(self._errs()) if he or txt]
            if recs:
                raise EngineError(rc, what, recs[0][1], "; ".join("device %d: %s" % (i, t) for i, _, t in recs))
        _raise(None, rc, what)

    def seal_batch(self, algo, blks, n, crc_mode=CRC_GEN, mem=MEM_HOST):
        self._call("jfsx_mctx_seal_batch", self.L.jfsx_mctx_seal_batch, algo, n, blks, crc_mode, mem)

    def open_batch(self, algo, blks, n, crc_mode=CRC_NONE, mem=MEM_HOST):
        self._call("jfsx_mctx_open_batch", self.L.jfsx_mctx_open_batch, algo, n, blks, crc_mode, mem)

    def crc32c_segments(self, ranges, n, mode=CRC_GEN, mem=MEM_HOST):
        self._call("jfsx_mctx_crc32c_segments", self.L.jfsx_mctx_crc32c_segments, n, ranges, mode, mem)

    def lz4_compress_batch(self, zblks, n, mem=MEM_HOST):
        self._call("jfsx_mctx_lz4_compress_batch", self.L.jfsx_mctx_lz4_compress_batch, n, zblks, mem)

    def lz4_decompress_batch(self, zblks, n, mem=MEM_HOST):
        self._call("jfsx_mctx_lz4_decompress_batch", self.L.jfsx_mctx_lz4_decompress_batch, n, zblks, mem)

    def zstd_decompress_batch(self, zblks, n, mem=MEM_HOST):
        self._call("jfsx_mctx_zstd_decompress_batch", self.L.jfsx_mctx_zstd_decompress_batch, n, zblks, mem)

    def zstd_compress_batch(self, zblks, n, mem=MEM_HOST):
        self._call("jfsx_mctx_zstd_compress_batch", self.L.jfsx_mctx_zstd_compress_batch, n, zblks, mem)


class Aggregator:
    """jfsx_agg: per-block calls from many threads coalesced into batches
    (SURVEY §8f-2).  Each method blocks its caller until that block is done,
    like dataEncryptor.Encrypt/Decrypt (encrypt.go:164-216) or the verify in
    cacheFile.ReadAt (disk_cache.go:1315-1327); ctypes drops the GIL for the
    wait, so Python threads submit concurrently.  Over a MultiEngine, one
    dispatcher per GPU takes groups from one shared queue."""

    def __init__(self, eng, max_blocks=0, max_bytes=0, window_us=200):
        self.eng = eng
        self.L = eng.L
        h = ctypes.c_void_p()
        if isinstance(eng, MultiEngine):
            self.ndev = eng.ndev
            eng._check(self.L.jfsx_agg_new_mctx(eng.m, max_blocks, max_bytes, window_us, ctypes.byref(h)),
                       "jfsx_agg_new_mctx")
        else:
            self.ndev = 1
            eng._check(self.L.jfsx_agg_new(eng.ctx, max_blocks, max_bytes, window_us, ctypes.byref(h)),
                       "jfsx_agg_new")
        self.h = h.value

    def dev_batches(self):
        """batches issued per device slot"""
        out = []
        for i in range(self.ndev):
            v = ctypes.c_uint64()
            self.eng._check(self.L.jfsx_agg_dev_batches(self.h, i, ctypes.byref(v)), "jfsx_agg_dev_batches")
            out.append(v.value)
        return out

    def close(self):
        if getattr(self, "h", None):
            self.L.jfsx_agg_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def seal(self, algo, blk, crc_mode=CRC_GEN, mem=MEM_HOST):
        """blk: a jfsx_blk (results are written into it); returns 0 or raises."""
        self.eng._check(self.L.jfsx_agg_seal(self.h, algo, ctypes.byref(blk), crc_mode, mem), "jfsx_agg_seal")

    def open(self, algo, blk, crc_mode=CRC_NONE, mem=MEM_HOST):
        self.eng._check(self.L.jfsx_agg_open(self.h, algo, ctypes.byref(blk), crc_mode, mem), "jfsx_agg_open")

    def crc32c(self, rng, mode=CRC_VERIFY, mem=MEM_HOST):
        self.eng._check(self.L.jfsx_agg_crc32c(self.h, ctypes.byref(rng), mode, mem), "jfsx_agg_crc32c")

    def lz4_compress(self, z, mem=MEM_HOST):
        """z: a jfsx_zblk (out_len/status are written into it)."""
        self.eng._check(self.L.jfsx_agg_lz4_compress(self.h, ctypes.byref(z), mem), "jfsx_agg_lz4_compress")

    def lz4_decompress(self, z, mem=MEM_HOST):
        self.eng._check(self.L.jfsx_agg_lz4_decompress(self.h, ctypes.byref(z), mem), "jfsx_agg_lz4_decompress")

    def zstd_decompress(self, z, mem=MEM_HOST):
        self.eng._check(self.L.jfsx_agg_zstd_decompress(self.h, ctypes.byref(z), mem), "jfsx_agg_zstd_decompress")

    def zstd_compress(self, z, mem=MEM_HOST):
        """z: a jfsx_zblk, dst_cap >= zstd_bound(src_len)."""
        self.eng._check(self.L.jfsx_agg_zstd_compress(self.h, ctypes.byref(z), mem), "jfsx_agg_zstd_compress")

    def data_encrypt(self, algo, key, nonce, wrapped, plaintext, obj_crc=False, seg_crc=False):
        """dataEncryptor.Encrypt through the aggregator (jfsx_agg_data_encrypt_ex):
        the object bytes, with its object-store CRC32C when obj_crc and
        checksum() of the plaintext when seg_crc (a tuple then)."""
        p = _u8(plaintext)
        w = _u8(wrapped)
        out = np.empty(3 + w.size + 12 + p.size + 16, np.uint8)
        olen = ctypes.c_uint64()
        crc = ctypes.c_uint32()
        segs = np.zeros(4 * max(1, -(-p.size // SEG)), np.uint8)
        self.eng._check(self.L.jfsx_agg_data_encrypt_ex(self.h, algo, _u8(key).ctypes.data, _u8(nonce).ctypes.data,
                                                        w.ctypes.data, w.size, p.ctypes.data, p.size, out.ctypes.data,
                                                        out.size, ctypes.byref(olen),
                                                        ctypes.byref(crc) if obj_crc else None,
                                                        segs.ctypes.data if seg_crc else None),
                        "jfsx_agg_data_encrypt_ex")
        res = (out.tobytes(),) + ((crc.value,) if obj_crc else ()) + ((segs.tobytes(),) if seg_crc else ())
        return res if len(res) > 1 else res[0]

    def data_decrypt(self, algo, key, obj, seg_crc=False):
        """dataEncryptor.Decrypt (after the key unwrap) through the aggregator;
        with seg_crc, (plaintext, checksum() of it)."""
        o = _u8(obj)
        out = np.empty(max(o.size, 1), np.uint8)
        n = ctypes.c_uint64()
        segs = np.zeros(4 * max(1, -(-_obj_plain_len(o) // SEG)), np.uint8)
        self.eng._check(self.L.jfsx_agg_data_decrypt_ex(self.h, algo, _u8(key).ctypes.data, o.ctypes.data, o.size,
                                                        out.ctypes.data, out.size, ctypes.byref(n), None, None,
                                                        segs.ctypes.data if seg_crc else None),
                        "jfsx_agg_data_decrypt_ex")
        pt = out[:n.value].tobytes()
        return (pt, segs.tobytes()) if seg_crc else pt

    def stats(self):
        """(calls, batches, blocks carried by those batches)"""
        v = [ctypes.c_uint64() for _ in range(3)]
        self.eng._check(self.L.jfsx_agg_stats(self.h, *[ctypes.byref(x) for x in v]), "jfsx_agg_stats")
        return tuple(x.value for x in v)
