"""Diagnostic: per-section cycle shares of lz4_compress_k from a
-DJFSX_LZ4_STAMP build (JFSX_LIB=juicefs_amd/_build/libjfsx_STAMP.so).
Shares only: the stamps' fences change the kernel's timing."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from juicefs_amd import engine as E  # noqa: E402

names = ["search", "catch-up+count", "literals", "emit match", "table+hash", "next count", "next-test tail"]
nb, L = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 4 << 20
eng = E.Engine(0)
lib = E._lib
lib.jfsx_debug_lz4_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
pool = bench._text_pool(16 << 20, 7)
bound = int(E.lz4_bound(L))
src = eng.alloc(nb * L)
cmp_ = eng.alloc(nb * bound)
for b in range(nb):
    o = (b * 2654435761) % (pool.size - L)
    src.upload(pool[o:o + L], b * L)
arr, n = eng.make_zblocks((src.ptr + b * L, L, cmp_.ptr + b * bound, bound) for b in range(nb))
out = (ctypes.c_ulonglong * 8)()
eng.lz4_compress_batch(arr, n, E.MEM_DEVICE)
lib.jfsx_debug_lz4_stamps(out, 1)
eng.lz4_compress_batch(arr, n, E.MEM_DEVICE)
lib.jfsx_debug_lz4_stamps(out, 1)
tot = sum(out[k] for k in range(7))
seqs = 429000 * nb
print("total stamp cycles %.3e, per sequence (per wave) %.0f" % (tot, tot / seqs))
for k in range(7):
    print("%-16s %5.1f %%  %7.0f cycles/seq" % (names[k], 100.0 * out[k] / tot, out[k] / seqs))
eng.close()
