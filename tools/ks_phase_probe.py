"""Where gcm_keysetup_k's latency goes: a probe build of libjfsx with
JFSX_KS_PHASES (scripts/build_variant.sh KSP "jfsx_gcm.hip" -DJFSX_KS_PHASES)
stamps the 100 MHz constant clock at each phase boundary of workgroup 0.
This seals n device-resident 64 KiB blocks per batch (the per-object path's
small groups), reps times, and prints the mean time of each phase in us.

usage: JFSX_LIB=juicefs_amd/_build/libjfsx_KSP.so python3 tools/ks_phase_probe.py [n] [reps]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from juicefs_amd import engine as E  # noqa: E402

MAIN = ["stage AES + CRC tables", "first task: GHASH table", "rows", "epilogue (lift, reduce)",
        "shared-segment CRCs"]
PHASES = ["stage AES tables", "key expansion", "bs masks, round-1 constants, k1", "E_K(0), E_K(J0)",
          "32 squarings H^(2^k)", "H^e (lane powers)", "basis x^i H^64", "init (len block)"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    eng = E.Engine()
    L = 65536
    src, dst = eng.alloc(n * L), eng.alloc(n * L)
    crc = eng.alloc(n * 4 * 2)
    specs = [{"key": bytes(range(i, i + 32)), "nonce": bytes(12), "src": src.ptr + i * L, "dst": dst.ptr + i * L,
              "len": L, "crc": crc.ptr + i * 8} for i in range(n)]
    blks, nb = eng.make_blocks(specs)
    f = eng.L.jfsx_debug_ks_phases
    f.argtypes = [ctypes.c_void_p]
    ts = (ctypes.c_ulonglong * 16)()
    acc = [0.0] * len(PHASES)
    mf = getattr(eng.L, "jfsx_debug_main_phases", None)
    if mf is not None:
        mf.argtypes = [ctypes.c_void_p]
    mts = (ctypes.c_ulonglong * 8)()
    macc = [0.0] * len(MAIN)
    for r in range(reps + 5):
        eng.seal_batch(E.AES256GCM, blks, nb, E.CRC_GEN, E.MEM_DEVICE)
        assert f(ts) == 0
        if r >= 5:
            for i in range(len(PHASES)):
                acc[i] += (ts[i + 1] - ts[i]) * 0.01  # 100 MHz ticks -> us
        if r >= 5 and mf is not None:
            assert mf(mts) == 0
            for i in range(len(MAIN)):
                macc[i] += (mts[i + 1] - mts[i]) * 0.01
    tot = sum(acc) / reps
    print("keysetup of %d blocks, mean over %d launches: %.1f us" % (n, reps, tot))
    for name, a in zip(PHASES, acc):
        print("  %-34s %6.2f us" % (name, a / reps))
    if mf is not None:
        print("main kernel, the workgroup of block 0's first 64 KiB task: %.1f us" % (sum(macc) / reps))
        for name, a in zip(MAIN, macc):
            print("  %-34s %6.2f us" % (name, a / reps))


if __name__ == "__main__":
    main()
