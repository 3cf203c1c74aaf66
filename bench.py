"""bench.py -- sealed+checksummed throughput of the MI355X block-transform engine.

Workload (BASELINE.json configs[1]): a device-resident batch of 4 MiB blocks,
AES-256-GCM Seal fused with CRC32C "full" segment checksums, per-block keys
and nonces, bit-exact to the reference's Go path (pkg/object/encrypt.go:192 +
pkg/chunk/disk_cache.go:1218-1231).  One "step" = one jfsx_seal_batch over
the whole batch (keysetup + transform + finalize + result copy-back).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--blocks B] [--mode seal|open|crc]

For N > 1 it runs one rank per GPU: either launched by torch.distributed.run
(the driver's form), or -- when WORLD_SIZE is unset -- it starts that launcher
itself as a child process before touching any GPU and exits with its code.
Blocks shard across ranks with no collective on the data path (the only
collectives are the timing barrier and the max-over-ranks reduction).  Every
rank checks its own sampled blocks against the oracle; rank 0 prints ONE JSON
line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x4A465321
BLOCK = 4 << 20
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--warmup-seconds", type=float, default=None,
                    help="host-memory modes (--mem host, agg): keep warming up until this much time has passed as "
                         "well as --warmup steps (default 8 s there, 0 elsewhere): a cold box's D2H path runs at "
                         "about 20 GB/s for its first seconds of traffic (tools/pin_probe.hip)")
    ap.add_argument("--blocks", type=int, default=16384, help="4 MiB blocks per GPU (16384 = 64 GiB)")
    ap.add_argument("--block-bytes", type=int, default=BLOCK)
    ap.add_argument("--mode", choices=["seal", "open", "crc", "decrypt", "agg", "aggcodec", "lz4", "unlz4", "zstd", "unzstd"], default="seal",
                    help="decrypt = dataEncryptor.Decrypt end to end: batched RSA-OAEP key unwrap + Open + CRC verify; "
                         "agg = one-block Seal calls from --threads threads on pinned host blocks, through the "
                         "aggregator (jfsx_agg) and, for comparison, as direct one-block batches")
    ap.add_argument("--threads", type=int, default=32, help="agg: submitting threads (reference: goroutines)")
    ap.add_argument("--codec", choices=["lz4", "unlz4", "zstd", "unzstd"], default="zstd",
                    help="aggcodec: the Compress / Decompress call of cachedStore.upload / load measured in the "
                         "reference's call shape")
    ap.add_argument("--agg-op", choices=["seal", "open", "checksum", "verify", "readat"], default="seal",
                    help="agg: the per-object call measured: Seal + CRC gen (cachedStore.upload) or Open + plaintext "
                         "CRC gen for the cache file (cachedStore.load, CS-3); heap buffers only: checksum() of a "
                         "page (jfsx_agg_crc32c), the whole-block cache-hit verify (jfsx_cache_verify, level full), "
                         "or configs[4]'s ragged ReadAt at random unaligned ranges (--level shrink|extend)")
    ap.add_argument("--buffers", choices=["pinned", "heap"], default="pinned",
                    help="agg: where the callers' blocks live -- engine-pinned memory, or ordinary pageable heap "
                         "memory as the reference's Go-heap slices (encrypt.go:183, :258; page.go:42-50), staged by "
                         "the engine's bounce pool")
    ap.add_argument("--agg-crc", choices=["none", "seg", "obj", "both"], default="seg",
                    help="agg --buffers heap seal/open: the checksums each data_encrypt_ex / data_decrypt_ex call "
                         "returns: checksum() of the plaintext (seg), the object-store CRC (obj), both, or none")
    ap.add_argument("--level", choices=["shrink", "extend"], default="shrink",
                    help="agg --agg-op readat: the cache checksum level (disk_cache.go:1265-1307)")
    ap.add_argument("--reads-per-block", type=int, default=4, help="agg --agg-op readat: random reads per image")
    ap.add_argument("--agg-window-us", type=int, default=500, help="agg: aggregation window")
    ap.add_argument("--log-clocks", action="store_true",
                    help="agg --buffers heap: sample the GPUs' DPM clock levels (sysfs, read only) over the run")
    ap.add_argument("--agg-max-mb", type=int, default=12,
                    help="agg: byte cap of one aggregated batch (several batches pipeline at once)")
    ap.add_argument("--algo", choices=["aes256gcm", "chacha20poly1305"], default="aes256gcm")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--crc", choices=["full", "none"], default="full", help="seal: CRC32C full or none (ablation)")
    ap.add_argument("--verify", type=int, default=4, help="blocks re-checked against the oracle after timing")
    ap.add_argument("--mem", choices=["device", "host"], default="device",
                    help="device: inputs resident in HBM (configs[1]); host: pinned host buffers streamed over PCIe "
                         "(configs[2], host ingest)")
    ap.add_argument("--ragged", action="store_true",
                    help="configs[4]: block lengths uniform in [64 KiB, 4 MiB] (seeded), non-multiples of 16/64/32768")
    ap.add_argument("--ragged-align", type=int, default=0,
                    help="diagnostic: round ragged lengths up to a multiple of this many bytes")
    ap.add_argument("--fixed-len", type=int, default=0,
                    help="diagnostic: every block this long, placed in --block-bytes slots")
    ap.add_argument("--packed", action="store_true",
                    help="place blocks back to back (256-B aligned) instead of one per --block-bytes slot")
    ap.add_argument("--aes", choices=["ttable", "bitslice"], default="ttable",
                    help="AES-GCM keystream kernel: T-table AES in LDS, or bitsliced AES on the VALU")
    ap.add_argument("--lz4-data", choices=["text", "random"], default="text",
                    help="lz4/unlz4 modes (SURVEY 8f-4): word text (compressible) or SplitMix64 bytes")
    ap.add_argument("--engine", choices=["process", "mctx"], default="process",
                    help="process: one process per GPU (torch.distributed ranks, the driver's form); mctx: ONE process "
                         "drives --gpus GPUs through the multi-device context (jfsx_mctx_*), the path the Go shim "
                         "ships (INTEGRATION.md)")
    ap.add_argument("--total-gib", type=float, default=0.0,
                    help="strong scaling: a fixed total of GiB per step split across the GPUs "
                         "(juicefs_amd.shard.shard_strong); each GPU loops over a resident batch of at most "
                         "--blocks blocks (device) or --host-pool-gib (host) to make up its share.  "
                         "configs[3]: --mode open --total-gib 2048")
    ap.add_argument("--host-pool-gib", type=float, default=8.0,
                    help="host mode: pinned input pool per GPU (the output pool is the same size), NUMA-local to "
                         "the GPU; a step loops over it to make up the GPU's blocks")
    ap.add_argument("--dry-run", action="store_true",
                    help="test hook: the launcher, process group, shard layout, barrier and max-over-ranks timing "
                         "with no engine (no GPU); prints the JSON line with value null")
    return ap.parse_args()


def spawn_ranks(args):
    """--gpus N > 1 without a torch.distributed.run environment: start the
    launcher as a child (one rank per GPU, rendezvous on 127.0.0.1) and return
    its exit code.  Called before anything initialises the GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dist_setup(args):
    from juicefs_amd import shard
    world, rank, local = shard.dist_env()
    return world, rank, local, shard.init()


def barrier(dist):
    from juicefs_amd import shard
    shard.barrier(dist)


def max_over_ranks(dist, x, local):
    from juicefs_amd import shard
    return shard.max_over_ranks(dist, x, local)


def ragged_len(seed, block, cap):
    """configs[4]: a length uniform in [64 KiB, cap], SplitMix64 of (seed, block)."""
    z = (seed * 0x9E3779B97F4A7C15 + block * 0xBF58476D1CE4E5B9 + 0x52616767) & (2**64 - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
    z ^= z >> 31
    lo = min(65536, cap)
    return lo + z % (cap - lo + 1)


def host_cores():
    """(threads to use, note): every core of the affinity mask, capped by the
    cgroup CPU quota when one is set (threads beyond the quota would only be
    throttled)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if quota is not None and quota < aff:
        return quota, "%d-CPU affinity mask, cgroup quota %d CPUs" % (aff, quota)
    return aff, "%d-CPU affinity mask" % aff


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


ORIG_AFFINITY = None  # the process's CPUs before any NUMA pinning (main)


def node_cpu_set(node):
    try:
        return parse_cpulist(open("/sys/devices/system/node/node%d/cpulist" % node).read())
    except (OSError, ValueError):
        return set()


def best_placement(fn, node):
    """Run a CPU baseline fn() (-> dict with "value", "cores", "sample") on
    every core the process may use, and again on the cores of NUMA node
    `node` (the GPU's socket) when that is a proper subset; returns the
    faster, with the other beside it as "other_placement".  The process's
    affinity is restored afterwards."""
    cur = os.sched_getaffinity(0)
    full = set(ORIG_AFFINITY or cur)
    runs = []
    places = [("all %d CPUs of the process" % len(full), full)]
    nc = node_cpu_set(node) & full if node is not None and node >= 0 else set()
    if nc and nc != full:
        places.append(("pinned to NUMA node %d (%d CPUs, the GPU's socket)" % (node, len(nc)), nc))
    try:
        for name, cpus in places:
            os.sched_setaffinity(0, cpus)
            r = fn()
            r["placement"] = name
            runs.append(r)
    finally:
        os.sched_setaffinity(0, cur)
    runs.sort(key=lambda r: -r["value"])
    best = dict(runs[0])
    if len(runs) > 1:
        best["other_placement"] = {k: runs[1][k] for k in ("value", "cores", "placement")}
    best["core_s_per_GB"] = round(best["cores"] / best["value"], 4) if best["value"] else None
    return best


def cpu_baseline(args, mode="seal", lens=None, node=None):
    """The reference's per-block CPU work, one worker per core, timed on this
    host over a bounded sample of the same workload (about --cpu-seconds):
      seal     checksum() + aead.Seal            (encrypt.go:192, disk_cache.go:1218-1231)
      open     aead.Open + the ReadAt CRC verify (encrypt.go:215, disk_cache.go:1315-1327)
      crc      the ReadAt CRC verify alone       (a cache hit)
      encrypt  dataEncryptor.Encrypt: header + Seal into the object buffer at
               offset 271, + checksum() of the plaintext (encrypt.go:164-194)
      objdecrypt  dataEncryptor.Decrypt: header parse + Open from offset 271,
               + checksum() of the plaintext for the cache file (encrypt.go:196-216)
    The AEAD runs through OpenSSL EVP (AES-NI/VAES + VPCLMULQDQ stitched GCM,
    SIMD ChaCha20-Poly1305: the class of Go's assembly), the
    CRC32C as 3-stream SSE4.2 like Go's castagnoliSSE42Triple.  lens: the
    bench's own ragged lengths (configs[4]); else 4 MiB blocks.  Run on every
    core and on the GPU's NUMA node (node given): the faster is the baseline,
    the other is reported beside it (best_placement)."""
    return best_placement(lambda: _cpu_baseline_once(args, mode, lens), node)


def _cpu_baseline_once(args, mode, lens):
    from oracle import oracle as orc
    threads, note = host_cores()
    algo = orc.AES256GCM if args.algo == "aes256gcm" else orc.CHACHA20P1305
    bmode = {"seal": orc.BASE_SEAL, "open": orc.BASE_OPEN, "crc": orc.BASE_CRC, "encrypt": orc.BASE_ENCRYPT,
             "objdecrypt": orc.BASE_DECRYPT}[mode]
    sample = [int(x) for x in lens[:256]] if lens is not None else None
    nblk = len(sample) if sample else 256  # 1 GiB of 4 MiB blocks: BASELINE.json configs[0]
    nbytes = sum(sample) if sample else nblk * BLOCK
    impl = "OpenSSL EVP"
    secs, _ = orc.bench_baseline(algo, bmode, threads, nblk, BLOCK, SEED, sample)
    if secs == -1.0 and mode == "seal" and not sample:
        impl = "oracle AES-NI/PCLMUL port"
        secs, _ = orc.bench_seal_crc(algo, threads, nblk, BLOCK, SEED)
    if secs < 0:
        raise SystemExit("bench: CPU baseline failed (%s, rc %s)" % (mode, secs))
    reps = max(1, min(64, int(args.cpu_seconds / max(secs, 1e-3))))
    total_s = 0.0
    for r in range(reps):
        if impl == "OpenSSL EVP":
            s_, _ = orc.bench_baseline(algo, bmode, threads, nblk, BLOCK, SEED + r, sample)
        else:
            s_, _ = orc.bench_seal_crc(algo, threads, nblk, BLOCK, SEED + r)
        if s_ < 0:
            raise SystemExit("bench: CPU baseline failed (%s, rc %s)" % (mode, s_))
        total_s += s_
    what = {"seal": "%s seal (%s) + CRC32C full (3-stream SSE4.2)" % (args.algo, impl),
            "open": "%s open (%s, tag checked) + CRC32C verify against the stored CRCs" % (args.algo, impl),
            "crc": "CRC32C verify against the stored CRCs (3-stream SSE4.2)",
            "encrypt": "dataEncryptor.Encrypt: object header (256-B wrapped key) + %s seal (%s) into the object "
                       "buffer at offset 271 + checksum() of the plaintext (3-stream SSE4.2); the output buffer is "
                       "reused (Go's make([]byte) and its zeroing are not charged)" % (args.algo, impl),
            "objdecrypt": "dataEncryptor.Decrypt: header parse + %s open (%s, tag checked) from offset 271 + "
                          "checksum() of the plaintext (3-stream SSE4.2)" % (args.algo, impl)}[mode]
    if sample and len(set(sample)) == 1:
        blocks = "%d blocks of %d bytes (%.3f GiB)" % (nblk, sample[0], nbytes / 2**30)
    elif sample:
        blocks = "%d ragged blocks (the bench's own lengths, %.3f GiB)" % (nblk, nbytes / 2**30)
    else:
        blocks = "1 GiB (256 x 4 MiB blocks)"
    return {"value": round(reps * nbytes / total_s / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d x %s %s, %d threads (%s), %s" % (reps, blocks, what, threads, note, cpu_model())}


def cpu_readat_baseline(args, lens, reads, level, node=None):
    """cacheFile.ReadAt (disk_cache.go:1255-1329) on the host cores: the copy
    out of the cache file and the level's CRC verify (3-stream SSE4.2), one
    thread per core, over the bench's own images and (block, off, size) reads,
    repeated to about --cpu-seconds; GB/s of bytes returned."""
    from oracle import oracle as orc
    lv = {"full": 1, "shrink": 2, "extend": 3}[level]

    def once():
        threads, note = host_cores()
        secs, nbytes = orc.bench_readat(threads, lv, lens, SEED, reads, 1)
        if secs < 0:
            raise SystemExit("bench: ReadAt CPU baseline failed (rc %s)" % secs)
        reps = max(1, min(64, int(args.cpu_seconds / max(secs, 1e-3))))
        secs, nbytes = orc.bench_readat(threads, lv, lens, SEED, reads, reps)
        if secs < 0:
            raise SystemExit("bench: ReadAt CPU baseline failed (rc %s)" % secs)
        return {"value": round(nbytes / secs / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
                "sample": "%d x %d ReadAt calls at level %s over %d cache-file images (%.3f GiB of data; the bench's "
                          "own images and ranges), copy + CRC32C verify (3-stream SSE4.2), %d threads (%s), %s" % (
                              reps, len(reads), level, len(lens), sum(lens) / 2**30, threads, note, cpu_model())}
    return best_placement(once, node)


def shard_plan(args, nshard, s):
    """The blocks of shard s (a rank, or one GPU of --engine mctx): (base
    global block index, blocks per step, resident blocks, blocks per loop).
    Weak scaling: --blocks per shard, one call per step.  Strong scaling
    (--total-gib): the fixed total is split by shard.shard_strong, and the
    shard loops over a resident batch (at most --blocks on the device, or the
    --host-pool-gib pinned pool in host mode) until its share is done."""
    from juicefs_amd import shard
    L = args.block_bytes
    cap = args.blocks if args.mem == "device" else max(1, int(args.host_pool_gib * 2**30) // L)
    if args.total_gib:
        total = max(nshard, int(round(args.total_gib * 2**30 / L)))
        r = shard.shard_strong(total, s, nshard)
        base, count = r.start, len(r)
    else:
        base, count = s * args.blocks, args.blocks
    resident = max(1, min(cap, count))
    loops = [resident] * (count // resident) + ([count % resident] if count % resident else [])
    return base, count, resident, loops


def dry_run(args, world, rank, local, dist):
    """No engine: exercises the rank launch, the shard layout (weak or strong),
    the barrier and the max-over-ranks timing the real bench uses
    (tests/test_dist_gloo.py)."""
    from juicefs_amd import shard
    base, count, resident, loops = shard_plan(args, world, rank)
    barrier(dist)
    t0 = time.perf_counter()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0 + 0.001 * rank, local)
    first = max_over_ranks(dist, float(base), local)
    total = shard.sum_over_ranks(dist, count, local)
    lo = -max_over_ranks(dist, -float(base), local)
    hi = max_over_ranks(dist, float(base + count), local)
    per_max = max_over_ranks(dist, float(count), local)
    # host mode pins the resident pool twice (in, out) plus its CRC arrays
    L = args.block_bytes
    pinned = resident * (2 * L + 4 * -(-L // (32 << 10))) if args.mem == "host" else 0
    pinned_max = max_over_ranks(dist, float(pinned), local)
    # the CPU leg runs without an engine too: rank 0, after the timed region
    cpu = cpu_baseline(args, "seal") if rank == 0 and not args.no_cpu else None
    if rank == 0:
        print(json.dumps({"metric": "dry run (no engine)", "value": None, "unit": "GB/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3),
                          "dry_run": True, "last_rank_first_block": int(first), "scaling": scaling(args),
                          "blocks_total": int(total), "block_range": [int(lo), int(hi)],
                          "per_gpu_blocks_max": int(per_max), "resident_blocks": resident, "loops_per_step": len(loops),
                          "pinned_bytes_per_rank_max": int(pinned_max), "cpu_baseline": cpu,
                          "config": {"blocks_per_gpu": args.blocks, "total_gib": args.total_gib or None,
                                     "parallelism": "block-sharded x%d, no collective" % world}}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def scaling(args):
    return "strong" if args.total_gib else "weak"


def main():
    global ORIG_AFFINITY
    ORIG_AFFINITY = os.sched_getaffinity(0)
    args = parse()
    if args.engine == "mctx":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("bench: --engine mctx is one process over --gpus GPUs; run it without the launcher")
        if args.mode not in ("seal", "open", "decrypt", "crc"):
            raise SystemExit("bench: --engine mctx measures the seal / open / decrypt / crc modes")
    elif args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    if args.total_gib and args.ragged:
        raise SystemExit("bench: --total-gib splits 4 MiB blocks; ragged batches are weak-scaled")
    world, rank, local, dist = dist_setup(args)
    if args.gpus > 1 and args.engine == "process" and world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.dry_run:
        return dry_run(args, world, rank, local, dist)
    from juicefs_amd import engine as E

    if args.mem == "host":
        return host_ingest(args, world, rank, local, dist)
    if args.mode in ("seal", "open", "decrypt", "crc"):
        return resident_bench(args, world, rank, local, dist)
    eng = E.Engine(local, E.CTX_BITSLICE if args.aes == "bitslice" else 0)
    if args.mode == "agg":
        if args.buffers == "heap" or args.agg_op in ("checksum", "verify", "readat"):
            return agg_heap_bench(args, world, rank, local, dist, eng)
        return agg_bench(args, world, rank, local, dist, eng)
    if args.mode == "aggcodec":
        return aggcodec_bench(args, world, rank, local, dist, eng)
    if args.mode in ("lz4", "unlz4"):
        return lz4_bench(args, world, rank, local, dist, eng)
    if args.mode == "unzstd":
        return zstd_bench(args, world, rank, local, dist, eng)
    return zstdc_bench(args, world, rank, local, dist, eng)


def open_engines(args, local):
    """(MultiEngine or None, [Engine per shard]): one context for this rank's
    GPU, or every context of a multi-device context over --gpus GPUs."""
    from juicefs_amd import engine as E
    flags = E.CTX_BITSLICE if args.aes == "bitslice" else 0
    if args.engine == "mctx":
        m = E.MultiEngine((1 << args.gpus) - 1, flags)
        return m, [m.member(k) for k in range(m.ndev)]
    return None, [E.Engine(local, flags)]


class Shard:
    """The resident blocks one GPU holds: buffers, lengths, descriptors' place
    in the combined array (off)."""


def make_shard(args, E, eng, nshard, s):
    sh = Shard()
    sh.eng, sh.s = eng, s
    sh.base, sh.count, sh.nb, sh.loops = shard_plan(args, nshard, s)
    nb, L = sh.nb, args.block_bytes
    sh.nseg = -(-L // E.SEG)
    # block b occupies slot [b*L, b*L + lens[b]); ragged lengths are a seeded
    # draw per global block index, so every shard and rerun sees the same batch
    lens = [ragged_len(SEED, sh.base + b, L) if args.ragged else (args.fixed_len or L) for b in range(nb)]
    if args.ragged and args.ragged_align:
        lens = [min(L, -(-x // args.ragged_align) * args.ragged_align) for x in lens]
    sh.lens = lens
    sh.src = eng.alloc(nb * L)
    sh.dst = eng.alloc(nb * L) if args.mode != "crc" else None
    sh.crc = eng.alloc(nb * 4 * sh.nseg)
    if args.packed:
        offs, o = [], 0
        for x in lens:
            offs.append(o)
            o += -(-x // 256) * 256
        for b in range(nb):
            eng.gen_synthetic_batch(sh.src, L, [lens[b]], SEED, sh.base + b, offset=offs[b])
    else:
        offs = [b * L for b in range(nb)]
        eng.gen_synthetic_batch(sh.src, L, lens, SEED, sh.base)  # one launch for the whole batch
    sh.offs = offs
    if args.mode == "crc":
        sh.specs = [(sh.src.ptr + offs[b], lens[b], sh.crc.ptr + 4 * sh.nseg * b) for b in range(nb)]
    else:
        sh.specs = []
        for b in range(nb):
            key, nonce = E.gen_key(SEED, sh.base + b)
            sh.specs.append({"key": key, "nonce": nonce, "src": sh.src.ptr + offs[b], "dst": sh.dst.ptr + offs[b],
                             "len": lens[b], "crc": sh.crc.ptr + 4 * sh.nseg * b})
    return sh


def make_ranges(specs):
    import ctypes
    from juicefs_amd import engine as E
    arr = (E.jfsx_range * max(len(specs), 1))()
    for i, (d, n, c) in enumerate(specs):
        arr[i].data, arr[i].len, arr[i].crc = d, n, c
    return arr


def loop_arrays(A, shards):
    """The calls of one step: loop j runs, on every shard, the first
    sh.loops[j] of its resident blocks.  (array, n, [(shard, offset, count)])
    per loop; a loop that covers every shard's whole batch uses the combined
    array itself, a shorter last loop a compacted copy of the prefixes."""
    import ctypes
    J = max(len(sh.loops) for sh in shards)
    out = []
    for j in range(J):
        cnts = [sh.loops[j] if j < len(sh.loops) else 0 for sh in shards]
        if all(c == sh.nb for c, sh in zip(cnts, shards)):
            out.append((A, sum(cnts), [(sh, sh.off, sh.nb) for sh in shards]))
        elif len(shards) == 1:
            out.append((A, cnts[0], [(shards[0], 0, cnts[0])]))
        else:
            T = type(A[0])
            n = sum(cnts)
            B = (T * max(n, 1))()
            o, parts = 0, []
            for c, sh in zip(cnts, shards):
                if c:
                    ctypes.memmove(ctypes.addressof(B[o]), ctypes.addressof(A[sh.off]), c * ctypes.sizeof(T))
                    parts.append((sh, o, c))
                o += c
            out.append((B, n, parts))
    return out


def resident_bench(args, world, rank, local, dist):
    """BASELINE configs[1] (seal), configs[3] (open / decrypt + CRC verify)
    and configs[4] (--ragged), and the cache-hit verify (crc): blocks resident
    in HBM, one call per loop of every shard's resident batch.  --engine
    process: this rank's GPU; --engine mctx: one jfsx_mctx_* call over every
    GPU's blocks (each block runs on the GPU that owns it)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    from juicefs_amd import engine as E
    from juicefs_amd import shard as S
    m, engs = open_engines(args, local)
    nshard = len(engs) if m else world
    shards = [make_shard(args, E, e, nshard, k if m else rank) for k, e in enumerate(engs)]
    off = 0
    for sh in shards:
        sh.off = off
        off += sh.nb
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    front = m if m else engs[0]
    specs = [x for sh in shards for x in sh.specs]
    mode = args.mode
    if mode == "crc":
        R = make_ranges(specs)
        front.crc32c_segments(R, len(specs), E.CRC_GEN, E.MEM_DEVICE)  # the cache files' stored CRCs
        loops = loop_arrays(R, shards)

        def step():
            for arr, n, _ in loops:
                front.crc32c_segments(arr, n, E.CRC_VERIFY, E.MEM_DEVICE)
        per_blk = [[lb + 4 * -(-lb // E.SEG) for lb in sh.lens] for sh in shards]
    else:
        A, _ = E.Engine.make_blocks(specs)
        if mode == "seal":
            loops = loop_arrays(A, shards)
            crc_mode = E.CRC_GEN if args.crc == "full" else E.CRC_NONE

            def step():
                for arr, n, _ in loops:
                    front.seal_batch(algo, arr, n, crc_mode, E.MEM_DEVICE)
        else:
            # Open + CRC verify (BASELINE configs[3]): seal an image first
            front.seal_batch(algo, A, len(specs), E.CRC_GEN, E.MEM_DEVICE)
            O, _ = E.Engine.make_blocks([dict(sp, src=sp["dst"], dst=sp["src"], tag=bytes(A[i].tag))
                                         for i, sp in enumerate(specs)])
            loops = loop_arrays(O, shards)
            if mode == "open":
                def step():
                    for arr, n, _ in loops:
                        front.open_batch(algo, arr, n, E.CRC_VERIFY, E.MEM_DEVICE)
            else:
                # Decrypt end to end: every object's key arrives RSA-OAEP
                # wrapped (encrypt.go:196-216); each loop unwraps its blocks'
                # keys on their GPUs straight into the descriptors, then opens
                import numpy as np
                from juicefs_amd import encrypt as enc
                rsae = enc.NewRSAEncryptor(enc.GenerateRsaKey(2048))
                comps = enc.rsa_crt_components(rsae.privKey)
                for sh in shards:
                    sh.dkey = sh.eng.rsa_key(*comps)
                    sh.wrapped = np.frombuffer(b"".join(rsae.Encrypt(bytes(sp["key"])) for sp in sh.specs), np.uint8)
                    sh.wlen = np.full(sh.nb, 256, np.uint32)
                    sh.mlen = np.zeros(sh.nb, np.int32)
                for arr, n, _ in loops:
                    for i in range(n):
                        ctypes.memset(ctypes.addressof(arr[i]) + E.jfsx_blk.key.offset, 0, 32)
                pool = ThreadPoolExecutor(len(shards))

                def unwrap(part, arr):
                    sh, o, c = part
                    sh.eng._check(sh.eng.L.jfsx_rsa_oaep_decrypt_batch(
                        sh.eng.ctx, sh.dkey, c, sh.wrapped.ctypes.data, 256, sh.wlen.ctypes.data,
                        ctypes.addressof(arr[o]) + E.jfsx_blk.key.offset, ctypes.sizeof(E.jfsx_blk),
                        sh.mlen.ctypes.data), "unwrap")

                def step():
                    for arr, n, parts in loops:
                        if len(parts) == 1:
                            unwrap(parts[0], arr)
                        else:
                            list(pool.map(lambda p: unwrap(p, arr), parts))
                        front.open_batch(algo, arr, n, E.CRC_VERIFY, E.MEM_DEVICE)
        per_blk = [[2 * lb + 16 + 4 * -(-lb // E.SEG) + 44 for lb in sh.lens] for sh in shards]
    # algorithmic bytes and plaintext bytes one step moves on each shard
    step_algo = [sum(sum(pb[:c]) for c in sh.loops) for pb, sh in zip(per_blk, shards)]
    step_plain = [sum(sum(sh.lens[:c]) for c in sh.loops) for sh in shards]

    for _ in range(args.warmup):
        step()
    for e in engs:
        e.sync()
        e.kernel_time(reset=True)
        e.set_timing(True)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    for e in engs:
        e.sync()
    barrier(dist)
    t1 = time.perf_counter()
    for e in engs:
        e.set_timing(False)
    el = max_over_ranks(dist, t1 - t0, local)
    ktimes = [e.kernel_time(reset=True) for e in engs]

    # checker only, after the timed region: every block against the oracle
    full, rsa = None, None
    if args.verify:
        full = check_resident(args, E, shards, A if mode != "crc" else None, O if mode in ("open", "decrypt") else None,
                              R if mode == "crc" else None, loops, algo)
    if mode == "decrypt":
        rsa = rsa_line(shards[0], rsae)
        for sh in shards:
            sh.eng.rsa_key_free(sh.dkey)

    total_plain = S.sum_over_ranks(dist, sum(step_plain), local) * args.steps
    value = total_plain / el / 1e9
    # per GPU: its algorithmic bytes over its own summed main-kernel time
    ach = [step_algo[k] * args.steps / (ms / 1e3) / 1e9 for k, (ms, n) in enumerate(ktimes) if n]
    achieved = sum(ach) / len(ach) if ach else None
    k_avg_ms = sum(ms / max(n, 1) for ms, n in ktimes) / len(ktimes)
    launches = sum(n for _, n in ktimes)
    cpu = None
    if rank == 0 and not args.no_cpu:
        # rank 0 only, after the timed region (at N > 1 the other ranks have
        # finished their GPU work by then)
        cpu = cpu_baseline(args, "open" if mode in ("open", "decrypt") else mode,
                           shards[0].lens if args.ragged else None, node=engs[0].numa_node())
        if mode == "decrypt" and rsa:
            # each object also pays one RSA-OAEP private-key unwrap on the host
            # (encrypt.go:207-210): per thread, block time + unwrap time
            def with_unwrap(gbs, cores):
                per_block = cores * BLOCK / (gbs * 1e9)
                return round(cores * BLOCK / (per_block + rsa["host_us_per_unwrap_1thread"] * 1e-6) / 1e9, 3)
            cpu["value"] = with_unwrap(cpu["value"], cpu["cores"])
            if cpu.get("other_placement"):  # the same unwrap cost on the other placement
                op_ = cpu["other_placement"]
                op_["value"] = with_unwrap(op_["value"], op_["cores"])
            if cpu.get("core_s_per_GB"):
                cpu["core_s_per_GB"] = round(cpu["cores"] / cpu["value"], 4)
            cpu["sample"] += "; plus one libcrypto RSA-OAEP unwrap per block (%.1f us, measured on 1 thread)" % (
                rsa["host_us_per_unwrap_1thread"])
    resident_plain = sum(shards[0].lens)
    traffic, traffic_src, binding = pmc_traffic(args, resident_plain)
    ngpu = len(engs) if m else world
    if rank == 0:
        what = {"seal": "sealed+checksummed GB/s, %s", "open": "opened+verified GB/s, %s",
                "decrypt": "decrypted (RSA unwrap + open + verify) GB/s, %s", "crc": "CRC32C-verified GB/s, %s"}[mode]
        blocks_txt = "ragged 64 KiB-4 MiB blocks" if args.ragged else "4 MiB blocks"
        sh0 = shards[0]
        if args.total_gib:
            workload = ("%s GiB per step split across %d GPUs (%s GiB each), %s %s + CRC32C %s; each GPU loops %d x "
                        "over a resident batch of %d blocks" % (
                            args.total_gib, ngpu, round(sh0.count * args.block_bytes / 2**30, 3), args.algo, mode,
                            "full" if mode == "seal" else "verify", len(sh0.loops), sh0.nb))
        else:
            workload = "%s GiB device-resident batch of %s blocks per GPU, %s %s + CRC32C %s" % (
                round(resident_plain / 2**30, 3), "ragged 64 KiB-4 MiB" if args.ragged else "4 MiB", args.algo, mode,
                "full" if mode == "seal" else "verify")
        line = {
            "metric": what % blocks_txt, "value": round(value, 2), "unit": "GB/s", "n_gpus": ngpu,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": scaling(args), "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (SplitMix64 blocks, per-block SplitMix64 keys/nonces), device-resident",
            "config": {"workload": workload, "blocks_per_gpu": sh0.count, "resident_blocks_per_gpu": sh0.nb,
                       "block_bytes": "ragged" if args.ragged else args.block_bytes, "algo": args.algo,
                       "mode": mode, "aes_kernel": args.aes if args.algo == "aes256gcm" and mode != "crc" else None,
                       "engine": "jfsx_mctx (one process, %d GPUs)" % ngpu if m else "one process per GPU",
                       "total_gib": args.total_gib or None,
                       "parallelism": "block-sharded x%d, no collective" % ngpu},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": ("crc_segments_k" if mode == "crc" else
                                    ("gcm_main_k" if args.algo == "aes256gcm" else "cp_main_k")),
                         "kernel_avg_ms": round(k_avg_ms, 3), "kernel_launches": launches,
                         "achieved_basis": "per GPU: algorithmic bytes of its launches / its summed main-kernel "
                                           "time (HIP events on the context's stream); mean over GPUs",
                         "algorithmic_bytes_per_launch": sum(per_blk[0]),
                         "plain_bytes_per_launch": resident_plain, "binding": binding},
            "cpu_baseline": cpu,
            "verified_blocks": full["blocks"] if full else 0,
            "full_check": full,
            **({"rsa_unwrap": rsa} if rsa else {}),
        }
        if m and len(ach) > 1:
            line["roofline"]["achieved_per_gpu"] = [round(a, 1) for a in ach]
        print(json.dumps(line), flush=True)
    for sh in shards:
        for b in (sh.src, sh.dst, sh.crc):
            if b is not None:
                b.free()
    if m:
        m.close()
    else:
        engs[0].close()
    if dist is not None:
        dist.destroy_process_group()


def rsa_line(sh, rsae):
    """The unwrap alone (one GPU batch of the shard's keys) beside the
    reference's host path (libcrypto RSA-OAEP, one thread) on a bounded
    sample."""
    t = time.perf_counter()
    sh.eng._check(sh.eng.L.jfsx_rsa_oaep_decrypt_batch(sh.eng.ctx, sh.dkey, sh.nb, sh.wrapped.ctypes.data, 256,
                                                       sh.wlen.ctypes.data, None, 0, sh.mlen.ctypes.data), "unwrap")
    gpu_s = time.perf_counter() - t
    sample = [bytes(sh.wrapped[256 * i:256 * i + 256]) for i in range(min(sh.nb, 200))]
    t = time.perf_counter()
    for w in sample:
        rsae.Decrypt(w)
    host_s = (time.perf_counter() - t) / len(sample)
    return {"unwraps": sh.nb, "gpu_ms_per_batch": round(gpu_s * 1e3, 3), "gpu_unwraps_per_s": round(sh.nb / gpu_s),
            "host_us_per_unwrap_1thread": round(host_s * 1e6, 1),
            "host_sample": "%d libcrypto RSA-OAEP decrypts, 1 thread" % len(sample)}


def check_resident(args, E, all_shards, A, O, R, loops, algo):
    """Every block of every shard against the oracle (host cores), after the
    timed region; exits non-zero on a difference.
      seal   the timed call's tags and CRC arrays, all blocks; ciphertext of a
             few blocks per shard
      open / decrypt
             setup: the sealed image's tags and CRC arrays, all blocks;
             timed: every block's Open status OK (tag and stored CRCs
             verified, keys unwrapped for decrypt), a few plaintexts per
             shard equal to the oracle's, and two negative controls -- a
             flipped tag fails (ETAG, output zeroed) and a corrupted stored
             CRC fails at its segment (ECRC)
      crc    setup: the GEN arrays, all blocks; timed: every VERIFY status
             OK and a corrupted stored CRC caught at its segment"""
    import ctypes
    from oracle import oracle as orc
    mode = args.mode
    out = {"blocks": 0}
    tags, crcs = [], []
    shards = all_shards
    if mode == "seal" and args.crc != "full":
        shards = []  # CRC ablation: no CRC arrays to compare; the ciphertext samples below
    for sh in shards:
        got = sh.crc.download(sh.nb * 4 * sh.nseg).reshape(sh.nb, 4 * sh.nseg)
        blks = [A[sh.off + i] for i in range(sh.nb)] if A is not None else None
        f = full_check(args, E, blks, got, sh.lens, sh.base)
        out["blocks"] += f["blocks"]
        tags.append(f.get("tags_sha256"))
        crcs.append(f["crc_arrays_sha256"])
        out["oracle_s"] = round(out.get("oracle_s", 0) + f["oracle_s"], 2)
        out["oracle_threads"] = f["oracle_threads"]
    out["crc_arrays_sha256"] = crcs[0] if len(crcs) == 1 else crcs
    if A is not None:
        out["tags_sha256"] = tags[0] if len(tags) == 1 else tags
    n = out["blocks"]
    if mode == "seal":
        samples = 0
        for sh in all_shards:
            for b in range(0, sh.nb, max(1, sh.nb // args.verify))[:args.verify]:
                p = orc.gen_block(SEED, sh.base + b, sh.lens[b])
                key, nonce = orc.gen_key(SEED, sh.base + b)
                c, tag = orc.seal(orc.AES256GCM if algo == E.AES256GCM else orc.CHACHA20P1305, key, nonce, p,
                                  fast=algo == E.AES256GCM)
                if bytes(A[sh.off + b].tag) != tag or sh.dst.download(sh.lens[b], offset=sh.offs[b]).tobytes() != c:
                    raise SystemExit("bench: block %d of GPU %d differs from the oracle" % (b, sh.s))
                samples += 1
        out["ciphertext_samples"] = samples
        if not shards:
            out["blocks"] = samples
            out["what"] = "timed Seal (CRC none): %d tags and ciphertexts equal to the oracle's" % samples
        else:
            out["what"] = ("timed Seal: tags and CRC arrays of all %d blocks, and %d ciphertexts, equal to the "
                           "oracle's" % (n, samples))
        return out
    # the timed calls' own results: the last loop that ran each block
    st_bad = 0
    for arr, cnt, _ in loops:
        for i in range(cnt):
            st_bad += arr[i].status != E.OK
    if mode == "decrypt":
        for sh in shards:
            st_bad += int((sh.mlen[:max(sh.loops)] != 32).sum())
        for arr, cnt, parts in loops:
            for s_, o, c in parts:
                st_bad += sum(bytes(arr[o + i].key) != bytes(s_.specs[i]["key"]) for i in range(c))
    if st_bad:
        raise SystemExit("bench: %d timed %s results failed" % (st_bad, mode))
    sh = shards[0]
    scratch = sh.eng.alloc(max(sh.lens[0], 16) + 4 * sh.nseg)
    bad_crc = bytearray(sh.crc.download(4 * sh.nseg).tobytes())
    seg = min(3, len(bad_crc) // 4 - 1)
    bad_crc[4 * seg] ^= 0x40
    scratch.upload(bytes(bad_crc), max(sh.lens[0], 16))
    if mode == "crc":
        one = make_ranges([(sh.src.ptr + sh.offs[0], sh.lens[0], scratch.ptr + max(sh.lens[0], 16))])
        sh.eng.crc32c_segments(one, 1, E.CRC_VERIFY, E.MEM_DEVICE)
        if one[0].status != E.ECRC or one[0].bad_seg != seg:
            raise SystemExit("bench: a corrupted stored CRC was not caught (%d, %d)" % (one[0].status, one[0].bad_seg))
        out["what"] = ("setup: CRC arrays of all %d blocks equal to the oracle's; timed VERIFY: all %d statuses OK, "
                       "and a corrupted stored CRC caught at segment %d (ECRC)" % (n, n, seg))
        scratch.free()
        return out
    # plaintext of a few blocks per shard: Open wrote it back over the source
    samples = 0
    for s in shards:
        for b in range(0, s.nb, max(1, s.nb // args.verify))[:args.verify]:
            if s.src.download(s.lens[b], offset=s.offs[b]).tobytes() != orc.gen_block(SEED, s.base + b, s.lens[b]).tobytes():
                raise SystemExit("bench: opened block %d of GPU %d differs from the oracle" % (b, s.s))
            samples += 1
    # negative controls on GPU 0's block 0 (output to scratch)
    key, nonce = E.gen_key(SEED, sh.base)
    tag = bytes(A[sh.off].tag)
    base = {"key": key, "nonce": nonce, "src": sh.dst.ptr + sh.offs[0], "dst": scratch.ptr, "len": sh.lens[0]}
    one, _ = E.Engine.make_blocks([dict(base, tag=bytes([tag[0] ^ 1]) + tag[1:], crc=sh.crc.ptr)])
    sh.eng.open_batch(algo, one, 1, E.CRC_VERIFY, E.MEM_DEVICE)
    zeroed = not scratch.download(sh.lens[0]).any()
    one2, _ = E.Engine.make_blocks([dict(base, tag=tag, crc=scratch.ptr + max(sh.lens[0], 16))])
    sh.eng.open_batch(algo, one2, 1, E.CRC_VERIFY, E.MEM_DEVICE)
    if one[0].status != E.ETAG or not zeroed or one2[0].status != E.ECRC or one2[0].crc_bad_seg != seg:
        raise SystemExit("bench: negative controls failed (%d %s %d %d)" % (one[0].status, zeroed, one2[0].status,
                                                                           one2[0].crc_bad_seg))
    scratch.free()
    out["plaintext_samples"] = samples
    out["what"] = ("setup (the sealed image): tags and CRC arrays of all %d blocks equal to the oracle's; timed %s: "
                   "all %d blocks tag- and CRC-verified (status OK%s), %d plaintexts equal to the oracle's, a flipped "
                   "tag fails (ETAG, output zeroed) and a corrupted stored CRC fails at segment %d (ECRC)" % (
                       n, "Decrypt" if mode == "decrypt" else "Open", n,
                       ", every key unwrapped to the data key" if mode == "decrypt" else "", samples, seg))
    return out


def full_check(args, E, blks, got, lens, base):
    """Every block of the batch against the oracle (checker only, after the
    timed region): the tags of the sealed image (blks: the seal descriptors,
    None for a CRC-only batch) and every block's checksum() array as the GPU
    wrote it, byte for byte, against the oracle's own AEAD and CRC over the
    same synthetic blocks on the host cores.  Exits non-zero on a difference;
    returns what was compared, with a SHA-256 of each array."""
    import hashlib
    import numpy as np
    from oracle import oracle as orc
    threads, _ = host_cores()
    world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    threads = max(1, threads // max(world, 1))  # the ranks of one node share its cores
    nb, stride = got.shape
    algo = orc.AES256GCM if args.algo == "aes256gcm" else orc.CHACHA20P1305
    etags, ecrcs, secs = orc.expect_batch(algo, threads, lens, SEED, base, stride)
    cl = np.array([4 * max(1, -(-int(x) // E.SEG)) for x in lens])
    valid = np.arange(stride)[None, :] < cl[:, None]
    bad_crc = np.nonzero(((got != ecrcs) & valid).any(axis=1))[0]
    if bad_crc.size:
        raise SystemExit("bench: block %d: CRC array differs from the oracle (%d blocks)" % (bad_crc[0], bad_crc.size))
    out = {"blocks": nb, "crc_arrays_sha256": hashlib.sha256(np.where(valid, got, 0).tobytes()).hexdigest(),
           "oracle_s": round(secs, 2), "oracle_threads": threads}
    if blks is not None:
        gt = np.frombuffer(b"".join(bytes(blks[i].tag) for i in range(nb)), np.uint8).reshape(nb, 16)
        bad = np.nonzero((gt != etags).any(axis=1))[0]
        if bad.size:
            raise SystemExit("bench: block %d: tag differs from the oracle (%d blocks)" % (bad[0], bad.size))
        out["tags_sha256"] = hashlib.sha256(gt.tobytes()).hexdigest()
    out["what"] = ("%s of all %d blocks equal to the oracle's" %
                   ("tags and CRC arrays" if blks is not None else "CRC arrays", nb))
    return out


PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
# labelled PMC summaries (scripts/pmc_r3.py), newest first; the round-2 file
# (FETCH / WRITE only, keyed by kernel) is the last resort for traffic
PMC_FILES = ("r6/pmc_r6.json", "r5/pmc_r5.json", "r4/pmc_r4.json", "r3/pmc_r3.json")
PMC_R2 = "r2/pmc_traffic.json"
R2_KEYS = {"seal_gcm": "gcm_ttable", "open_gcm": "gcm_ttable", "seal_gcm_bitslice": "gcm_bitslice",
           "seal_chacha": "chacha", "open_chacha": "chacha", "crc_verify": "crc_verify",
           "seal_gcm_ragged": "gcm_ttable", "open_gcm_ragged": "gcm_ttable", "ingest_gcm": "gcm_ttable",
           "seal_chacha_ragged": "chacha", "open_chacha_ragged": "chacha"}


def pmc_variant(args):
    """The key of this bench line in the PMC summaries."""
    if args.mode == "crc":
        return "crc_verify"
    if args.mode in ("lz4", "unlz4", "zstd", "unzstd"):
        return "%s_%s" % (args.mode, args.lz4_data)
    if args.mode not in ("seal", "open", "decrypt"):
        return None
    algo = "gcm" if args.algo == "aes256gcm" else "chacha"
    if args.mem == "host":
        return "ingest_" + algo
    v = "%s_%s" % ("seal" if args.mode == "seal" else "open", algo)
    if algo == "gcm" and args.aes == "bitslice":
        v += "_bitslice"
    return v + ("_ragged" if args.ragged else "")


CODEC_TRAFFIC_NOTE = ("memory-side L2 requests (2 x FETCH_SIZE + WRITE_SIZE): they include Infinity-Cache hits "
                      "on the per-wave hash tables and scratch, and these kernels' access widths are uncalibrated "
                      "for that formula (MI355X_MICROARCH, HBM): an upper bound on HBM bytes, not a measurement")


def _load(rel):
    try:
        return json.load(open(os.path.join(PROFILES, rel)))
    except (OSError, ValueError):
        return None


def pmc_traffic(args, plain_per_launch):
    """(traffic, source, binding) of the dominant kernel from the committed
    PMC passes: traffic = HBM bytes per launch (FETCH_SIZE / WRITE_SIZE of
    the same variant, corrected as the MI355X guide prescribes, per plaintext
    byte x this launch's plaintext bytes); binding = the LDS and VALU busy
    fractions of the same kernel (SQ counters).  The newest summary holding
    the variant wins (profiles/r4, then r3, then round 2's FETCH / WRITE
    file); where none covers it, source names the gap instead of leaving a
    silent null."""
    key = pmc_variant(args)
    if key is None or (args.crc != "full" and args.mode == "seal"):
        return None, "no PMC pass for this mode (%s)" % (key or args.mode), None
    traffic = src = binding = None
    for rel in PMC_FILES:
        v = ((_load(rel) or {}).get("variants") or {}).get(key)
        if not v:
            continue
        if traffic is None and "bytes_per_plain_byte" in v:
            traffic = int(v["bytes_per_plain_byte"] * plain_per_launch)
            src = "profiles/%s %s (%s; %s)" % (rel, key, v.get("fetch_pass"), v.get("write_pass"))
        if binding is None and ("lds_busy" in v or "valu_issue" in v or "salu_issue" in v):
            binding = {k: v[k] for k in ("lds_busy", "valu_issue", "lds_conflict_share", "salu_issue",
                                         "salu_per_byte", "valu_per_byte") if k in v}
            binding["source"] = "profiles/%s %s (%s)" % (rel, key, v.get("lds_pass") or v.get("valu_pass"))
    if traffic is None and key in R2_KEYS:
        k2 = ((_load(PMC_R2) or {}).get("kernels") or {}).get(R2_KEYS[key])
        if k2:
            traffic = int(k2["bytes_per_plain_byte"] * plain_per_launch)
            src = "profiles/%s %s (64 GiB FETCH_SIZE / WRITE_SIZE passes, round 2)" % (PMC_R2, R2_KEYS[key])
    if traffic is None:
        src = "MISSING: no committed PMC pass covers variant %s (profiles/%s)" % (key, ", ".join(PMC_FILES))
        print("bench: warning: " + src, file=sys.stderr)
    return traffic, src, binding


def parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus |= set(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def numa_pin(node):
    """Restrict this process to those of its CPUs that sit on NUMA node
    `node` (the GPU's socket); returns the CPUs it now runs on, or 0 when the
    node's CPUs are unknown or none of them is allowed (affinity unchanged)."""
    try:
        cpus = parse_cpulist(open("/sys/devices/system/node/node%d/cpulist" % node).read())
    except (OSError, ValueError):
        return 0
    inter = os.sched_getaffinity(0) & cpus
    if not inter:
        return 0
    os.sched_setaffinity(0, inter)
    return len(inter)


PCIE_GEN5_X16_GBS = 64.0  # per direction, 32 GT/s x 16 lanes (before 128b/130b and TLP overhead)


def warm_up(args, step, host=False):
    """--warmup untimed steps; in the host-memory modes also until
    --warmup-seconds have passed (default 8 s): the copy engines' D2H rate
    ramps up over the first seconds of traffic on a cold box (tools/pin_probe.hip
    measured 19.9 GB/s, then 50.5 later in the same process)."""
    secs = args.warmup_seconds if args.warmup_seconds is not None else (8.0 if host else 0.0)
    t0 = time.perf_counter()
    done = 0
    while done < args.warmup or time.perf_counter() - t0 < secs:
        step()
        done += 1
    args.warm = {"steps": done, "seconds": round(time.perf_counter() - t0, 1)}
    return done


def host_ingest(args, world, rank, local, dist):
    """BASELINE configs[2]: blocks in pinned host memory, sealed through the
    engine's H2D | transform | D2H pipeline (JFSX_MEM_HOST); value = plaintext
    bytes / s including both PCIe transfers.  Each GPU's pinned pool is capped
    (--host-pool-gib in, the same out) and bound to the GPU's NUMA node; a step
    loops over the pool to make up the GPU's blocks (weak: --blocks per GPU;
    strong: its share of --total-gib)."""
    import ctypes
    import numpy as np
    from juicefs_amd import engine as E
    from juicefs_amd import shard as S
    if args.mode != "seal":
        raise SystemExit("bench: host ingest measures the seal path (configs[2])")
    m, engs = open_engines(args, local)
    nshard = len(engs) if m else world
    L = args.block_bytes
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    shards, specs = [], []
    for k, eng in enumerate(engs):
        sh = Shard()
        sh.eng, sh.s = eng, (k if m else rank)
        sh.base, sh.count, sh.nb, sh.loops = shard_plan(args, nshard, sh.s)
        sh.nseg = -(-L // E.SEG)
        sh.lens = [L] * sh.nb
        sh.node = eng.numa_node()
        # one process per GPU: run on the GPU's socket (the pool's pages are
        # bound to its node either way, by memory policy, not by first touch)
        sh.cpus = numa_pin(sh.node) if (not m and sh.node >= 0) else 0
        sh.pcie_before = eng.pcie_probe()
        sh.hin = eng.alloc_pinned_node(sh.nb * L, sh.node)
        sh.hout = eng.alloc_pinned_node(sh.nb * L, sh.node)
        sh.hcrc = eng.alloc_pinned_node(sh.nb * 4 * sh.nseg, sh.node)
        sh.pool_node = E.host_numa_node(sh.hin, sh.nb * L)
        chunk = min(sh.nb, 256)
        tmp = eng.alloc(chunk * L)
        for b0 in range(0, sh.nb, chunk):  # synthetic input: generated on the device, copied once into the pool
            c = min(chunk, sh.nb - b0)
            eng.gen_synthetic_batch(tmp, L, [L] * c, SEED, sh.base + b0)
            eng.L.jfsx_memcpy_d2h(eng.ctx, sh.hin + b0 * L, tmp.ptr, c * L)
        tmp.free()
        sh.off = len(specs)
        for b in range(sh.nb):
            key, nonce = E.gen_key(SEED, sh.base + b)
            specs.append({"key": key, "nonce": nonce, "src": sh.hin + b * L, "dst": sh.hout + b * L, "len": L,
                          "crc": sh.hcrc + 4 * sh.nseg * b})
        shards.append(sh)
    A, _ = E.Engine.make_blocks(specs)
    loops = loop_arrays(A, shards)
    front = m if m else engs[0]

    def step():
        for arr, n, _ in loops:
            front.seal_batch(algo, arr, n, E.CRC_GEN, E.MEM_HOST)
    warm_up(args, step, host=True)
    for e in engs:
        e.sync()
        e.kernel_time(reset=True)
        e.set_timing(True)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    for e in engs:
        e.sync()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0, local)
    for e in engs:
        e.set_timing(False)
    ktimes = [e.kernel_time(reset=True) for e in engs]
    # the link probed again right after the run (the probe before it has read
    # below what the pipeline itself moved on some boxes); the faster of the two
    for sh in shards:
        after = sh.eng.pcie_probe()
        sh.pcie = {k: max(sh.pcie_before.get(k, 0.0), after.get(k, 0.0)) for k in set(sh.pcie_before) | set(after)}
        sh.pcie_runs = {"before_run": sh.pcie_before, "after_run": after}
        # the pipeline moves equal bytes both ways at once: its bound is the
        # slower direction of the simultaneous (duplex) probe
        sh.peak = min(sh.pcie.get("duplex_h2d", sh.pcie["h2d"]), sh.pcie.get("duplex_d2h", sh.pcie["d2h"]))
    full = None
    if args.verify:
        from oracle import oracle as orc
        full = {"blocks": 0, "oracle_s": 0.0}
        samples = 0
        for sh in shards:
            for b in range(0, sh.nb, max(1, sh.nb // args.verify))[:args.verify]:
                p = orc.gen_block(SEED, sh.base + b, L)
                key, nonce = orc.gen_key(SEED, sh.base + b)
                c, tag = orc.seal(orc.AES256GCM if algo == E.AES256GCM else orc.CHACHA20P1305, key, nonce, p,
                                  fast=True)
                got = np.ctypeslib.as_array((ctypes.c_uint8 * L).from_address(sh.hout + b * L)).tobytes()
                if bytes(A[sh.off + b].tag) != tag or got != c:
                    raise SystemExit("bench: block %d of GPU %d differs from the oracle" % (b, sh.s))
                samples += 1
            crcs = np.ctypeslib.as_array((ctypes.c_uint8 * (sh.nb * 4 * sh.nseg)).from_address(sh.hcrc))
            f = full_check(args, E, [A[sh.off + i] for i in range(sh.nb)], crcs.reshape(sh.nb, 4 * sh.nseg).copy(),
                           sh.lens, sh.base)
            full["blocks"] += f["blocks"]
            full["oracle_s"] = round(full["oracle_s"] + f["oracle_s"], 2)
            full["oracle_threads"] = f["oracle_threads"]
            full.setdefault("tags_sha256", []).append(f["tags_sha256"])
            full.setdefault("crc_arrays_sha256", []).append(f["crc_arrays_sha256"])
        full["ciphertext_samples"] = samples
        full["what"] = ("timed Seal: tags and CRC arrays of all %d pool blocks, and %d ciphertexts, equal to the "
                        "oracle's" % (full["blocks"], samples))
    step_plain = sum(sum(sh.loops) * L for sh in shards)
    value = S.sum_over_ranks(dist, step_plain, local) * args.steps / el / 1e9
    ngpu = len(engs) if m else world
    peak = S.sum_over_ranks(dist, sum(sh.peak for sh in shards), local)
    cpu = cpu_baseline(args, "seal", node=shards[0].node) if rank == 0 and not args.no_cpu else None
    launches = sum(n for _, n in ktimes)
    plain_launch = int(step_plain * args.steps / max(launches, 1))
    traffic, traffic_src, binding = pmc_traffic(args, plain_launch)
    pinned = sum(2 * sh.nb * L + sh.nb * 4 * sh.nseg for sh in shards)
    if rank == 0:
        sh0 = shards[0]
        print(json.dumps({
            "metric": "sealed+checksummed GB/s, 4 MiB blocks (host ingest)", "value": round(value, 2), "unit": "GB/s",
            "n_gpus": ngpu, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": scaling(args),
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), pinned host memory",
            "config": {"workload": "host-ingest: %s GiB per GPU per step (%d pass(es) over a %s GiB pinned pool), "
                                   "%s seal + CRC32C full, 8-slot H2D|transform|D2H pipeline" % (
                                       round(sh0.count * L / 2**30, 3), len(sh0.loops), round(sh0.nb * L / 2**30, 3),
                                       args.algo),
                       "blocks_per_gpu": sh0.count, "pool_blocks_per_gpu": sh0.nb, "block_bytes": L,
                       "algo": args.algo, "mem": "host", "total_gib": args.total_gib or None,
                       "warmup_run": getattr(args, "warm", None),
                       "engine": "jfsx_mctx (one process, %d GPUs)" % ngpu if m else "one process per GPU",
                       "pinned_bytes_per_process": pinned,
                       "numa": [{"gpu_node": sh.node, "pool_node": sh.pool_node, "cpus_on_node": sh.cpus}
                                for sh in shards],
                       "parallelism": "block-sharded x%d, no collective" % ngpu},
            "roofline": {"bound": "pcie", "achieved": round(value, 2), "peak": round(peak, 2), "unit": "GB/s",
                         "frac": round(value / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_note": "HBM bytes per launch of gcm_main_k (one launch per pipeline group)",
                         "peak_basis": "sum over GPUs of min over directions of simultaneous H2D + D2H copies of "
                                       "1 GiB on the pipeline's streams (jfsx_pcie_probe, the better of a probe "
                                       "before and one after the run); one-way rates in pcie_measured",
                         "link_peak": PCIE_GEN5_X16_GBS * ngpu,
                         "frac_of_link": round(value / (PCIE_GEN5_X16_GBS * ngpu), 4),
                         "link_basis": "PCIe Gen5 x16 per direction, 64 GB/s per GPU (32 GT/s x 16 lanes); each "
                                       "direction carries the plaintext rate",
                         "frac_of_one_way_d2h": round(value / S.sum_over_ranks(
                             dist, sum(sh.pcie["d2h"] for sh in shards), local), 4),
                         "pcie_measured": [sh.pcie for sh in shards] if m else sh0.pcie,
                         "pcie_probes": [sh.pcie_runs for sh in shards] if m else sh0.pcie_runs,
                         "kernel_avg_ms": round(sum(ms for ms, _ in ktimes) / max(launches, 1), 3),
                         "kernel_launches": launches, "plain_bytes_per_launch": plain_launch, "binding": binding},
            "cpu_baseline": cpu, "verified_blocks": full["blocks"] if full else 0, "full_check": full}), flush=True)
    for sh in shards:
        for h in (sh.hin, sh.hout, sh.hcrc):
            sh.eng.free_pinned(h)
    if m:
        m.close()
    else:
        engs[0].close()
    if dist is not None:
        dist.destroy_process_group()


def agg_bench(args, world, rank, local, dist, eng):
    """The reference's call shape: every object is sealed by its own
    synchronous call (dataEncryptor.Encrypt, encrypt.go:164-194) from one of
    many goroutines (max-uploads, cmd/flags.go:126-127).  Blocks live in pinned
    host memory (JFSX_MEM_HOST).  value = plaintext GB/s with the calls going
    through the aggregator (jfsx_agg); direct = the same calls as one-block
    jfsx_seal_batch calls (serialised on the context)."""
    import ctypes
    import threading
    import numpy as np
    from juicefs_amd import engine as E
    # each caller owns a contiguous range of nb / threads blocks (its own
    # buffers): no two blocks in flight together are neighbours in memory, so
    # no copy coalesces across callers (the engine merges adjacent ones)
    L = args.block_bytes
    nb = max(1, min(args.blocks, 1024) // args.threads) * args.threads
    nseg = -(-L // E.SEG)
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    # the blocks live on the GPU's NUMA node and the callers run there
    node = eng.numa_node()
    cpus = numa_pin(node) if node >= 0 else 0
    hin, hout = eng.alloc_pinned_node(nb * L, node), eng.alloc_pinned_node(nb * L, node)
    hcrc = eng.alloc_pinned_node(nb * 4 * nseg, node)
    pool_node = E.host_numa_node(hin, nb * L)
    tmp = eng.alloc(L)
    base = rank * nb
    for b in range(nb):
        eng.gen_synthetic(tmp, L, SEED, base + b)
        eng.sync()
        eng.L.jfsx_memcpy_d2h(eng.ctx, hin + b * L, tmp.ptr, L)
    tmp.free()
    specs = []
    for b in range(nb):
        key, nonce = E.gen_key(SEED, base + b)
        specs.append({"key": key, "nonce": nonce, "src": hin + b * L, "dst": hout + b * L, "len": L,
                      "crc": hcrc + 4 * nseg * b})
    blks, n = eng.make_blocks(specs)
    T = args.threads
    per = nb // T
    is_open = args.agg_op == "open"
    hdec = hcrc2 = None
    if is_open:
        # the objects to open: sealed once here (tags into blks, plaintext
        # CRC arrays into hcrc); the timed calls open them into hdec and write
        # the cache file's CRC arrays (JFSX_CRC_GEN of the plaintext) to hcrc2
        eng.seal_batch(algo, blks, nb, E.CRC_GEN, E.MEM_HOST)
        hdec = eng.alloc_pinned_node(nb * L, node)
        hcrc2 = eng.alloc_pinned_node(nb * 4 * nseg, node)
        ospecs = [dict(sp, src=hout + b * L, dst=hdec + b * L, crc=hcrc2 + 4 * nseg * b, tag=bytes(blks[b].tag))
                  for b, sp in enumerate(specs)]
        oblks, _ = eng.make_blocks(ospecs)

    def run(call, steps):
        errs = []

        def worker(t):
            try:
                for _ in range(steps):
                    for b in range(t * per, (t + 1) * per):
                        call(b)
            except BaseException as e:  # noqa: B902 -- reported below
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return time.perf_counter() - t0

    def direct(b):
        if is_open:
            eng._check(eng.L.jfsx_open_batch(eng.ctx, algo, 1, ctypes.byref(oblks[b]), E.CRC_GEN, E.MEM_HOST), "open")
        else:
            eng._check(eng.L.jfsx_seal_batch(eng.ctx, algo, 1, ctypes.byref(blks[b]), E.CRC_GEN, E.MEM_HOST), "seal")

    d_steps = max(1, args.steps // 5)
    run(direct, 1)
    d_el = run(direct, d_steps)
    with E.Aggregator(eng, window_us=args.agg_window_us, max_bytes=args.agg_max_mb << 20) as agg:
        def through(b):
            if is_open:
                agg.open(algo, oblks[b], E.CRC_GEN, E.MEM_HOST)
            else:
                agg.seal(algo, blks[b], E.CRC_GEN, E.MEM_HOST)
        warm_up(args, lambda: run(through, 1), host=True)
        c0, b0, k0 = agg.stats()
        barrier(dist)
        cpu0 = host_cpu_seconds()
        el = max_over_ranks(dist, run(through, args.steps), local)
        cpu_used = host_cpu_seconds() - cpu0
        c1, b1, k1 = agg.stats()
    verified = 0
    if args.verify:
        from oracle import oracle as orc
        for b in range(0, nb, max(1, nb // args.verify))[:args.verify]:
            p = orc.gen_block(SEED, base + b, L)
            key, nonce = orc.gen_key(SEED, base + b)
            c, tag = orc.seal(orc.AES256GCM if algo == E.AES256GCM else orc.CHACHA20P1305, key, nonce, p, fast=True)
            got = np.ctypeslib.as_array((ctypes.c_uint8 * L).from_address(hout + b * L)).tobytes()
            if bytes(blks[b].tag) != tag or got != c:
                raise SystemExit("bench: block %d differs from the oracle" % b)
            if is_open:
                pl = np.ctypeslib.as_array((ctypes.c_uint8 * L).from_address(hdec + b * L)).tobytes()
                if pl != p.tobytes():
                    raise SystemExit("bench: block %d: opened plaintext differs from the oracle's" % b)
            verified += 1
        if is_open:
            bad = [b for b in range(nb) if oblks[b].status != E.OK]
            if bad:
                raise SystemExit("bench: %d opened blocks failed (block %d: status %d)"
                                 % (len(bad), bad[0], oblks[bad[0]].status))
    full = None
    if args.verify:
        crcs = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * 4 * nseg)).from_address(hcrc2 if is_open else hcrc))
        full = full_check(args, E, blks, crcs.reshape(nb, 4 * nseg).copy(), [L] * nb, base)
        full["what"] = ("per-object Open calls through the aggregator (every status OK): setup tags and the timed "
                        "calls' plaintext CRC arrays: " if is_open else
                        "per-object Seal calls through the aggregator: ") + full["what"]
        verified = nb
    value = world * nb * L * args.steps / el / 1e9
    cpu = (cpu_baseline(args, "open" if is_open else "seal", node=node) if rank == 0 and not args.no_cpu
           else None)
    gb = world * nb * L * args.steps / 1e9
    host_cpu = {"cpu_seconds": round(cpu_used, 3), "cpu_s_per_GB": round(cpu_used / gb, 4),
                "cores_busy": round(cpu_used / el, 2),
                "cpu_baseline_core_s_per_GB": cpu["core_s_per_GB"] if cpu else None,
                "note": "getrusage(RUSAGE_SELF) over the timed region: every thread of this process (the Python "
                        "callers and their ctypes calls, the aggregator's dispatchers); no bounce copies (pinned "
                        "blocks)"}
    pcie, probes = best_link_probe(eng)
    duplex = min(pcie["duplex_h2d"], pcie["duplex_d2h"])
    if rank == 0:
        print(json.dumps({
            "metric": "per-object %s GB/s, %d threads, 4 MiB host blocks (aggregator)" % (
                "opened+checksummed" if is_open else "sealed+checksummed", T),
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), pinned host memory",
            "config": {"workload": "%d one-block %s calls per step from %d threads, each on its own range of "
                                   "blocks, %s + CRC32C full, JFSX_MEM_HOST" % (nb, "Open" if is_open else "Seal", T,
                                                                               args.algo), "blocks_per_gpu": nb, "block_bytes": L, "algo": args.algo,
                       "mode": "agg", "op": args.agg_op, "window_us": args.agg_window_us,
                       "max_batch_bytes": args.agg_max_mb << 20,
                       "dispatchers_per_gpu": int(os.environ.get("JFSX_AGG_DISPATCHERS", "4")),
                       "warmup_run": getattr(args, "warm", None),
                       "numa": {"gpu_node": node, "pool_node": pool_node, "cpus_on_node": cpus}},
            "aggregator": {"calls": c1 - c0, "batches": b1 - b0,
                           "mean_batch_blocks": round((k1 - k0) / max(b1 - b0, 1), 2)},
            "direct_one_block_calls_GBs": round(nb * L * d_steps / d_el / 1e9, 2),
            "direct_note": "the same calls as one-block jfsx_seal_batch / jfsx_open_batch calls from the same threads, "
                           "no aggregator "
                           "(host batches share the context's pipeline)",
            "roofline": {"bound": "pcie", "achieved": round(value, 2), "peak": duplex, "unit": "GB/s",
                         "frac": round(value / duplex, 4), "peak_basis": "min over directions of simultaneous H2D + "
                         "D2H copies (jfsx_pcie_probe after the run, best of 3 per rate)", "pcie_measured": pcie,
                         "pcie_probes": probes,
                         "frac_of_link": round(value / PCIE_GEN5_X16_GBS, 4)},
            "host_cpu": host_cpu, "cpu_baseline": cpu, "verified_blocks": verified, "full_check": full}), flush=True)
    for h in (hin, hout, hcrc, hdec, hcrc2):
        if h:
            eng.free_pinned(h)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def best_link_probe(eng, runs=3):
    """the link's rates for the per-object lines: jfsx_pcie_probe after the
    run, the best of `runs` probes per rate (one probe has read a duplex rate
    15% under the others on a quiet box; the ceiling is what the link can
    do), with every probe kept"""
    probes = [eng.pcie_probe() for _ in range(runs)]
    best = {k: max(p.get(k, 0.0) for p in probes) for k in probes[0]}
    return best, probes


class ClockLog:
    """--log-clocks: the GPUs' DPM levels (pp_dpm_sclk / mclk / fclk / socclk,
    the level marked '*') and gpu_busy_percent, read from sysfs every 100 ms in
    a thread over the warm-up and the timed region (read only; a diagnostic of
    run-to-run spread).  summary(): per card that was busy, the share of
    samples at each level, per phase."""

    FILES = ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk")

    def __init__(self, period=0.1, device=0):
        import glob
        import threading
        self.cards = sorted(glob.glob("/sys/class/drm/card[0-9]*/device"))
        self.ours = None  # the card of this process's GPU, by PCI address (hipDeviceGetPCIBusId)
        self.pci = None
        try:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")  # the runtime libjfsx already loaded into this process
            buf = ctypes.create_string_buffer(64)
            if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
                raise RuntimeError("hipDeviceGetPCIBusId failed")
            self.pci = buf.value.decode().lower().rsplit(".", 1)[0] + "."
            for c in self.cards:
                if os.path.basename(os.path.realpath(c)).startswith(self.pci):
                    self.ours = c.split("/")[-2]
            if self.ours is None:
                self.pci += " (cards at %s)" % ", ".join(os.path.basename(os.path.realpath(c)) for c in self.cards)
        except Exception as e:  # noqa: BLE001 -- diagnostic only: fall back to every busy card
            self.pci = "unknown: %s" % e
        self.period, self.phase, self.samples = period, "warmup", []
        self.ev = threading.Event()
        self.th = threading.Thread(target=self._loop, daemon=True)

    @staticmethod
    def _read(path):
        try:
            with open(path) as f:
                return f.read()
        except OSError:
            return None

    def _loop(self):
        while not self.ev.wait(self.period):
            row = {}
            for c in self.cards:
                busy = self._read(c + "/gpu_busy_percent")
                lv = {}
                for n in self.FILES:
                    t = self._read(c + "/" + n)
                    cur = [ln.split(":", 1)[1].strip() for ln in (t or "").splitlines() if ln.rstrip().endswith("*")]
                    lv[n[7:]] = cur[0].rstrip("*").strip() if cur else None
                row[c.split("/")[-2]] = (int(busy) if busy and busy.strip().isdigit() else None, lv)
            self.samples.append((self.phase, row))

    def start(self):
        self.th.start()

    def mark(self, phase):
        self.phase = phase

    def stop(self):
        self.ev.set()
        self.th.join()

    def summary(self):
        import collections
        out = {}
        for card in {k for _, row in self.samples for k in row}:
            busy = [row[card][0] for _, row in self.samples if row.get(card) and row[card][0] is not None]
            if card != self.ours and (not busy or max(busy) == 0):
                continue
            per = {}
            for phase in ("warmup", "timed"):
                rows = [row[card] for ph, row in self.samples if ph == phase and card in row]
                if not rows:
                    continue
                d = {"samples": len(rows), "busy_mean": round(sum(b or 0 for b, _ in rows) / len(rows), 1)}
                for n in ("sclk", "mclk", "fclk", "socclk"):
                    cnt = collections.Counter(lv.get(n) for _, lv in rows)
                    d[n] = {str(k): round(v / len(rows), 3) for k, v in cnt.most_common()}
                per[phase] = d
            out[card + (" (this GPU)" if card == self.ours else "")] = per
        if out and self.ours is None:
            out["note"] = "this GPU's card not identified (PCI %s): every busy card is listed" % self.pci
        return out or {"note": "no busy card readable under /sys/class/drm"}


def host_cpu_seconds():
    """user + system CPU seconds of this process so far (every thread: the
    callers, the aggregator's dispatchers, the engine's bounce copies)"""
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def readat_ranges(lens, per_block, seed):
    """configs[4]'s reads: per image, per_block (off, size) ranges, uniform
    offsets and sizes (unaligned, SplitMix64 of (seed, block, k)), each
    inside the data: [(block, off, size)]"""
    out = []
    for b, n in enumerate(lens):
        for k in range(per_block):
            z = ragged_len(seed ^ 0x5245414441, b * 64 + k, 2**40)
            off = z % n
            size = 1 + (z >> 20) % (n - off)
            out.append((b, off, size))
    return out


def agg_heap_bench(args, world, rank, local, dist, eng):
    """The drop-in's per-object calls on ordinary pageable heap memory (the
    reference's Go-heap slices: io.ReadAll's result and a fresh make([]byte)
    in Encrypt, encrypt.go:183, :258; cache pages, page.go:42-50), from
    --threads callers at once (max-uploads, cmd/flags.go:124-128):
      seal      jfsx_agg_data_encrypt_ex: plaintext -> object (header with a
                256-B wrapped key, C, tag) + --agg-crc checksums
      open      jfsx_agg_data_decrypt_ex: object -> plaintext + checksums
      checksum  jfsx_agg_crc32c GEN: checksum() of a page (disk_cache.go:1218-1231)
      verify    jfsx_cache_verify, level full, whole block: the cache hit
                (disk_cache.go:1255-1329 with off 0, size = length)
      readat    jfsx_cache_verify at --level shrink|extend on configs[4]'s
                ragged images, random unaligned ranges
    The engine copies each pageable block into its own pinned bounce buffer on
    the calling thread (include/jfsx.h JFSX_MEM_HOST).  value = plaintext (or
    returned) GB/s; host_cpu = this process's CPU seconds over the timed
    region, beside the CPU baseline's cores x seconds for the same bytes."""
    import ctypes
    import threading
    import numpy as np
    from juicefs_amd import engine as E
    op = args.agg_op
    T = args.threads
    L = args.block_bytes
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    node = eng.numa_node()
    cpus = numa_pin(node) if node >= 0 else 0
    ragged = op == "readat" or args.ragged
    nb = max(1, min(args.blocks, 512) // T) * T
    base = rank * nb
    lens = [ragged_len(SEED, base + b, L) for b in range(nb)] if ragged else [L] * nb
    nseg = -(-L // E.SEG)
    cs = 4 * nseg          # CRC array stride
    S = L + 287            # object stride: 3 + 256 + 12 header, C, 16-B tag
    IS = L + cs            # cache-file image stride: data, BE32 CRCs
    # heap (pageable) buffers, filled from the device generator
    pt = np.empty(nb * L, np.uint8)
    tmp = eng.alloc(L)
    for b in range(nb):
        eng.gen_synthetic(tmp, lens[b], SEED, base + b)
        eng.sync()
        eng._check(eng.L.jfsx_memcpy_d2h(eng.ctx, pt.ctypes.data + b * L, tmp.ptr, lens[b]), "memcpy")
    tmp.free()
    keys = np.zeros((nb, 32), np.uint8)
    nonces = np.zeros((nb, 12), np.uint8)
    for b in range(nb):
        k, nn = E.gen_key(SEED, base + b)
        keys[b] = np.frombuffer(bytes(k), np.uint8)
        nonces[b] = np.frombuffer(bytes(nn), np.uint8)
    wrapped = np.random.default_rng(SEED).integers(0, 256, 256, dtype=np.uint8)
    segs = np.zeros(nb * cs, np.uint8)       # checksum() arrays the calls return
    ocrc = np.zeros(nb, np.uint32)           # object-store CRCs (seal) / expected (open)
    want_seg = args.agg_crc in ("seg", "both")
    want_obj = args.agg_crc in ("obj", "both")
    pp, kp, np_, wp, sp, op_ = (pt.ctypes.data, keys.ctypes.data, nonces.ctypes.data, wrapped.ctypes.data,
                                segs.ctypes.data, ocrc.ctypes.data)
    objs = out = imgs = reads = None
    verified = {}
    agg = E.Aggregator(eng, window_us=args.agg_window_us, max_bytes=args.agg_max_mb << 20)
    A = agg.h
    if op in ("seal", "open"):
        objs = np.empty(nb * S, np.uint8)
        obp = objs.ctypes.data
        enc_agg, enc_dir = eng.L.jfsx_agg_data_encrypt_ex, eng.L.jfsx_data_encrypt_ex
        dec_agg, dec_dir = eng.L.jfsx_agg_data_decrypt_ex, eng.L.jfsx_data_decrypt_ex

        def encrypt(b, olen, h=A, fn=enc_agg, obj=want_obj, seg=want_seg):
            return fn(h, algo, kp + 32 * b, np_ + 12 * b, wp, 256, pp + L * b, lens[b], obp + S * b, S,
                      ctypes.byref(olen), op_ + 4 * b if obj else None, sp + cs * b if seg else None)
        if op == "open":
            # the stored objects (and their object CRCs) made once, untimed
            olen = ctypes.c_uint64()
            for b in range(nb):
                rc = encrypt(b, olen, obj=True, seg=False)
                if rc:
                    raise SystemExit("bench: setup encrypt failed (%d)" % rc)
            out = np.empty(nb * L, np.uint8)
            dp = out.ctypes.data
            got = np.zeros(nb, np.uint32)
            gp = got.ctypes.data

            def call_with(h, fn):
                def call(b, st):
                    return fn(h, algo, kp + 32 * b, obp + S * b, lens[b] + 287, dp + L * b, L, ctypes.byref(st),
                              op_ + 4 * b if want_obj else None, gp + 4 * b if want_obj else None,
                              sp + cs * b if want_seg else None)
                return call
            through, direct = call_with(A, dec_agg), call_with(eng.ctx, dec_dir)
        else:
            def through(b, st):
                return encrypt(b, st)

            def direct(b, st):
                return encrypt(b, st, h=eng.ctx, fn=enc_dir)
    elif op == "checksum":
        R = (E.jfsx_range * nb)()
        for b in range(nb):
            R[b].data, R[b].len, R[b].crc = pp + L * b, lens[b], sp + cs * b
        crc_agg, crc_dir = eng.L.jfsx_agg_crc32c, eng.L.jfsx_crc32c_segments

        def through(b, st):
            return crc_agg(A, ctypes.byref(R[b]), E.CRC_GEN, E.MEM_HOST)

        def direct(b, st):
            return crc_dir(eng.ctx, 1, ctypes.byref(R[b]), E.CRC_GEN, E.MEM_HOST)
    else:
        # cache-file images (data || checksum()); the trailers made by the
        # engine itself, untimed (checked against the oracle afterwards)
        imgs = np.empty(nb * IS, np.uint8)
        ip = imgs.ctypes.data
        for b in range(nb):
            ctypes.memmove(ip + IS * b, pp + L * b, lens[b])
        R = (E.jfsx_range * nb)()
        for b in range(nb):
            R[b].data, R[b].len, R[b].crc = ip + IS * b, lens[b], ip + IS * b + lens[b]
        eng.crc32c_segments(R, nb, E.CRC_GEN, E.MEM_HOST)
        # ReadAt's destination: per block for the whole-block verify, per
        # calling thread for the random reads (several reads of one image)
        out = np.empty((nb if op == "verify" else T) * L, np.uint8)
        dp = out.ctypes.data
        level = "full" if op == "verify" else args.level
        lv = {"full": 1, "shrink": 2, "extend": 3}[level]
        reads = ([(b, 0, lens[b]) for b in range(nb)] if op == "verify"
                 else readat_ranges(lens, args.reads_per_block, SEED + base))
        cv = eng.L.jfsx_cache_verify
        flen = [lens[b] + 4 * max(1, -(-lens[b] // E.SEG)) for b in range(nb)]
        nret = np.zeros(len(reads), np.uint64)

        def through(r, st):
            b, off, size = reads[r]
            n, g, e, s, t = st
            rc = cv(eng.ctx, ip + IS * b, flen[b], lens[b], lv, off, size, dp + L * (b if op == "verify" else t),
                    ctypes.byref(n), ctypes.byref(g), ctypes.byref(e), ctypes.byref(s))
            nret[r] = n.value
            return rc
        direct = None
    units = list(range(len(reads))) if reads is not None else list(range(nb))
    unit_bytes = [reads[r][2] for r in units] if reads is not None else lens
    per = len(units) // T
    errs = []

    def run(call, steps):
        def worker(t):
            try:
                st = ((ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int64(), t)
                      if op in ("verify", "readat") else ctypes.c_uint64())
                for _ in range(steps):
                    for u in units[t * per:(t + 1) * per]:
                        rc = call(u, st)
                        if rc:
                            raise RuntimeError("unit %d: jfsx rc %d" % (u, rc))
            except BaseException as e:  # noqa: B902 -- reported below
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise SystemExit("bench: %s" % errs[0])
        return time.perf_counter() - t0
    step_bytes = sum(unit_bytes[:per * T])
    d_val = None
    if direct is not None:
        d_steps = max(1, args.steps // 5)
        run(direct, 1)
        d_val = round(step_bytes * d_steps / run(direct, d_steps) / 1e9, 2)
    clocks = ClockLog() if args.log_clocks else None
    if clocks:
        clocks.start()
    warm_up(args, lambda: run(through, 1), host=True)
    if clocks:
        clocks.mark("timed")
    c0, b0, k0 = agg.stats()
    m0 = eng.metrics(reset=False)
    barrier(dist)
    cpu0 = host_cpu_seconds()
    el = max_over_ranks(dist, run(through, args.steps), local)
    cpu_used = host_cpu_seconds() - cpu0
    if clocks:
        clocks.stop()
    c1, b1, k1 = agg.stats()
    agg.close()
    value = world * step_bytes * args.steps / el / 1e9
    # checker only, after the timed region
    full = None
    if args.verify:
        import hashlib
        from oracle import oracle as orc
        oalgo = orc.AES256GCM if algo == E.AES256GCM else orc.CHACHA20P1305
        samples = list(range(0, nb, max(1, nb // max(args.verify, 1))))[:args.verify]
        if op in ("seal", "open"):
            arr = segs.reshape(nb, cs).copy()
            tags = objs.reshape(nb, S)
            f = full_check(args, E, None, arr, lens, base) if want_seg else {"blocks": nb}
            etags, _, _ = orc.expect_batch(oalgo, host_cores()[0], lens, SEED, base, cs)
            gt = np.stack([tags[b, lens[b] + 271:lens[b] + 287] for b in range(nb)])
            bad = np.nonzero((gt != etags).any(axis=1))[0]
            if bad.size:
                raise SystemExit("bench: object %d: tag differs from the oracle (%d objects)" % (bad[0], bad.size))
            f["tags_sha256"] = hashlib.sha256(gt.tobytes()).hexdigest()
            for b in samples:
                p = orc.gen_block(SEED, base + b, lens[b])
                key, nonce = orc.gen_key(SEED, base + b)
                o = tags[b, :lens[b] + 287].tobytes()
                if o != orc.data_encrypt(oalgo, key, nonce, wrapped.tobytes(), p.tobytes()):
                    raise SystemExit("bench: object %d differs from the oracle's Encrypt" % b)
                if op == "open" and out[L * b:L * b + lens[b]].tobytes() != p.tobytes():
                    raise SystemExit("bench: object %d: decrypted plaintext differs from the oracle's" % b)
            if want_obj or op == "open":
                bad = [b for b in range(nb) if int(orc.object_checksum(tags[b, :lens[b] + 287].tobytes(), hw=True))
                       != int(ocrc[b])]
                if bad:
                    raise SystemExit("bench: object %d: object CRC differs from the oracle (%d)" % (bad[0], len(bad)))
            f["what"] = ("per-object %s calls on heap buffers: tags of all %d objects%s%s equal to the oracle's, %d "
                         "whole objects%s equal to the oracle's Encrypt" % (
                             "Encrypt" if op == "seal" else "Decrypt", nb,
                             ", the calls' plaintext checksum() arrays" if want_seg else "",
                             ", every object CRC" if (want_obj or op == "open") else "", len(samples),
                             " and their decrypted plaintexts" if op == "open" else ""))
            full = f
        elif op == "checksum":
            full = full_check(args, E, None, segs.reshape(nb, cs).copy(), lens, base)
            full["what"] = "checksum() calls on heap pages: " + full["what"]
        else:
            trail = np.stack([np.pad(imgs[IS * b + lens[b]:IS * b + lens[b] + 4 * max(1, -(-lens[b] // E.SEG))],
                                     (0, cs - 4 * max(1, -(-lens[b] // E.SEG)))) for b in range(nb)])
            full = full_check(args, E, None, trail, lens, base)
            want = np.array([min(s, lens[b] - o) for b, o, s in reads], np.uint64)
            if (nret != want).any():
                r = int(np.nonzero(nret != want)[0][0])
                raise SystemExit("bench: read %d returned %d bytes, ReadAt returns %d" % (r, nret[r], want[r]))
            for r in range(0, len(reads), max(1, len(reads) // max(args.verify, 1)))[:args.verify]:
                b, o, s = reads[r]
                img = imgs[IS * b:IS * b + lens[b] + 4 * max(1, -(-lens[b] // E.SEG))]
                rc, data = orc.cache_readat(img.tobytes(), lens[b], lv, o, s)[:2]
                # the timed read's bytes (whole-block verify), or the same read
                # made again (random reads share their thread's destination)
                mine = (out[L * b:L * b + s].tobytes() if op == "verify"
                        else eng.cache_verify(img, lens[b], lv, o, s)[1])
                if rc != 0 or data != mine:
                    raise SystemExit("bench: read %d differs from the oracle's ReadAt" % r)
            full["what"] = ("cache-file trailers of all %d images equal to the oracle's; every one of %d %s reads "
                            "returned ReadAt's byte count with status OK (each verified its window); %d reads' bytes "
                            "equal to the oracle's ReadAt" % (nb, len(reads), level,
                                                             min(args.verify, len(reads))))
    m1 = eng.metrics(reset=False)
    cpu = None
    if rank == 0 and not args.no_cpu:
        if op in ("verify", "readat"):
            cpu = cpu_readat_baseline(args, lens, reads, "full" if op == "verify" else args.level, node=node)
        else:
            cpu = cpu_baseline(args, {"seal": "encrypt", "open": "objdecrypt", "checksum": "crc"}[op],
                               lens if (ragged or L != BLOCK) else None, node=node)
    pcie, probes = best_link_probe(eng)
    if op in ("seal", "open"):  # the block goes up and comes back down: both directions at once
        link_peak = min(pcie["duplex_h2d"], pcie["duplex_d2h"])
        peak_basis = "min over directions of simultaneous H2D + D2H copies (jfsx_pcie_probe after the run, best of 3)"
    else:  # checksum / ReadAt verify: only the data goes up (results land in the pinned mirror)
        link_peak = pcie["h2d"]
        peak_basis = "H2D copies alone (jfsx_pcie_probe after the run, best of 3): the CRC calls move data one way"
    gb = world * step_bytes * args.steps / 1e9
    host_cpu = {"cpu_seconds": round(cpu_used, 3), "cpu_s_per_GB": round(cpu_used / gb, 4),
                "cores_busy": round(cpu_used / el, 2),
                "note": "getrusage(RUSAGE_SELF) over the timed region: every thread of this process (the Python "
                        "callers and their ctypes calls, the aggregator's dispatchers, the bounce copies in and out)"}
    if cpu:
        host_cpu["cpu_baseline_core_s_per_GB"] = cpu["core_s_per_GB"]
    what = {"seal": "encrypted+checksummed", "open": "decrypted+checksummed", "checksum": "checksummed",
            "verify": "cache-hit verified (ReadAt, level full)", "readat": "read (ReadAt, level %s)" % args.level}[op]
    if rank == 0:
        print(json.dumps({
            "metric": "per-object %s GB/s, %d threads, %s heap buffers" % (
                what, T, "ragged 64 KiB-4 MiB" if ragged else "4 MiB"),
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), pageable heap memory (numpy)",
            "config": {"workload": "%d %s calls per step from %d threads on pageable heap buffers%s" % (
                len(units), {"seal": "jfsx_agg_data_encrypt_ex", "open": "jfsx_agg_data_decrypt_ex",
                             "checksum": "jfsx_agg_crc32c (GEN)", "verify": "jfsx_cache_verify (level full, whole block)",
                             "readat": "jfsx_cache_verify (level %s, random unaligned ranges)" % args.level}[op],
                T, (", %s, checksums: %s" % (args.algo, args.agg_crc)) if op in ("seal", "open") else ""),
                "blocks_per_gpu": nb, "block_bytes": "ragged" if ragged else L, "algo": args.algo,
                "mode": "agg", "op": op, "buffers": "heap", "agg_crc": args.agg_crc if op in ("seal", "open") else None,
                "level": args.level if op == "readat" else None,
                "reads": len(reads) if reads is not None else None, "window_us": args.agg_window_us,
                "max_batch_bytes": args.agg_max_mb << 20, "warmup_run": getattr(args, "warm", None),
                "numa": {"gpu_node": node, "cpus_on_node": cpus}},
            "aggregator": {"calls": c1 - c0, "batches": b1 - b0,
                           "mean_batch_blocks": round((k1 - k0) / max(b1 - b0, 1), 2)} if op != "verify" and
            op != "readat" else None,
            "direct_calls_GBs": d_val,
            "engine_metrics_delta": {k: m1[k] - m0[k] for k in
                                     ("seal_batches", "seal_bytes", "open_batches", "open_bytes", "crc_batches",
                                      "crc_bytes")},
            "host_cpu": host_cpu,
            **({"clocks": clocks.summary()} if clocks else {}),
            "roofline": {"bound": "pcie", "achieved": round(value, 2), "peak": link_peak, "unit": "GB/s",
                         "frac": round(value / link_peak, 4), "peak_basis": peak_basis,
                         "pcie_measured": pcie, "pcie_probes": probes, "h2d_one_way": pcie["h2d"],
                         "frac_of_link": round(value / PCIE_GEN5_X16_GBS, 4)},
            "cpu_baseline": cpu, "verified_blocks": nb if full else 0, "full_check": full}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def aggcodec_bench(args, world, rank, local, dist, eng):
    """The codec stage in the reference's call shape: cachedStore.upload /
    load call Compress / Decompress once per block, from up to max-uploads
    (default 20, cmd/flags.go:125-128) goroutines (cached_store.go:387, :738).
    Blocks are 4 MiB of word text in pinned host memory.  value = uncompressed
    GB/s of one-block calls through the aggregator (jfsx_agg) from --threads
    threads; beside it the same blocks as one 256-block batch call and as
    one-block calls on the context (no aggregator), and the C library on
    every host core."""
    import ctypes
    import threading
    import numpy as np
    from juicefs_amd import engine as E
    from tests import zstd_lib
    L = args.block_bytes
    # a few rounds of --threads concurrent calls (a one-wave-per-object codec
    # call takes 0.1-2 s on a 4 MiB block, so the per-call shape is kept short)
    nb = min(args.blocks, 3 * args.threads)
    codec = args.codec
    comp = codec in ("lz4", "zstd")
    bound = int(E.lz4_bound(L) if codec in ("lz4", "unlz4") else E.zstd_bound(L))
    pool = _text_pool(16 << 20, SEED + rank)
    raw = eng.alloc_pinned(nb * L)
    cmp_ = eng.alloc_pinned(nb * bound)
    out = eng.alloc_pinned(nb * L)
    rawv = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * L)).from_address(raw))
    for b in range(nb):
        o = ((rank * nb + b) * 2654435761) % (pool.size - L)
        rawv[b * L:(b + 1) * L] = pool[o:o + L]
    carr, _ = eng.make_zblocks((raw + b * L, L, cmp_ + b * bound, bound) for b in range(nb))
    if codec in ("lz4", "unlz4"):
        eng.lz4_compress_batch(carr, nb, E.MEM_HOST)
    else:
        eng.zstd_compress_batch(carr, nb, E.MEM_HOST)
    clens = [carr[b].out_len for b in range(nb)]
    if comp:
        arr, _ = eng.make_zblocks((raw + b * L, L, cmp_ + b * bound, bound) for b in range(nb))
    else:
        arr, _ = eng.make_zblocks((cmp_ + b * bound, clens[b], out + b * L, L) for b in range(nb))
    batch_fn = {"lz4": eng.L.jfsx_lz4_compress_batch, "unlz4": eng.L.jfsx_lz4_decompress_batch,
                "zstd": eng.L.jfsx_zstd_compress_batch, "unzstd": eng.L.jfsx_zstd_decompress_batch}[codec]
    T = args.threads

    def run(call, steps):
        errs = []

        def worker(t):
            try:
                for _ in range(steps):
                    for b in range(t, nb, T):
                        call(b)
            except BaseException as e:  # noqa: B902 -- reported below
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return time.perf_counter() - t0

    def direct(b):
        eng._check(batch_fn(eng.ctx, 1, ctypes.byref(arr[b]), E.MEM_HOST), "one-block " + codec)
    batch_fn(eng.ctx, nb, arr, E.MEM_HOST)  # warm the workspace
    t0 = time.perf_counter()
    eng._check(batch_fn(eng.ctx, nb, arr, E.MEM_HOST), codec + " batch")
    batch_s = time.perf_counter() - t0
    print("bench: aggcodec %s: %d-block batch %.3f s" % (codec, nb, batch_s), file=sys.stderr, flush=True)
    nd = min(nb, 8)  # one-block calls on the context, serialised: a bounded sample
    t0 = time.perf_counter()
    for b in range(nd):
        direct(b)
    d_el = (time.perf_counter() - t0) * nb / nd
    print("bench: aggcodec %s: %d one-block calls %.3f s" % (codec, nd, d_el * nd / nb), file=sys.stderr, flush=True)
    with E.Aggregator(eng, window_us=args.agg_window_us) as agg:
        f = {"lz4": agg.lz4_compress, "unlz4": agg.lz4_decompress, "zstd": agg.zstd_compress,
             "unzstd": agg.zstd_decompress}[codec]
        run(lambda b: f(arr[b]), args.warmup)
        c0, b0, k0 = agg.stats()
        barrier(dist)
        el = max_over_ranks(dist, run(lambda b: f(arr[b]), args.steps), local)
        c1, b1, k1 = agg.stats()
    # every call's result: compressed bytes equal to the library's, or the block back
    verified = 0
    for b in range(0, nb, max(1, nb // max(args.verify, 1)))[:max(args.verify, 1)]:
        src_b = rawv[b * L:(b + 1) * L].tobytes()
        if arr[b].status != E.OK:
            raise SystemExit("bench: block %d status %d" % (b, arr[b].status))
        if comp:
            got = np.ctypeslib.as_array((ctypes.c_uint8 * arr[b].out_len).from_address(cmp_ + b * bound)).tobytes()
            if codec == "zstd" and got != zstd_lib.compress_simple(src_b, 1):
                raise SystemExit("bench: block %d differs from libzstd level 1" % b)
            if codec == "lz4":
                from oracle import oracle as orc
                if got != orc.lz4_compress(src_b):
                    raise SystemExit("bench: block %d differs from the LZ4 library" % b)
        else:
            got = np.ctypeslib.as_array((ctypes.c_uint8 * L).from_address(out + b * L)).tobytes()
            if got != src_b:
                raise SystemExit("bench: block %d does not decode" % b)
        verified += 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = [rawv[b * L:(b + 1) * L].tobytes() for b in range(min(nb, 64))]
        if codec in ("lz4", "unlz4"):
            cpu = lz4_cpu_baseline(sample, L, decompress=codec == "unlz4")
        elif codec == "zstd":
            cpu = zstdc_cpu_baseline(sample, L)
        else:
            cpu = zstd_cpu_baseline([zstd_lib.compress_simple(x, 1) for x in sample], L)
    value = world * nb * L * args.steps / el / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "per-call %s GB/s (uncompressed bytes), %d threads, 4 MiB host blocks (aggregator)" % (codec, T),
            "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (zipf word text), pinned host memory",
            "config": {"workload": "%d one-block %s calls per step from %d threads, JFSX_MEM_HOST" % (nb, codec, T),
                       "blocks_per_gpu": nb, "block_bytes": L, "mode": "aggcodec", "codec": codec,
                       "window_us": args.agg_window_us, "ratio": round(sum(clens) / (nb * L), 4)},
            "aggregator": {"calls": c1 - c0, "batches": b1 - b0,
                           "mean_batch_blocks": round((k1 - k0) / max(b1 - b0, 1), 2)},
            "batch_%d_blocks_GBs" % nb: round(nb * L / batch_s / 1e9, 3),
            "direct_one_block_calls_GBs": round(nb * L / d_el / 1e9, 3), "direct_sample_blocks": nd,
            "roofline": None, "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    for h in (raw, cmp_, out):
        eng.free_pinned(h)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def _text_pool(nbytes, seed):
    """Word text (zipf-distributed words of a 300-word vocabulary): the
    compressible synthetic input of the lz4 modes."""
    import numpy as np
    rng = np.random.default_rng(seed)
    nw = 300
    lens = rng.integers(1, 10, nw)
    tab = np.full((nw, 11), 32, np.uint8)
    for i in range(nw):
        tab[i, :lens[i]] = rng.integers(97, 123, lens[i], dtype=np.uint8)
    idx = rng.zipf(1.3, nbytes // 2 + 8) % nw
    L = lens[idx] + 1
    k = int(np.searchsorted(np.cumsum(L), nbytes)) + 1
    idx, L = idx[:k], L[:k]
    off = np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L)
    return tab[np.repeat(idx, L), off][:nbytes]


def lz4_cpu_baseline(blocks, L, decompress=False):
    """LZ4_compress_default (or LZ4_decompress_safe) of the system LZ4 C
    library (the library hungys/go-lz4 wraps) over a bounded sample, one thread
    per core (ctypes releases the GIL)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    lib = ctypes.CDLL("liblz4.so.1")
    threads, note = host_cores()
    cap = lib.LZ4_compressBound(L)
    outs = [ctypes.create_string_buffer(max(cap, L)) for _ in range(threads)]
    comp = []
    if decompress:
        for b in blocks:
            c = ctypes.create_string_buffer(cap)
            r = lib.LZ4_compress_default(b, c, L, cap)
            comp.append((c, r))

    def work(i):
        if decompress:
            c, r = comp[i]
            return lib.LZ4_decompress_safe(c, outs[i % threads], r, L)
        return lib.LZ4_compress_default(blocks[i], outs[i % threads], L, cap)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(min(threads, len(blocks)))))
        t0 = time.perf_counter()
        list(ex.map(work, range(len(blocks))))
        el = time.perf_counter() - t0
    return {"value": round(len(blocks) * L / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d x 4 MiB blocks, %s of the system liblz4 %d (the LZ4 C library github.com/hungys/go-lz4 "
                      "binds), %d threads (%s)" % (len(blocks), "LZ4_decompress_safe" if decompress else
                                                    "LZ4_compress_default", lib.LZ4_versionNumber(), threads, note)}


def lz4_bench(args, world, rank, local, dist, eng):
    """SURVEY 8f-4 / cachedStore.upload's Compress (cached_store.go:387) and
    load's Decompress (:738): a device-resident batch of 4 MiB blocks through
    the LZ4 stage.  value = uncompressed GB/s."""
    import numpy as np
    from juicefs_amd import engine as E
    nb = args.blocks
    L = args.block_bytes
    base = rank * nb
    bound = int(E.lz4_bound(L))
    src = eng.alloc(nb * L)
    cmp_ = eng.alloc(nb * bound)
    if args.lz4_data == "text":
        pool = _text_pool(16 << 20, SEED + rank)
        for b in range(nb):
            o = ((base + b) * 2654435761) % (pool.size - L)
            src.upload(pool[o:o + L], b * L)
    else:
        eng.gen_synthetic_batch(src, L, [L] * nb, SEED, base)
    carr, n = eng.make_zblocks((src.ptr + b * L, L, cmp_.ptr + b * bound, bound) for b in range(nb))
    eng.lz4_compress_batch(carr, n, E.MEM_DEVICE)
    clens = [carr[b].out_len for b in range(nb)]
    if args.mode == "lz4":
        def step():
            eng.lz4_compress_batch(carr, n, E.MEM_DEVICE)
        algo_bytes = nb * L + sum(clens)
    else:
        out = eng.alloc(nb * L)
        darr, _ = eng.make_zblocks((cmp_.ptr + b * bound, clens[b], out.ptr + b * L, L) for b in range(nb))

        def step():
            eng.lz4_decompress_batch(darr, n, E.MEM_DEVICE)
        algo_bytes = nb * L + sum(clens)
    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.kernel_time(reset=True)
    eng.set_timing(True)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0, local)
    eng.set_timing(False)
    k_ms, k_n = eng.kernel_time(reset=True)
    k_avg = k_ms / max(k_n, 1)
    # spot check against the oracle (checker only)
    verified = 0
    if args.verify:
        from oracle import oracle as orc
        for b in range(0, nb, max(1, nb // args.verify))[:args.verify]:
            p = src.download(L, b * L).tobytes()
            c = cmp_.download(clens[b], b * bound).tobytes()
            if c != orc.lz4_compress(p):
                raise SystemExit("bench: block %d compresses differently from the oracle" % b)
            if args.mode == "unlz4":
                if darr[b].status != E.OK or out.download(L, b * L).tobytes() != p:
                    raise SystemExit("bench: block %d does not decode" % b)
            verified += 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = [src.download(L, b * L).tobytes() for b in range(min(nb, 256))]
        cpu = lz4_cpu_baseline(sample, L, decompress=args.mode == "unlz4")
    if rank == 0:
        print(json.dumps({
            "metric": "LZ4 %s GB/s (uncompressed bytes), 4 MiB blocks" % (
                "compressed" if args.mode == "lz4" else "decompressed"),
            "value": round(world * nb * L * args.steps / el / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (%s), device-resident" % (
                "zipf word text, 4 MiB windows of a 16 MiB pool" if args.lz4_data == "text" else "SplitMix64 blocks"),
            "config": {"workload": "%s GiB device-resident batch of 4 MiB blocks per GPU, LZ4 %s" % (
                round(nb * L / 2**30, 3), "compress" if args.mode == "lz4" else "decompress"),
                "blocks_per_gpu": nb, "block_bytes": L, "mode": args.mode, "data": args.lz4_data,
                "ratio": round(sum(clens) / (nb * L), 4), "parallelism": "block-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "achieved": round(algo_bytes / (k_avg / 1e3) / 1e9, 1) if k_n else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo_bytes / (k_avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if k_n else None,
                         "traffic": pmc_traffic(args, nb * L)[0], "traffic_source": pmc_traffic(args, nb * L)[1],
                         "traffic_note": CODEC_TRAFFIC_NOTE, "binding": pmc_traffic(args, nb * L)[2],
                         "kernel": lz4_kernel_name(args.mode, nb),
                         "kernel_avg_ms": round(k_avg, 3), "algorithmic_bytes_per_launch": algo_bytes,
                         "plain_bytes_per_launch": nb * L},
            "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def lz4_kernel_name(mode, nb, cus=256):
    """The LZ4 kernel a batch of nb blocks runs (launch_lz4_compress: the LDS
    table while the batch fits 16 blocks per CU, JFSX_LZ4_TABLE overrides)."""
    if mode != "lz4":
        return "lz4_decompress_k"
    env = os.environ.get("JFSX_LZ4_TABLE")
    return "lz4_compress_lds_k" if env == "lds" or (env != "global" and nb <= 16 * cus) else "lz4_compress_k"


def zstd_cpu_baseline(frames, L):
    """ZSTD_decompress of the system zstd library (the C library DataDog/zstd
    binds) over the distinct frames, one thread per core."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    from tests import zstd_lib
    z = zstd_lib.lib()
    threads, note = host_cores()
    outs = [ctypes.create_string_buffer(L) for _ in range(threads)]

    def work(i):
        f = frames[i % len(frames)]
        return z.ZSTD_decompress(outs[i % threads], L, f, len(f))
    reps = max(len(frames), 4 * threads)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(threads)))
        t0 = time.perf_counter()
        list(ex.map(work, range(reps)))
        el = time.perf_counter() - t0
    return {"value": round(reps * L / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d x 4 MiB frames (%d distinct), ZSTD_decompress of the system libzstd %d (the C library "
                      "github.com/DataDog/zstd binds), %d threads (%s)" % (reps, len(frames), zstd_lib.version(),
                                                                          threads, note)}


def zstd_bench(args, world, rank, local, dist, eng):
    """SURVEY 8f-4 / cachedStore.load's Decompress (cached_store.go:738) for
    "zstd" volumes: a device-resident batch of level-1 zstd frames of 4 MiB
    blocks (compressed on the host by the system libzstd: 256 distinct blocks,
    repeated over the batch) through jfsx_zstd_decompress_batch.  value =
    decompressed GB/s."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from juicefs_amd import engine as E
    from tests import zstd_lib
    nb = args.blocks
    L = args.block_bytes
    base = rank * nb
    nd = min(nb, 256)
    if args.lz4_data == "text":
        pool = _text_pool(16 << 20, SEED + rank)
        blocks = [pool[(((base + b) * 2654435761) % (pool.size - L)):][:L].tobytes() for b in range(nd)]
    else:
        rng = np.random.default_rng(SEED + rank)
        blocks = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(nd)]
    with ThreadPoolExecutor(16) as ex:
        frames = list(ex.map(lambda b: zstd_lib.compress(b, 1), blocks))
    fcap = max(len(f) for f in frames)
    cmp_ = eng.alloc(nb * fcap)
    for b in range(nb):
        cmp_.upload(np.frombuffer(frames[b % nd], np.uint8), b * fcap)
    out = eng.alloc(nb * L)
    darr, n = eng.make_zblocks((cmp_.ptr + b * fcap, len(frames[b % nd]), out.ptr + b * L, L) for b in range(nb))
    csum = sum(len(frames[b % nd]) for b in range(nb))

    def step():
        eng.zstd_decompress_batch(darr, n, E.MEM_DEVICE)
    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.metrics(reset=True)
    eng.kernel_time(reset=True)
    eng.set_timing(True)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0, local)
    eng.set_timing(False)
    k_ms, k_n = eng.kernel_time(reset=True)
    k_avg = k_ms / max(k_n, 1)
    serial = eng.metrics()["zstd_serial"]
    verified = 0
    if args.verify:
        for b in range(0, nb, max(1, nb // args.verify))[:args.verify]:
            if darr[b].status != E.OK or out.download(L, b * L).tobytes() != blocks[b % nd]:
                raise SystemExit("bench: zstd block %d does not decode" % b)
            verified += 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = zstd_cpu_baseline(frames, L)
    algo_bytes = nb * L + csum
    if rank == 0:
        print(json.dumps({
            "metric": "zstd decompressed GB/s (uncompressed bytes), 4 MiB blocks",
            "value": round(world * nb * L * args.steps / el / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (%s), level-1 frames from the system libzstd %d, device-resident" % (
                "zipf word text, 4 MiB windows of a 16 MiB pool" if args.lz4_data == "text" else "random bytes",
                zstd_lib.version()),
            "config": {"workload": "%s GiB device-resident batch of 4 MiB blocks per GPU, zstd decompress" % (
                round(nb * L / 2**30, 3)), "blocks_per_gpu": nb, "block_bytes": L, "mode": args.mode,
                "data": args.lz4_data, "ratio": round(csum / (nb * L), 4),
                "parallelism": "block-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "achieved": round(algo_bytes / (k_avg / 1e3) / 1e9, 1) if k_n else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo_bytes / (k_avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if k_n else None,
                         "traffic": pmc_traffic(args, nb * L)[0], "traffic_source": pmc_traffic(args, nb * L)[1],
                         "traffic_note": CODEC_TRAFFIC_NOTE, "binding": pmc_traffic(args, nb * L)[2],
                         "kernel": "zstd_decompress_k" if os.environ.get("JFSX_ZSTD_SERIAL") == "1"
                         else "zstd_decompress_par_k", "kernel_avg_ms": round(k_avg, 3),
                         "objects_to_serial_decoder": serial,
                         "algorithmic_bytes_per_launch": algo_bytes, "plain_bytes_per_launch": nb * L},
            "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def zstdc_cpu_baseline(blocks, L):
    """ZSTD_compress(level 1) of the system zstd library (the call
    zstd.CompressLevel makes) over the sample blocks, one thread per core."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    from tests import zstd_lib
    z = zstd_lib.lib()
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    threads, note = host_cores()
    cap = z.ZSTD_compressBound(L)
    outs = [ctypes.create_string_buffer(cap) for _ in range(threads)]

    def work(i):
        return z.ZSTD_compress(outs[i % threads], cap, blocks[i % len(blocks)], L, 1)
    reps = max(len(blocks), 4 * threads)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(threads)))
        t0 = time.perf_counter()
        list(ex.map(work, range(reps)))
        el = time.perf_counter() - t0
    return {"value": round(reps * L / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d x 4 MiB blocks (%d distinct), ZSTD_compress level 1 of the system libzstd %d (the C "
                      "library github.com/DataDog/zstd binds), %d threads (%s)" % (reps, len(blocks),
                                                                                  zstd_lib.version(), threads, note)}


def zstdc_bench(args, world, rank, local, dist, eng):
    """SURVEY 8f-4 / cachedStore.upload's Compress (cached_store.go:387) for
    "zstd" volumes: a device-resident batch of 4 MiB blocks through
    jfsx_zstd_compress_batch (zstd.CompressLevel(dst, src, 1) per block).
    value = uncompressed GB/s."""
    import numpy as np
    from juicefs_amd import engine as E
    from tests import zstd_lib
    nb, L = args.blocks, args.block_bytes
    base = rank * nb
    bound = int(E.zstd_bound(L))
    src = eng.alloc(nb * L)
    if args.lz4_data == "text":
        pool = _text_pool(16 << 20, SEED + rank)
        for b in range(nb):
            o = ((base + b) * 2654435761) % (pool.size - L)
            src.upload(pool[o:o + L], b * L)
    else:
        eng.gen_synthetic_batch(src, L, [L] * nb, SEED, base)
    cmp_ = eng.alloc(nb * bound)
    arr, n = eng.make_zblocks((src.ptr + b * L, L, cmp_.ptr + b * bound, bound) for b in range(nb))

    def step():
        eng.zstd_compress_batch(arr, n, E.MEM_DEVICE)
    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.kernel_time(reset=True)
    eng.set_timing(True)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0, local)
    eng.set_timing(False)
    k_ms, k_n = eng.kernel_time(reset=True)
    k_avg = k_ms / max(k_n, 1)
    clens = [arr[b].out_len for b in range(nb)]
    verified = 0
    if args.verify:
        for b in range(0, nb, max(1, nb // args.verify))[:args.verify]:
            p = src.download(L, b * L).tobytes()
            if arr[b].status != E.OK or cmp_.download(clens[b], b * bound).tobytes() != zstd_lib.compress_simple(p, 1):
                raise SystemExit("bench: block %d compresses differently from libzstd level 1" % b)
            verified += 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = [src.download(L, b * L).tobytes() for b in range(min(nb, 64))]
        cpu = zstdc_cpu_baseline(sample, L)
    algo_bytes = nb * L + sum(clens)
    if rank == 0:
        print(json.dumps({
            "metric": "zstd level-1 compressed GB/s (uncompressed bytes), 4 MiB blocks",
            "value": round(world * nb * L * args.steps / el / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (%s), device-resident" % (
                "zipf word text, 4 MiB windows of a 16 MiB pool" if args.lz4_data == "text" else "SplitMix64 blocks"),
            "config": {"workload": "%s GiB device-resident batch of 4 MiB blocks per GPU, zstd level-1 compress" % (
                round(nb * L / 2**30, 3)), "blocks_per_gpu": nb, "block_bytes": L, "mode": args.mode,
                "data": args.lz4_data, "ratio": round(sum(clens) / (nb * L), 4),
                "parallelism": "block-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "achieved": round(algo_bytes / (k_avg / 1e3) / 1e9, 1) if k_n else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo_bytes / (k_avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if k_n else None,
                         "traffic": pmc_traffic(args, nb * L)[0], "traffic_source": pmc_traffic(args, nb * L)[1],
                         "traffic_note": CODEC_TRAFFIC_NOTE, "binding": pmc_traffic(args, nb * L)[2],
                         "kernel": "zstd_compress_k", "kernel_avg_ms": round(k_avg, 3),
                         "algorithmic_bytes_per_launch": algo_bytes, "plain_bytes_per_launch": nb * L},
            "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
