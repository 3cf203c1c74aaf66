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
    ap.add_argument("--agg-window-us", type=int, default=500, help="agg: aggregation window")
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


def cpu_baseline(args, mode="seal", lens=None):
    """The reference's per-block CPU work, one worker per core, timed on this
    host over a bounded sample of the same workload (about --cpu-seconds):
      seal  checksum() + aead.Seal            (encrypt.go:192, disk_cache.go:1218-1231)
      open  aead.Open + the ReadAt CRC verify (encrypt.go:215, disk_cache.go:1315-1327)
      crc   the ReadAt CRC verify alone       (a cache hit)
    The AEAD runs through OpenSSL EVP (AES-NI/VAES + VPCLMULQDQ stitched GCM,
    SIMD ChaCha20-Poly1305: the class of Go's assembly), the
    CRC32C as 3-stream SSE4.2 like Go's castagnoliSSE42Triple.  lens: the
    bench's own ragged lengths (configs[4]); else 4 MiB blocks."""
    from oracle import oracle as orc
    threads, note = host_cores()
    algo = orc.AES256GCM if args.algo == "aes256gcm" else orc.CHACHA20P1305
    bmode = {"seal": orc.BASE_SEAL, "open": orc.BASE_OPEN, "crc": orc.BASE_CRC}[mode]
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
            "crc": "CRC32C verify against the stored CRCs (3-stream SSE4.2)"}[mode]
    blocks = ("%d ragged blocks (the bench's own lengths, %.3f GiB)" % (nblk, nbytes / 2**30) if sample
              else "1 GiB (256 x 4 MiB blocks)")
    return {"value": round(reps * nbytes / total_s / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d x %s %s, %d threads (%s), %s" % (reps, blocks, what, threads, note, cpu_model())}


def dry_run(args, world, rank, local, dist):
    """No engine: exercises the rank launch, the shard layout, the barrier and
    the max-over-ranks timing the real bench uses (tests/test_dist_gloo.py)."""
    from juicefs_amd import shard
    blocks = shard.shard(args.blocks, rank)
    barrier(dist)
    t0 = time.perf_counter()
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0 + 0.001 * rank, local)
    first = max_over_ranks(dist, float(blocks[0]), local)
    if rank == 0:
        print(json.dumps({"metric": "dry run (no engine)", "value": None, "unit": "GB/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3),
                          "dry_run": True, "last_rank_first_block": int(first),
                          "config": {"blocks_per_gpu": args.blocks,
                                     "parallelism": "block-sharded x%d, no collective" % world}}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local, dist = dist_setup(args)
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.dry_run:
        return dry_run(args, world, rank, local, dist)
    from juicefs_amd import engine as E

    eng = E.Engine(local, E.CTX_BITSLICE if args.aes == "bitslice" else 0)
    if args.mode == "agg":
        return agg_bench(args, world, rank, local, dist, eng)
    if args.mode == "aggcodec":
        return aggcodec_bench(args, world, rank, local, dist, eng)
    if args.mode in ("lz4", "unlz4"):
        return lz4_bench(args, world, rank, local, dist, eng)
    if args.mode == "unzstd":
        return zstd_bench(args, world, rank, local, dist, eng)
    if args.mode == "zstd":
        return zstdc_bench(args, world, rank, local, dist, eng)
    if args.mem == "host":
        return host_ingest(args, world, rank, local, dist, eng)
    nb, L = args.blocks, args.block_bytes
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    nseg = -(-L // E.SEG)
    src = eng.alloc(nb * L)
    dst = eng.alloc(nb * L) if args.mode != "crc" else None
    crc = eng.alloc(nb * 4 * nseg)
    base = rank * nb  # global block index: blocks shard across ranks (juicefs_amd.shard.shard)
    # block b occupies slot [b*L, b*L + lens[b]); ragged lengths are a seeded
    # draw per global block index, so every rank and rerun sees the same batch
    lens = [ragged_len(SEED, base + b, L) if args.ragged else (args.fixed_len or L) for b in range(nb)]
    if args.ragged and args.ragged_align:
        lens = [min(L, -(-x // args.ragged_align) * args.ragged_align) for x in lens]
    if args.packed:
        offs, o = [], 0
        for x in lens:
            offs.append(o)
            o += -(-x // 256) * 256
        for b in range(nb):
            eng.gen_synthetic_batch(src, L, [lens[b]], SEED, base + b, offset=offs[b])
    else:
        offs = [b * L for b in range(nb)]
        eng.gen_synthetic_batch(src, L, lens, SEED, base)  # one launch for the whole batch

    if args.mode == "crc":
        ranges = (E.jfsx_range * nb)()
        for b in range(nb):
            ranges[b].data, ranges[b].len, ranges[b].crc = src.ptr + offs[b], lens[b], crc.ptr + 4 * nseg * b
        eng.crc32c_segments(ranges, nb, E.CRC_GEN, E.MEM_DEVICE)

        def step():
            eng.crc32c_segments(ranges, nb, E.CRC_VERIFY, E.MEM_DEVICE)
        algo_bytes = sum(lb + 4 * -(-lb // E.SEG) for lb in lens)
    else:
        specs = []
        for b in range(nb):
            key, nonce = E.gen_key(SEED, base + b)
            specs.append({"key": key, "nonce": nonce, "src": src.ptr + offs[b], "dst": dst.ptr + offs[b], "len": lens[b],
                          "crc": crc.ptr + 4 * nseg * b})
        blks, n = eng.make_blocks(specs)
        if args.mode == "seal":
            def step():
                eng.seal_batch(algo, blks, n, E.CRC_GEN if args.crc == "full" else E.CRC_NONE, E.MEM_DEVICE)
        else:
            # Open + CRC verify (BASELINE configs[3]): make a sealed image first
            eng.seal_batch(algo, blks, n, E.CRC_GEN, E.MEM_DEVICE)
            oblks, _ = eng.make_blocks([dict(s, src=s["dst"], dst=s["src"], tag=bytes(blks[i].tag))
                                        for i, s in enumerate(specs)])
            if args.mode == "open":
                def step():
                    eng.open_batch(algo, oblks, n, E.CRC_VERIFY, E.MEM_DEVICE)
            else:
                # Decrypt end to end: every object's key arrives RSA-OAEP
                # wrapped (encrypt.go:196-216); each step unwraps all n keys on
                # the GPU straight into the descriptors, then opens
                import ctypes
                import numpy as np
                from juicefs_amd import encrypt as enc
                rsae = enc.NewRSAEncryptor(enc.GenerateRsaKey(2048))
                dkey = eng.rsa_key(*enc.rsa_crt_components(rsae.privKey))
                wrapped = np.frombuffer(b"".join(rsae.Encrypt(bytes(specs[i]["key"])) for i in range(n)), np.uint8)
                wlen = np.full(n, 256, np.uint32)
                mlen = np.zeros(n, np.int32)
                for i in range(n):
                    ctypes.memset(ctypes.addressof(oblks[i]) + E.jfsx_blk.key.offset, 0, 32)

                def step():
                    eng._check(eng.L.jfsx_rsa_oaep_decrypt_batch(
                        eng.ctx, dkey, n, wrapped.ctypes.data, 256, wlen.ctypes.data,
                        ctypes.addressof(oblks[0]) + E.jfsx_blk.key.offset, ctypes.sizeof(E.jfsx_blk),
                        mlen.ctypes.data), "unwrap")
                    eng.open_batch(algo, oblks, n, E.CRC_VERIFY, E.MEM_DEVICE)
        algo_bytes = sum(2 * lb + 16 + 4 * -(-lb // E.SEG) + 44 for lb in lens)

    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.kernel_time(reset=True)
    eng.set_timing(True)
    barrier(dist)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    barrier(dist)
    t1 = time.perf_counter()
    eng.set_timing(False)
    el = max_over_ranks(dist, t1 - t0, local)
    k_ms, k_n = eng.kernel_time(reset=True)
    k_avg_ms = k_ms / max(k_n, 1)

    # post-timing spot check of a few blocks against the oracle (checker only)
    verified = 0
    if args.mode in ("open", "decrypt"):
        bad = [i for i in range(nb) if oblks[i].status != E.OK]
        if args.mode == "decrypt":
            bad += [i for i in range(nb) if mlen[i] != 32 or bytes(oblks[i].key) != bytes(specs[i]["key"])]
        if bad:
            raise SystemExit("bench: %d blocks failed to open (first %d)" % (len(bad), bad[0]))
        verified = nb
    rsa = None
    if args.mode == "decrypt":
        # the unwrap alone (GPU batch) beside the reference's host path
        # (libcrypto RSA-OAEP, one thread) on a bounded sample
        t = time.perf_counter()
        eng._check(eng.L.jfsx_rsa_oaep_decrypt_batch(eng.ctx, dkey, n, wrapped.ctypes.data, 256, wlen.ctypes.data,
                                                     None, 0, mlen.ctypes.data), "unwrap")
        gpu_s = time.perf_counter() - t
        sample = [bytes(wrapped[256 * i:256 * i + 256]) for i in range(min(n, 200))]
        t = time.perf_counter()
        for w in sample:
            rsae.Decrypt(w)
        host_s = (time.perf_counter() - t) / len(sample)
        rsa = {"unwraps": n, "gpu_ms_per_batch": round(gpu_s * 1e3, 3), "gpu_unwraps_per_s": round(n / gpu_s),
               "host_us_per_unwrap_1thread": round(host_s * 1e6, 1),
               "host_sample": "%d libcrypto RSA-OAEP decrypts, 1 thread" % len(sample)}
        eng.rsa_key_free(dkey)
    full = None
    if args.verify and args.mode in ("seal", "open", "crc") and (args.crc == "full" or args.mode != "seal"):
        # every block's tag and CRC array against the oracle (host cores)
        full = full_check(args, E, blks if args.mode != "crc" else None,
                          crc.download(nb * 4 * nseg).reshape(nb, 4 * nseg), lens, base)
    if args.verify and args.mode == "seal":
        # and the ciphertext bytes of a few blocks
        from oracle import oracle as orc
        for b in range(0, nb, max(1, nb // args.verify))[:args.verify]:
            p = orc.gen_block(SEED, base + b, lens[b])
            key, nonce = orc.gen_key(SEED, base + b)
            c, tag = orc.seal(orc.AES256GCM if algo == E.AES256GCM else orc.CHACHA20P1305, key, nonce, p,
                              fast=algo == E.AES256GCM)
            if bytes(blks[b].tag) != tag or dst.download(lens[b], offset=offs[b]).tobytes() != c:
                raise SystemExit("bench: block %d differs from the oracle" % b)
    if full:
        verified = nb

    total_plain = world * sum(lens) * args.steps
    value = total_plain / el / 1e9
    achieved = algo_bytes / (k_avg_ms / 1e3) / 1e9 if k_n else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, "open" if args.mode in ("open", "decrypt") else args.mode,
                           lens if args.ragged else None)
        if args.mode == "decrypt" and rsa:
            # each object also pays one RSA-OAEP private-key unwrap on the host
            # (encrypt.go:207-210): per thread, block time + unwrap time
            per_block = cpu["cores"] * BLOCK / (cpu["value"] * 1e9)
            cpu["value"] = round(cpu["cores"] * BLOCK / (per_block + rsa["host_us_per_unwrap_1thread"] * 1e-6) / 1e9, 3)
            cpu["sample"] += "; plus one libcrypto RSA-OAEP unwrap per block (%.1f us, measured on 1 thread)" % (
                rsa["host_us_per_unwrap_1thread"])
    traffic, traffic_src, binding = pmc_traffic(args, sum(lens))
    if rank == 0:
        line = {
            "metric": ("sealed+checksummed GB/s, %s" if args.mode == "seal" else
                       ("opened+verified GB/s, %s" if args.mode == "open" else
                        ("decrypted (RSA unwrap + open + verify) GB/s, %s" if args.mode == "decrypt" else
                         "CRC32C-verified GB/s, %s"))) % (
                          "ragged 64 KiB-4 MiB blocks" if args.ragged else "4 MiB blocks"),
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64 blocks, "
            "per-block SplitMix64 keys/nonces), device-resident",
            "config": {"workload": "%s GiB device-resident batch of %s blocks per GPU, %s %s + CRC32C %s" % (
                round(sum(lens) / 2**30, 3), "ragged 64 KiB-4 MiB" if args.ragged else "4 MiB", args.algo, args.mode,
                "full" if args.mode == "seal" else "verify"),
                "blocks_per_gpu": nb, "block_bytes": "ragged" if args.ragged else L, "algo": args.algo,
                "mode": args.mode, "aes_kernel": args.aes if args.algo == "aes256gcm" and args.mode != "crc" else None,
                "parallelism": "block-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": ("crc_segments_k" if args.mode == "crc" else
                                    ("gcm_main_k" if args.algo == "aes256gcm" else "cp_main_k")),
                         "kernel_avg_ms": round(k_avg_ms, 3), "algorithmic_bytes_per_launch": algo_bytes,
                         "plain_bytes_per_launch": sum(lens), "binding": binding},
            "cpu_baseline": cpu,
            "verified_blocks": verified,
            "full_check": full,
            **({"rsa_unwrap": rsa} if rsa else {}),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


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
PMC_FILES = ("r4/pmc_r4.json", "r3/pmc_r3.json")
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


def pcie_probe(eng, nbytes=1 << 30):
    """jfsx_pcie_probe: GB/s between engine-pinned host memory and HBM on the
    ring's own H2D and D2H streams, each direction alone and both at once
    (8 chunks per direction issued alternately, as the ring issues them)."""
    return eng.pcie_probe(nbytes)


def host_ingest(args, world, rank, local, dist, eng):
    """BASELINE configs[2]: blocks in pinned host memory, sealed through the
    engine's H2D | transform | D2H ring (JFSX_MEM_HOST); value = plaintext
    bytes / s including both PCIe transfers."""
    import ctypes
    import numpy as np
    from juicefs_amd import engine as E
    nb, L = args.blocks, args.block_bytes
    nseg = -(-L // E.SEG)
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    pcie_before = pcie_probe(eng)
    hin = eng.alloc_pinned(nb * L)
    hout = eng.alloc_pinned(nb * L)
    hcrc = eng.alloc_pinned(nb * 4 * nseg)
    tmp = eng.alloc(L)
    base = rank * nb
    for b in range(nb):  # synthetic input: generated on device, copied once into pinned memory
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

    def step():
        eng.seal_batch(algo, blks, n, E.CRC_GEN, E.MEM_HOST)
    for _ in range(args.warmup):
        step()
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
    # the link probed again right after the ring (the probe before it has read
    # below what the ring itself moved on some boxes); the faster of the two
    pcie_after = pcie_probe(eng)
    pcie = {k: max(pcie_before.get(k, 0.0), pcie_after.get(k, 0.0)) for k in set(pcie_before) | set(pcie_after)}
    pcie_runs = {"before_ring": pcie_before, "after_ring": pcie_after}
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
            verified += 1
    full = None
    if args.verify:
        crcs = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * 4 * nseg)).from_address(hcrc)).reshape(nb, 4 * nseg)
        full = full_check(args, E, blks, crcs.copy(), [L] * nb, base)
        verified = nb
    value = world * nb * L * args.steps / el / 1e9
    cpu = cpu_baseline(args, "seal") if rank == 0 and world == 1 and not args.no_cpu else None
    plain_launch = int(nb * L * args.steps / max(k_n, 1))
    traffic, traffic_src, binding = pmc_traffic(args, plain_launch)
    if rank == 0:
        # the ring moves equal bytes both ways at once: its bound is the
        # slower direction of the simultaneous (duplex) probe
        peak = min(pcie.get("duplex_h2d", pcie["h2d"]), pcie.get("duplex_d2h", pcie["d2h"]))
        print(json.dumps({
            "metric": "sealed+checksummed GB/s, 4 MiB blocks (host ingest)", "value": round(value, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), pinned host memory",
            "config": {"workload": "host-ingest: %s GiB pinned per step x %d steps per GPU, %s seal + CRC32C full, "
                                   "3-slot H2D|transform|D2H ring" % (nb * L / 2**30, args.steps, args.algo),
                       "blocks_per_gpu": nb, "block_bytes": L, "algo": args.algo, "mem": "host"},
            "roofline": {"bound": "pcie", "achieved": round(value, 2), "peak": peak, "unit": "GB/s",
                         "frac": round(value / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_note": "HBM bytes per launch of gcm_main_k (one launch per ring slot)",
                         "peak_basis": "min over directions of simultaneous H2D + D2H copies of 1 GiB on the "
                                       "ring's streams (jfsx_pcie_probe, the better of a probe before and one after "
                                       "the ring); one-way rates in pcie_measured",
                         "frac_of_one_way_d2h": round(value / pcie["d2h"], 4),
                         "pcie_measured": pcie, "pcie_probes": pcie_runs,
                         "kernel_avg_ms": round(k_ms / max(k_n, 1), 3),
                         "kernel_launches": k_n, "plain_bytes_per_launch": plain_launch, "binding": binding},
            "cpu_baseline": cpu, "verified_blocks": verified, "full_check": full}), flush=True)
    eng.free_pinned(hin)
    eng.free_pinned(hout)
    eng.free_pinned(hcrc)
    eng.close()
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
    nb, L = min(args.blocks, 1024), args.block_bytes
    nseg = -(-L // E.SEG)
    algo = E.AES256GCM if args.algo == "aes256gcm" else E.CHACHA20P1305
    hin, hout, hcrc = eng.alloc_pinned(nb * L), eng.alloc_pinned(nb * L), eng.alloc_pinned(nb * 4 * nseg)
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
        eng._check(eng.L.jfsx_seal_batch(eng.ctx, algo, 1, ctypes.byref(blks[b]), E.CRC_GEN, E.MEM_HOST), "seal")

    d_steps = max(1, args.steps // 5)
    run(direct, 1)
    d_el = run(direct, d_steps)
    with E.Aggregator(eng, window_us=args.agg_window_us) as agg:
        def through(b):
            agg.seal(algo, blks[b], E.CRC_GEN, E.MEM_HOST)
        run(through, args.warmup)
        c0, b0, k0 = agg.stats()
        barrier(dist)
        el = max_over_ranks(dist, run(through, args.steps), local)
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
            verified += 1
    value = world * nb * L * args.steps / el / 1e9
    cpu = cpu_baseline(args, "seal") if rank == 0 and world == 1 and not args.no_cpu else None
    if rank == 0:
        print(json.dumps({
            "metric": "per-object sealed+checksummed GB/s, %d threads, 4 MiB host blocks (aggregator)" % T,
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), pinned host memory",
            "config": {"workload": "%d one-block Seal calls per step from %d threads, %s + CRC32C full, JFSX_MEM_HOST"
                                   % (nb, T, args.algo), "blocks_per_gpu": nb, "block_bytes": L, "algo": args.algo,
                       "mode": "agg", "window_us": args.agg_window_us},
            "aggregator": {"calls": c1 - c0, "batches": b1 - b0,
                           "mean_batch_blocks": round((k1 - k0) / max(b1 - b0, 1), 2)},
            "direct_one_block_calls_GBs": round(nb * L * d_steps / d_el / 1e9, 2),
            "roofline": None, "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    for h in (hin, hout, hcrc):
        eng.free_pinned(h)
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
                         "kernel": "lz4_compress_k" if args.mode == "lz4" else "lz4_decompress_k",
                         "kernel_avg_ms": round(k_avg, 3), "algorithmic_bytes_per_launch": algo_bytes,
                         "plain_bytes_per_launch": nb * L},
            "cpu_baseline": cpu, "verified_blocks": verified}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


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
