"""world_size-2 gloo run of the multi-GPU layout (juicefs_amd.shard): each rank
seals its own shard of blocks (oracle stands in for the engine on CPU), the
timing reduction is the max over ranks, and the union of the shards equals the
single-process result."""
import json
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from juicefs_amd import shard
    from oracle import oracle as orc
    dist = shard.init("gloo")
    res = {}
    for b in shard.shard(3, rank):
        key, nonce = orc.gen_key(99, b)
        c, tag = orc.seal(orc.AES256GCM, key, nonce, orc.gen_block(99, b, 40000 + b))
        res[b] = tag.hex()
    shard.barrier(dist)
    t = shard.max_over_ranks(dist, 1.0 + rank)
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        with open(os.path.join(outdir, "out.json"), "w") as f:
            json.dump({"t": t, "tags": merged}, f)
    dist.destroy_process_group()


def test_two_rank_sharding(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    out = json.load(open(os.path.join(str(tmp_path), "out.json")))
    assert out["t"] == 2.0  # max over ranks
    from oracle import oracle as orc
    assert sorted(int(k) for k in out["tags"]) == list(range(6))
    for b in range(6):
        key, nonce = orc.gen_key(99, b)
        _, tag = orc.seal(orc.AES256GCM, key, nonce, orc.gen_block(99, b, 40000 + b))
        assert out["tags"][str(b)] == tag.hex()


def test_strong_split_covers_all():
    from juicefs_amd import shard
    for total in (1, 7, 16384):
        for world in (1, 2, 4, 8):
            got = [i for r in range(world) for i in shard.shard_strong(total, r, world)]
            assert got == list(range(total))


def test_bench_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` with no torch.distributed.run environment
    starts the launcher itself (two ranks, gloo on CPU here); rank 0 prints one
    line with n_gpus 2 and the max over ranks of the timing."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--blocks", "5", "--cpu-seconds", "0.2"], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    assert rec["last_rank_first_block"] == 5  # rank 1 owns blocks [5, 10)
    assert rec["ms_per_step"] >= 1.0  # rank 1's extra 1 ms: the max over ranks is reported
    # the CPU leg at N > 1: rank 0 times the baseline after the timed region
    cpu = rec["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port" and cpu["core_s_per_GB"] > 0


def _bench_dry(args):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--no-cpu"] + args, env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_strong_split_two_ranks():
    """configs[3] as BASELINE states it: a fixed 2 TiB scan split across the
    GPUs (--total-gib 2048).  At world 2 (gloo) the ranks' shards are
    contiguous, disjoint and cover all 524,288 blocks; each rank loops 16x over
    its 16,384-block resident batch; the line says "strong"."""
    rec = _bench_dry(["--gpus", "2", "--total-gib", "2048", "--mode", "open"])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["blocks_total"] == 524288 and rec["block_range"] == [0, 524288]
    assert rec["per_gpu_blocks_max"] == 262144 and rec["last_rank_first_block"] == 262144
    assert rec["resident_blocks"] == 16384 and rec["loops_per_step"] == 16
    # an uneven split: 3 ranks would not divide 1000 blocks, 2 do; odd totals still cover every block
    rec = _bench_dry(["--gpus", "2", "--total-gib", str(1001 * 4 / 1024), "--blocks", "300"])
    assert rec["blocks_total"] == 1001 and rec["per_gpu_blocks_max"] == 501
    assert rec["resident_blocks"] == 300 and rec["loops_per_step"] == 2


def test_bench_host_pool_is_capped():
    """Host ingest pins at most --host-pool-gib per GPU (twice: in and out) and
    loops over it: 64 GiB per GPU through an 8 GiB pool is 8 passes."""
    rec = _bench_dry(["--mem", "host", "--blocks", "16384", "--host-pool-gib", "8"])
    assert rec["resident_blocks"] == 2048 and rec["loops_per_step"] == 8
    rec = _bench_dry(["--gpus", "2", "--mem", "host", "--total-gib", "256", "--host-pool-gib", "8"])
    assert rec["blocks_total"] == 65536 and rec["resident_blocks"] == 2048 and rec["loops_per_step"] == 16


def test_bench_host_pool_cap_holds_at_eight_ranks():
    """The 8-GPU node's host ingest (gloo stand-in for the 8 ranks): each rank
    pins at most the cap (--host-pool-gib in and out, plus CRC arrays) while
    the ranks together cover the whole strong total."""
    cap = 8
    rec = _bench_dry(["--gpus", "8", "--mem", "host", "--total-gib", "2048", "--host-pool-gib", str(cap)])
    assert rec["n_gpus"] == 8 and rec["blocks_total"] == 524288 and rec["block_range"] == [0, 524288]
    assert rec["per_gpu_blocks_max"] == 65536 and rec["resident_blocks"] == 2048
    assert rec["pinned_bytes_per_rank_max"] <= 2 * cap * 2**30 + 2048 * 512
    assert rec["pinned_bytes_per_rank_max"] >= 2 * cap * 2**30

