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
