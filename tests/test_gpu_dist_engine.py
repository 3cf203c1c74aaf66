"""The multi-GPU bench's per-rank sequence on one GPU: torch initialises the
device and an RCCL ("nccl") process group, then the engine (libjfsx.so, its
own HIP calls in the same process) seals a batch checked against the oracle,
and the timing collectives (barrier, all_reduce MAX on a device tensor) run
around it -- what each rank of `bench.py --gpus N` does (juicefs_amd/shard.py)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_engine_inside_an_rccl_process_group(monkeypatch):
    import torch
    import torch.distributed as dist
    from juicefs_amd import engine as E
    from juicefs_amd import shard
    from oracle import oracle as orc
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", world_size=1, rank=0)
    try:
        shard.barrier(dist)
        eng = E.Engine(0)
        try:
            n, L = 4, (1 << 20) + 5
            src, dst = eng.alloc(n * (L + 11)), eng.alloc(n * (L + 11))
            crc = eng.alloc(n * 4 * 33)
            specs = []
            for b in range(n):
                p = orc.gen_block(7, b, L)
                src.upload(p, b * (L + 11))
                key, nonce = orc.gen_key(7, b)
                specs.append({"key": key, "nonce": nonce, "src": src.ptr + b * (L + 11),
                              "dst": dst.ptr + b * (L + 11), "len": L, "crc": crc.ptr + 4 * 33 * b})
            blks, m = eng.make_blocks(specs)
            eng.seal_batch(E.AES256GCM, blks, m, E.CRC_GEN, E.MEM_DEVICE)
            for b in range(n):
                p = orc.gen_block(7, b, L)
                key, nonce = orc.gen_key(7, b)
                c, tag = orc.seal(orc.AES256GCM, key, nonce, p, fast=True)
                assert bytes(blks[b].tag) == tag
                assert dst.download(L, b * (L + 11)).tobytes() == c
                assert crc.download(4 * 33, 4 * 33 * b).tobytes() == orc.checksum(p, hw=True)
        finally:
            eng.close()
        assert shard.max_over_ranks(dist, 1.5, 0) == 1.5
        t = torch.ones(1024, device="cuda:0")
        dist.all_reduce(t)
        assert float(t.sum().item()) == 1024.0
    finally:
        dist.destroy_process_group()
