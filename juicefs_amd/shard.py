"""Multi-GPU layout: one process per GPU, blocks sharded by rank.

Every block has its own key and nonce, and its tag and CRCs depend only on
that block.  So blocks shard across GPUs with no data-path collective
(SURVEY.md 8e).  The only collectives are the timing barrier and the
max-over-ranks reduction that bench.py reports.  RCCL ("nccl") is used on
GPUs and gloo on CPU.
"""
import os


def dist_env():
    """(world, rank, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None):
    """Initialise the process group when WORLD_SIZE > 1; returns the dist
    module or None."""
    world, _, local = dist_env()
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend)
    return dist


def shard(blocks_per_rank, rank):
    """Global block indices of a rank under weak scaling: [rank*B, (rank+1)*B)."""
    return range(rank * blocks_per_rank, (rank + 1) * blocks_per_rank)


def shard_strong(total_blocks, rank, world):
    """Contiguous near-equal split of a fixed total (strong scaling)."""
    lo = rank * total_blocks // world
    hi = (rank + 1) * total_blocks // world
    return range(lo, hi)


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x, local=0):
    if dist is None:
        return x
    import torch
    dev = "cpu"
    if dist.get_backend() == "nccl":
        dev = "cuda:%d" % local
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x, local=0):
    """Sum of x over the ranks (the whole job's blocks under strong scaling)."""
    if dist is None:
        return x
    import torch
    dev = "cpu"
    if dist.get_backend() == "nccl":
        dev = "cuda:%d" % local
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
