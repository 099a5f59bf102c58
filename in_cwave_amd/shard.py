"""Stream sharding across the GPUs of one node.

Streams are independent, so the batch axis is split into contiguous ranges, one per rank
(one process per GPU); there is no collective on the data path.  The only collectives are the
optional end-of-job ones: gathering rendered PCM to rank 0 and reducing the meters.  With the
"nccl" backend torch.distributed runs RCCL over xGMI on MI355X; tests use "gloo" on CPU.
"""
import numpy as np


def shard_range(n_total, rank, world):
    """contiguous [first, first+count) of rank; the first n_total % world ranks get one more"""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def gather_pcm(dist, local, n_total, rank, world, device=None):
    """all-gather equal-width rows [count, bytes] of uint8 PCM to every rank -> [n_total, bytes]"""
    import torch
    counts = [shard_range(n_total, r, world)[1] for r in range(world)]
    width = local.shape[1]
    mx = max(counts)
    t = torch.zeros((mx, width), dtype=torch.uint8, device=device)
    t[: local.shape[0]] = torch.as_tensor(np.ascontiguousarray(local), device=device)
    bufs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    return np.concatenate([b[:c].cpu().numpy() for b, c in zip(bufs, counts)], axis=0)


def reduce_meters(dist, clips, peak_db, desubnorm, device=None):
    """global meters as the reference keeps them in `am` (adv_modulator.c:54-56): clip counters
    summed, peaks max-reduced, de-subnorm counters summed"""
    import torch
    c = torch.tensor(np.asarray(clips, dtype=np.int64).reshape(-1), device=device)
    p = torch.tensor(np.asarray(peak_db, dtype=np.float64).reshape(-1), device=device)
    d = torch.tensor([int(desubnorm)], dtype=torch.int64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    dist.all_reduce(p, op=dist.ReduceOp.MAX)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    return c.cpu().numpy(), p.cpu().numpy(), int(d.item())
