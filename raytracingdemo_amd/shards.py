"""Row-interleaved image shards for the one-process-per-GPU driver.

Image row j is rendered by rank j mod world (interleaving
balances the depth-complexity gradient of a frame).  Every rank holds
`rows_per_rank(H, world)` rows (the last one padding where H % world != 0), so
the shards gather with one equal-sized collective; rank 0 de-interleaves.
"""
from __future__ import annotations


def rows_per_rank(H: int, world: int) -> int:
    return (H + world - 1) // world


def shard_rows(rank: int, world: int, H: int) -> range:
    """Image rows of `rank`'s shard, in shard order (row r of the shard is image row rank + r*world)."""
    return range(rank, H, world)


def deinterleave(gathered, H: int):
    """Full images from gathered shards.

    gathered: tensor [world, F, rows, W, ...] (shard k from rank k, rows =
    rows_per_rank(H, world)).  Returns [F, H, W, ...] with image row
    j = r*world + k taken from shard k, row r; padding rows are dropped.
    """
    world, F, rows = gathered.shape[0], gathered.shape[1], gathered.shape[2]
    rest = tuple(gathered.shape[3:])
    nd = gathered.dim()
    perm = (1, 2, 0) + tuple(range(3, nd))
    full = gathered.permute(*perm).reshape((F, rows * world) + rest)
    return full[:, :H]


def deinterleave_into(gathered, H: int, out):
    """deinterleave() written into `out` ([F, H, W, ...]) with one copy kernel
    (no temporary when the shards have no padding rows)."""
    world, F, rows = gathered.shape[0], gathered.shape[1], gathered.shape[2]
    rest = tuple(gathered.shape[3:])
    if rows * world == H:
        perm = (1, 2, 0) + tuple(range(3, gathered.dim()))
        out.view((F, rows, world) + rest).copy_(gathered.permute(*perm))
    else:
        out.copy_(deinterleave(gathered, H))
    return out


def gather_frames(shard, H: int, world: int, rank: int, dst: int = 0, out=None):
    """Gather every rank's [F, rows, W, ...] shard to `dst` and de-interleave there.

    The shards land in one [world, F, rows, W, ...] buffer (`out`, allocated
    once by the caller, or here) through views of it, so the collective writes
    straight into the layout `deinterleave` reads: one copy in all.  Returns
    [F, H, W, ...] on `dst`, None elsewhere.
    """
    import torch.distributed as dist
    if rank == dst:
        buf = out if out is not None else shard.new_empty((world,) + tuple(shard.shape))
        dist.gather(shard, list(buf.unbind(0)), dst=dst)
        return deinterleave(buf, H)
    dist.gather(shard, None, dst=dst)
    return None
