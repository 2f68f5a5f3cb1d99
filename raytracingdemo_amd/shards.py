"""Image shards for the one-process-per-GPU driver (bench.py).

The partition is the library's (include/rt.h rt_render_shard_device; the
index arithmetic of rt_device.h rt_shard_rows / rt_gathered_row): bands of
BAND = 8 image rows — one row of 8x8 tiles — interleaved over the ranks, band
b of a frame on rank b mod world.  Interleaving spreads the depth-complexity
gradient of a frame; whole bands keep each rank's tiles
coherent (single interleaved rows cost a rank half its rate at 8 ranks).
Every rank holds `rows_per_rank(H, world)` rows (padding where its bands are
fewer or the last band is partial), so the shards gather with one equal-sized
collective; rank 0 de-interleaves with one gather kernel.  `band=1` gives
single interleaved rows (row j on rank j mod world), the layout of the
row-shard entry points (rt_render_paths_device with row0 = rank, row_stride =
world).
"""
from __future__ import annotations

BAND = 8


def _bands(H: int, band: int) -> int:
    return (H + band - 1) // band


def rows_per_rank(H: int, world: int, band: int = BAND) -> int:
    """Rows of the tallest shard (every shard's buffer is padded to it)."""
    return (_bands(H, band) + world - 1) // world * band


def shard_rows(rank: int, world: int, H: int, band: int = BAND) -> list[int]:
    """Image rows of `rank`'s shard, in shard order (its bands back to back)."""
    return [b * band + k for b in range(rank, _bands(H, band), world) for k in range(band) if b * band + k < H]


def source_rows(H: int, world: int, rows: int, band: int = BAND) -> list[int]:
    """For every image row j: its position in the [world * rows] stack of
    padded shards (shard g = (j // band) % world, row ((j // band) // world) *
    band + j % band of it)."""
    out = []
    for j in range(H):
        b = j // band
        out.append((b % world) * rows + (b // world) * band + j % band)
    return out


_IDX: dict = {}
_FLAT_MAX = 8  # index tensors kept per cache (one per shape and device; _FLAT's hold F*H int64)


def _index(H: int, world: int, rows: int, device, band: int):
    import torch
    key = (H, world, rows, str(device), band)
    if key not in _IDX:
        while len(_IDX) >= _FLAT_MAX:
            _IDX.pop(next(iter(_IDX)))
        _IDX[key] = torch.tensor(source_rows(H, world, rows, band), dtype=torch.long, device=device)
    return _IDX[key]


def deinterleave(gathered, H: int, band: int = BAND):
    """Full images from gathered shards.

    gathered: tensor [world, F, rows, W, ...] (shard k from rank k, rows =
    rows_per_rank(H, world), padding rows last).  Returns [F, H, W, ...] with
    image row j taken from its shard (source_rows)."""
    world, F, rows = gathered.shape[0], gathered.shape[1], gathered.shape[2]
    rest = tuple(gathered.shape[3:])
    stack = gathered.transpose(0, 1).reshape((F, world * rows) + rest)
    return stack.index_select(1, _index(H, world, rows, gathered.device, band))


_FLAT: dict = {}


def _flat_index(H: int, world: int, F: int, rows: int, device, band: int):
    """For every (frame f, image row j), f-major: the row of the gathered
    [world, F, rows] block that holds it, (g F + f) rows + r for source row
    g rows + r (source_rows) — so the de-interleave is one row gather of the
    gathered buffer as it lies, without first transposing it."""
    import torch
    key = (H, world, F, rows, str(device), band)
    if key not in _FLAT:
        src = _index(H, world, rows, device, band)
        g, r = src // rows, src % rows
        f = torch.arange(F, dtype=torch.long, device=device)[:, None]
        while len(_FLAT) >= _FLAT_MAX:  # bounded: a sweep over sizes keeps only the latest shapes
            _FLAT.pop(next(iter(_FLAT)))
        _FLAT[key] = ((g[None, :] * F + f) * rows + r[None, :]).reshape(-1)
    return _FLAT[key]


def deinterleave_into(gathered, H: int, out, band: int = BAND):
    """deinterleave() written into `out` ([F, H, W, ...]) with one row-gather
    kernel straight from the gathered [world, F, rows, W, ...] buffer (one
    read and one write of the frames)."""
    world, F, rows = gathered.shape[0], gathered.shape[1], gathered.shape[2]
    import torch
    flat = gathered.reshape((world * F * rows, -1))
    idx = _flat_index(H, world, F, rows, gathered.device, band)
    if out.device != gathered.device:  # (host-side gathers: one copy across)
        out.copy_(flat.index_select(0, idx).reshape(out.shape))
    else:
        torch.index_select(flat, 0, idx, out=out.view(F * H, -1))
    return out


def gather_frames(shard, H: int, world: int, rank: int, dst: int = 0, out=None, band: int = BAND):
    """Gather every rank's [F, rows, W, ...] shard to `dst` and de-interleave there.

    The shards land in one [world, F, rows, W, ...] buffer (`out`, allocated
    once by the caller, or here) through views of it, so the collective writes
    straight into the layout `deinterleave` reads.  Returns [F, H, W, ...] on
    `dst`, None elsewhere.
    """
    import torch.distributed as dist
    if rank == dst:
        buf = out if out is not None else shard.new_empty((world,) + tuple(shard.shape))
        dist.gather(shard, list(buf.unbind(0)), dst=dst)
        return deinterleave(buf, H, band)
    dist.gather(shard, None, dst=dst)
    return None
