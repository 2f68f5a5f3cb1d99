"""Multi-rank path of bench.py on CPU: world size 2 (and 3) over gloo.

Each rank takes the image rows `shard_rows(rank, world, H)` of a frame, pads
its shard to `rows_per_rank`, the shards are gathered to rank 0 with one
collective (bench.py uses RCCL; the logic is backend-independent) and
`deinterleave` must rebuild the single-process frame bit for bit.  The frame
content comes from the oracle (test infrastructure), rendered on the CPU.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from raytracingdemo_amd.shards import deinterleave, deinterleave_into, gather_frames, rows_per_rank, shard_rows  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frames(W: int, H: int, F: int) -> np.ndarray:
    """F reference-semantics frames (rgb) of a small scene, from the oracle."""
    import pyoracle
    from conftest import golden_scene
    o = pyoracle.Oracle()
    tris = golden_scene("teapot.obj")
    b = o.bvh(tris, "bsah", 4)
    c = o.scene_center(tris)
    out = []
    for f in range(F):
        pos, d = o.camera_path(c, 36, 3 * f)
        out.append(b.render(pos, d, W, H, want=("rgb",))["rgb"].reshape(H, W, 3))
    return np.stack(out)


def _worker(rank: int, world: int, port: int, W: int, H: int, F: int, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _frames(W, H, F)
        rows = rows_per_rank(H, world)
        mine = list(shard_rows(rank, world, H))
        shard = torch.full((F, rows, W, 3), 255, dtype=torch.uint8)  # padding rows stay 255
        shard[:, : len(mine)] = torch.from_numpy(full[:, mine])
        img = gather_frames(shard, H, world, rank)  # the bench's gather + de-interleave
        if rank == 0:
            img = img.numpy()
            q.put(("ok", bool(np.array_equal(img, full)), img.shape))
    except Exception as e:  # surface worker failures to the test
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 37), (2, 40), (3, 29)])
def test_row_interleaved_shards_gather_to_full_frame(world, H):
    W, F = 24, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, F, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, ok, shape = q.get(timeout=10)
    assert status == "ok", ok
    assert ok and shape == (F, H, W, 3)


def test_deinterleave_single_process():
    H, W, F = 11, 5, 3
    full = torch.arange(F * H * W, dtype=torch.int32).reshape(F, H, W)
    for world in (1, 2, 3, 4, 8, 11, 13):
        rows = rows_per_rank(H, world)
        sh = torch.full((world, F, rows, W), -1, dtype=torch.int32)
        for r in range(world):
            idx = list(shard_rows(r, world, H))
            sh[r, :, : len(idx)] = full[:, idx]
        assert torch.equal(deinterleave(sh, H), full)
        # the bench's single-copy form (padded and unpadded shards)
        out = torch.empty_like(full)
        assert torch.equal(deinterleave_into(sh, H, out), full)
    H = 16  # whole bands of 8 rows: no padding for 1 or 2 ranks
    full = torch.arange(F * H * W * 3, dtype=torch.int32).reshape(F, H, W, 3)
    for world in (1, 2, 3, 4):
        rows = rows_per_rank(H, world)
        sh = torch.zeros((world, F, rows, W, 3), dtype=torch.int32)
        for r in range(world):
            idx = shard_rows(r, world, H)
            sh[r, :, : len(idx)] = full[:, idx]
        assert torch.equal(deinterleave_into(sh, H, torch.empty_like(full)), full)


def test_deinterleave_from_combined_payloads():
    """bench.py ships one payload per rank and step — the rgb frames, then the
    per-frame hit counts 8-B aligned — and rank 0 de-interleaves the rgb part
    of the gathered [world, payload] buffer as a strided view (the host path
    of a rehearsal; on the GPU the same layout is the library's de-interleave
    job with block_bytes = payload)."""
    H, W, F = 37, 6, 3
    full = torch.randint(0, 256, (F, H, W, 3), dtype=torch.uint8)
    for world in (1, 2, 3, 8):
        rows = rows_per_rank(H, world)
        rgb_bytes = F * rows * W * 3
        cnt_off = (rgb_bytes + 7) // 8 * 8
        pay_bytes = cnt_off + F * 8
        g = torch.zeros((world, pay_bytes), dtype=torch.uint8)
        for r in range(world):
            idx = shard_rows(r, world, H)
            shard = torch.zeros((F, rows, W, 3), dtype=torch.uint8)
            shard[:, :len(idx)] = full[:, idx]
            g[r, :rgb_bytes] = shard.reshape(-1)
            g[r, cnt_off:].view(torch.int64)[:] = torch.arange(F) + 100 * r
        view = g[:, :rgb_bytes].view(world, F, rows, W, 3)
        assert torch.equal(deinterleave_into(view, H, torch.empty_like(full)), full)
        cnt = g[:, cnt_off:].view(torch.int64)
        assert torch.equal(cnt.sum(0), world * torch.arange(F) + 100 * sum(range(world)))


def test_python_shards_match_the_library_layout():
    """shards.py (bench.py's partition) and the library's rt_shard_height /
    rt_deinterleave_rows (rt_render_shard_device's layout) agree."""
    import raytracingdemo_amd as rt
    for H in (1, 7, 8, 9, 37, 1080, 2160, 1081):
        for world in (1, 2, 3, 4, 7, 8):
            rows = [shard_rows(r, world, H) for r in range(world)]
            assert sorted(j for rr in rows for j in rr) == list(range(H))
            assert [len(rr) for rr in rows] == [rt.shard_height(H, world, r) for r in range(world)]
            assert max(len(rr) for rr in rows) <= rows_per_rank(H, world)
            assert all(rr == sorted(rr) for rr in rows)

def _facts_worker(rank: int, world: int, port: int, ordinals, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        me = torch.tensor([rank, rank, ordinals[rank], 0x40 + ordinals[rank]], dtype=torch.int64)
        allv = [torch.empty_like(me) for _ in range(world)]
        dist.all_gather(allv, me)
        table = [[int(x) for x in v.tolist()] for v in allv]
        for gpus, backend in ((world, "nccl"), (world + 1, "nccl"), (world, "gloo")):
            q.put((rank, gpus, backend, bench.rank_problems(table, backend, dist.get_world_size(), world, gpus,
                                                            False)))
    except Exception as e:
        q.put((rank, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ordinals,ok", [([0, 1], True), ([0, 0], False), ([3, 1, 2], True), ([1, 2, 1], False)])
def test_bench_rank_self_check(ordinals, ok):
    """bench.py's N-rank self-check (rank_problems on the rows all_gather
    collects from every rank, gloo here): one device ordinal per rank, the
    process group's size equal to --gpus and the nccl (RCCL) backend pass;
    a repeated ordinal, a --gpus that disagrees or another backend fail."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    world = len(ordinals)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_facts_worker, args=(r, world, port, ordinals, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(3 * world)]
    for p in procs:
        p.join(timeout=60)
    for rank, gpus, backend, problems in res:
        assert gpus is not None, problems
        if gpus == world and backend == "nccl":
            assert (problems == []) == ok, (ordinals, problems)
        else:
            assert problems, (gpus, backend)
