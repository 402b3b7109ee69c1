"""World-size-2 gloo test of bench.py's distributed skeleton (CPU): frame sharding is
disjoint and complete, and the max/sum reductions used for timing and totals agree on
every rank.  The data path itself has no collective (frames shard independently)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, frames_per_rank, q):
    import torch
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = bench.shard_frames(rank, frames_per_rank)
    elapsed = bench.reduce_max(0.5 + rank, world, torch.device("cpu"))
    total = bench.reduce_sum(float(count), world, torch.device("cpu"))
    bench.barrier(world)
    q.put((rank, first, count, elapsed, total))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_frame_sharding_and_reductions(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 7, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames = sorted(f for _, first, count, _, _ in res for f in range(first, first + count))
    assert frames == list(range(7 * world))                     # disjoint and complete
    assert all(r[3] == 0.5 + (world - 1) for r in res)          # max over ranks
    assert all(r[4] == 7.0 * world for r in res)                # sum over ranks


def _shard_worker(rank, world, port, frames_total, q):
    """One rank of a strong-scaled batch: it generates its own contiguous shard of S1 frames
    (by global frame index, as bench.py does), detects them (the CPU oracle stands in for
    the GPU here) and all-gathers per-frame hashes of its keypoint lists."""
    import hashlib

    import torch.distributed as dist

    import bench
    import workloads
    from oracle import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = bench.strong_shard(rank, world, frames_total)
    mine = []
    for f in range(first, first + count):
        pts = oracle.detect(workloads.s1_frame(f, 160, 120), 16, 9, 1)
        mine.append((f, hashlib.sha256(pts.tobytes()).hexdigest(), len(pts)))
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    q.put((rank, gathered))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strong_shards_reassemble_in_frame_order(world):
    """Config 4's layout at world 2/3 over gloo: every rank sees the same gathered list, the
    shards concatenate to frames 0..F-1 in order, and each frame's hash equals the one a
    single process computes for it."""
    import hashlib

    import workloads
    from oracle import oracle

    frames_total = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, frames_total, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    views = [r[1] for r in res]
    assert all(v == views[0] for v in views)                     # same on every rank
    merged = [e for shard in views[0] for e in shard]
    assert [e[0] for e in merged] == list(range(frames_total))   # frame order
    for f, digest, n in merged:
        pts = oracle.detect(workloads.s1_frame(f, 160, 120), 16, 9, 1)
        assert digest == hashlib.sha256(pts.tobytes()).hexdigest() and n == len(pts), f


def test_strong_shard_partition():
    import bench

    for world in range(1, 9):
        spans = [bench.strong_shard(r, world, 512) for r in range(world)]
        assert spans[0][0] == 0
        assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert spans[-1][0] + spans[-1][1] == 512
        assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
