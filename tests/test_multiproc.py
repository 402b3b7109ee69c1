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
