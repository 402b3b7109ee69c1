"""Host-side bench.py logic (CPU): the kernel-timing sample interval and the roofline fields
built from a timed region (one definition of the algorithmic bytes,
percentiles only from enough samples)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


@pytest.mark.parametrize("local", [0, 1, 5, 7])
def test_select_device_one_rank_per_gpu(local):
    """The driver's torchrun path: LOCAL_RANK r -> cuda:r over the default backend (RCCL);
    --ranks-share-device -> every rank on cuda:0 over gloo."""
    assert bench.select_device(False, 8, local) == (local, "nccl")
    assert bench.select_device(True, 8, local) == (0, "gloo")
    assert bench.select_device(False, 1, 0) == (0, None)
    args = bench.parse_args(["--gpus", "8"])
    assert not args.ranks_share_device and args.lanes == 3


@pytest.mark.parametrize("batch,lanes,need,copies", [
    (512 * 1920 * 1080, 3, 1 << 29, 3),      # headline: one 1.06 GB copy per lane
    (64 * 1920 * 1080, 3, 1 << 29, 6),       # 8-GPU strong shard: >= 512 MiB, lanes multiple
    (128 * 3840 * 2160, 3, 0, 3),            # config 5
    (10, 1, 0, 1), (10, 2, 25, 4)])
def test_copies_per_lane(batch, lanes, need, copies):
    """At least one distinct input copy per lane (no two launches in flight read the same
    bytes), >= min_bytes in all, a multiple of the lanes."""
    n = bench.n_copies(batch, lanes, need)
    assert n == copies and n % lanes == 0 and n * batch >= need


def test_copies_differ_and_lanes_keep_their_copies():
    import numpy as np

    import workloads
    # copy c's frame k is S1 frame first + k + 211 c: a different roll at every position
    for k in range(0, 600, 7):
        for c in (1, 2, 3, 4, 5):
            assert workloads.s1_roll(k) != workloads.s1_roll(k + bench.COPY_ROLL * c)
    # step k on lane k % L reads copy k % C, C a multiple of L: a lane keeps to its copies
    L, C = 3, bench.n_copies(64, 3, 200)
    for k in range(50):
        assert (k % C) % L == k % L
    assert np.unique([(k % C) for k in range(50) if k % L == 1]).tolist() == [1, 4]


def test_raster_order_check():
    import numpy as np
    pts = np.array([[5, 3], [9, 3], [4, 4], [3, 3], [8, 3]], dtype=np.uint32)
    assert bench.raster_order_ok(pts, [0, 3, 5], 100)          # frame boundary at 3
    assert not bench.raster_order_ok(pts, [0, 5], 100)
    assert bench.raster_order_ok(pts[:0], [0, 0], 100)


def test_roofline_from_timed_region():
    W, H, F, K = 1920, 1080, 512, 2_000_000
    in_bytes = F * W * H
    alg = in_bytes + 8 * K + 4 * F
    # 3 lanes, 20 launches spanning 8.0 ms of GPU time, each launch 1.2 ms long on its own
    t = bench.Timed(elapsed=0.0081, span_ms=8.0, det=[1.2] * 20, com=[0.015] * 20, last=1,
                    steps=20, lanes=3)
    r = bench.roofline_of(t, alg, in_bytes, (None, None))
    assert r["kernel_ms_avg"] == pytest.approx(0.4)
    assert r["achieved"] == pytest.approx(alg / 0.4e-3 / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-3)
    assert r["frac_input_bytes_only"] < r["frac"]
    assert r["alg_bytes_per_launch"] == alg and r["input_bytes_per_launch"] == in_bytes
    assert r["launches_in_flight_avg"] == pytest.approx(3.0)
    assert r["launch_ms"] is not None and r["timed_launches"] == 20
    few = bench.Timed(0.001, 1.0, [0.4] * 4, [0.01] * 4, 0, 4, 1)
    r4 = bench.roofline_of(few, alg, in_bytes, (None, None))
    assert r4["launch_ms"] is None and r4["compaction_kernel_ms"] is None    # mean only


def test_batch_parity_checks_every_frame():
    """bench.batch_parity on CPU tensors: each lane's last result equal to
    the checker on every frame passes; one moved point in any frame of any lane fails, and so
    do wrong offsets."""
    import numpy as np
    import torch

    import workloads
    from oracle import oracle

    W, H, F = 160, 90, 5
    copies = [torch.from_numpy(np.stack([workloads.s1_frame(i + 211 * c, W, H) for i in range(F)]))
              for c in range(2)]
    ref = [oracle.avx2_detect_batch(c, 16, 9, 1) for c in copies]

    class Bufs:
        pass

    def bufs_from(refs):
        b = Bufs()
        b.out = [torch.from_numpy(np.concatenate([p.astype(np.int32), np.zeros((7, 2), np.int32)]))
                 for p, _ in refs]
        b.offs = [torch.from_numpy(o.astype(np.int64)) for _, o in refs]
        return b

    tm = bench.Timed(0.01, 1.0, [], [], 1, 4, 2, lane_copy={0: 0, 1: 1}, copy_steps={0: 2, 1: 2})
    rec, kp = bench.batch_parity(oracle, copies, bufs_from(ref), tm, 16, 9, 1, W)
    assert rec["bit_exact"] and rec["oracle_frames"] == "all" and rec["raster_order"]
    assert kp == (ref[0][1][-1] + ref[1][1][-1]) / 2
    assert [c["copy"] for c in rec["lanes_compared"]] == [0, 1]
    # a point moved in the last frame of lane 1
    bad = bufs_from(ref)
    n = int(ref[1][1][-1])
    bad.out[1][n - 1, 0] += 1
    assert not bench.batch_parity(oracle, copies, bad, tm, 16, 9, 1, W)[0]["bit_exact"]
    # offsets shifted between two frames of lane 0 (same points, wrong frame split)
    bad = bufs_from(ref)
    bad.offs[0][2] += 1
    assert not bench.batch_parity(oracle, copies, bad, tm, 16, 9, 1, W)[0]["bit_exact"]


def test_batch_parity_compares_copies_no_lane_read_last():
    """with more copies than lanes, the copies the lanes did not read last are
    detected once more (`redo`) and compared too; a wrong result there fails the record."""
    import numpy as np
    import torch

    import workloads
    from oracle import oracle

    W, H, F = 160, 90, 3
    copies = [torch.from_numpy(np.stack([workloads.s1_frame(i + 211 * c, W, H) for i in range(F)]))
              for c in range(4)]
    ref = [oracle.avx2_detect_batch(c, 16, 9, 1) for c in copies]

    class Bufs:
        pass

    def put(b, lane, r):
        p, o = r
        b.out[lane] = torch.from_numpy(np.concatenate([p.astype(np.int32), np.zeros((7, 2), np.int32)]))
        b.offs[lane] = torch.from_numpy(o.astype(np.int64))

    def run(corrupt_copy=None):
        b = Bufs()
        b.out, b.offs = [None, None], [None, None]
        put(b, 0, ref[2])
        put(b, 1, ref[3])
        redone = []

        def redo(c):
            put(b, 0, ref[c])
            if c == corrupt_copy:
                b.out[0][0, 0] += 1
            redone.append(c)
            return 0
        tm = bench.Timed(0.01, 1.0, [], [], 1, 4, 2, lane_copy={0: 2, 1: 3},
                         copy_steps={0: 1, 1: 1, 2: 1, 3: 1})
        rec, _ = bench.batch_parity(oracle, copies, b, tm, 16, 9, 1, W, redo=redo)
        return rec, redone

    rec, redone = run()
    assert rec["bit_exact"] and rec["copies_compared"] == 4 and redone == [0, 1]
    assert [c["result"] for c in rec["lanes_compared"]] == ["timed", "timed", "after", "after"]
    assert not run(corrupt_copy=1)[0]["bit_exact"]
