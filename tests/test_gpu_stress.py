"""Batch-scale stress of the HIP path: thresholds x circle counts x NMS modes on full-size
batches (the geometry the bench runs: tall bands, long units, FIFO overflow, LDS score-list
overflow, bitmap slots).  Every case launches twice and compares the two results on the
device (races show up as run-to-run differences), then checks the densest frames and frame 0
against the CPU oracle.  Needs an MI355X."""
import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu

W, H = 1920, 1080


def launch_twice_and_check(frames, t, n, nms, n_check=2):
    import torch

    F = frames.shape[0]
    cfg = Config(t, n, NonMaximalSuppression(nms))
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    out = torch.empty((1, 2), dtype=torch.int32, device="cuda")
    fast_hip.detect_device(frames, cfg, out, offs)          # sizing launch
    torch.cuda.synchronize()
    total = int(offs[-1])
    out = torch.empty((max(total, 1), 2), dtype=torch.int32, device="cuda")
    fast_hip.detect_device(frames, cfg, out, offs)
    first_pts, first_offs = out.clone(), offs.clone()
    fast_hip.detect_device(frames, cfg, out, offs)
    torch.cuda.synchronize()
    assert int(first_offs[-1]) == total, (t, n, nms)
    assert torch.equal(offs, first_offs), (t, n, nms)
    assert torch.equal(out, first_pts), (t, n, nms)
    o = offs.cpu().numpy()
    counts = np.diff(o)
    pts = out[:total].cpu().numpy().astype(np.uint32)
    for f in sorted({0, *np.argsort(counts)[-n_check:].tolist()}):
        want = oracle.detect(frames[f].cpu().numpy(), t, n, nms)
        assert np.array_equal(pts[o[f]:o[f + 1]], want), (f, t, n, nms, len(want))
    # every frame of the batch: the CPU checker (the AVX2 port over a thread pool, pinned to
    # the scalar oracle by tests/test_oracle.py), offsets and points of the whole output
    # (the reference compares whole Vecs: tests/compare.rs:45-61)
    ref_pts, ref_offs = oracle.avx2_detect_batch(frames, t, n, nms)
    assert np.array_equal(o.astype(np.uint64), ref_offs), (t, n, nms)
    assert np.array_equal(pts, ref_pts), (t, n, nms)
    return total


@pytest.fixture(scope="module")
def s1_batch():
    return workloads.s1_frames_torch(0, 512, W, H)


@pytest.mark.parametrize("nms", [0, 1, 2])
@pytest.mark.parametrize("n", [9, 12, 16])
@pytest.mark.parametrize("t", [3, 8, 30])
def test_s1_batch(s1_batch, t, n, nms):
    launch_twice_and_check(s1_batch, t, n, nms)


@pytest.fixture(scope="module")
def mixed_batch():
    """64 frames: S2, S3, noise and half-noise/half-S1, interleaved."""
    import torch

    rng = np.random.default_rng(2024)
    frames = []
    for i in range(16):
        frames.append(workloads.s2_frame(100 + i))
        frames.append(workloads.s3_frame(200 + i))
        frames.append(rng.integers(0, 256, (H, W), dtype=np.uint8))
        half = workloads.s1_frame(300 + i)
        half[: H // 2] = rng.integers(0, 256, (H // 2, W), dtype=np.uint8)
        frames.append(half)
    return torch.from_numpy(np.stack(frames)).cuda()


@pytest.mark.parametrize("nms", [0, 1, 2])
@pytest.mark.parametrize("n", [9, 16])
@pytest.mark.parametrize("t", [6, 20])
def test_mixed_batch_full_geometry(mixed_batch, t, n, nms):
    ctx = fast_hip.context(0)
    ctx.set_geometry(1)                           # 64 frames with the full-size geometry
    try:
        launch_twice_and_check(mixed_batch, t, n, nms, n_check=3)
    finally:
        ctx.set_geometry(0)


@pytest.mark.parametrize("nms", [1, 0, 2])
def test_config4_exact_batch(s1_batch, nms):
    """BASELINE.json config 4's exact per-GPU workload: 512 S1 1080p frames, t=16 n=9,
    max-t NMS (and the bench's NMS-off / SAD legs) -- launched twice (device-side
    equality), every frame against the CPU checker, frame 0 and the 3 densest frames against
    the scalar oracle."""
    launch_twice_and_check(s1_batch, 16, 9, nms, n_check=3)


@pytest.mark.parametrize("nms", [1, 2])
def test_nms_overflow_tiers(nms):
    """Bands whose keypoints overflow the LDS score list, at every density the band NMS pass
    distinguishes (band_nms_spill): ranked scores in LDS, ranked scores in the band's slot,
    and no stored scores (recompute all).  Frames mix S1 rows with uniform-noise rows (~28%
    keypoints at t=16 n=9) at rates from 3% to 60%, so band densities sweep across the tiers;
    every frame is checked against the oracle."""
    import torch

    rng = np.random.default_rng(77)
    frames = []
    for k, rate in enumerate((0.03, 0.06, 0.1, 0.15, 0.2, 0.3, 0.45, 0.6)):
        f = workloads.s1_frame(400 + k)
        noisy = rng.random(H) < rate
        f[noisy] = rng.integers(0, 256, (int(noisy.sum()), W), dtype=np.uint8)
        frames.append(f)
    batch = torch.from_numpy(np.stack(frames)).cuda()
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    F = batch.shape[0]
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    out = torch.empty((F * W * H // 4, 2), dtype=torch.int32, device="cuda")
    ctx = fast_hip.context(0)
    for geometry in (0, 1):                 # the batch's own geometry, then the tall bands
        ctx.set_geometry(geometry)
        try:
            fast_hip.detect_device(batch, cfg, out, offs)
            torch.cuda.synchronize()
        finally:
            ctx.set_geometry(0)
        o = offs.cpu().numpy()
        for f in range(F):
            got = out[o[f]:o[f + 1]].cpu().numpy().astype(np.uint32)
            want = oracle.detect(frames[f], 16, 9, nms)
            assert np.array_equal(got, want), (geometry, f, nms, len(got), len(want))
