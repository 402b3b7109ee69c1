"""Parity across band geometries and BASELINE config 5's batch shape.

The band height R decides which band NMS tier a band takes (LDS list <= 2048 keypoints, the
slot spill past it, or the score-free dense pass) and, since round 2, a launch's R follows the
keypoint density measured on the previous launch of the same configuration.  These tests pin
R explicitly over {nsub, 27, 43, 88, 256} (fdf_ctx_set_band_rows) at 1080p and 4K on frames
whose bands land in every tier, and run config 5's batch (4K t=8 n=12 SAD) three times so
the density feedback changes R between launches: every result equals the CPU oracle
(oracle/fast_oracle.c, pinned to the reference's goldens), launch after launch."""
import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu

ROWS = [1, 27, 43, 88, 256]      # 1 -> the geometry's sub-band multiple (nsub)


def _detect_rows(frames, cfg, rows):
    """detector_batch on a private context with the band height pinned to `rows`."""
    ctx = _native.Context(0)
    ctx.lock = __import__("threading").Lock()
    try:
        ctx.set_band_rows(rows)
        lib = _native.load()
        import ctypes
        f, h, w = frames.shape
        c = _native.FdfConfig(cfg.threshold, cfg.count, int(cfg.non_maximal_supression))
        offs = np.zeros(f + 1, dtype=np.uint64)
        n = ctypes.c_size_t(0)
        rc = lib.fdf_detect_batch(ctx.handle, frames.ctypes.data, f, w, h, w * h, ctypes.byref(c),
                                  None, 0, offs.ctypes.data, ctypes.byref(n))
        assert rc in (_native.FDF_OK, _native.FDF_ERR_CAPACITY)
        out = np.zeros((max(n.value, 1), 2), dtype=np.uint32)
        rc = lib.fdf_fetch_last(ctx.handle, out.ctypes.data, None, n.value, ctypes.byref(n))
        _native.check(rc, "fdf_fetch_last")
        return out[: n.value], offs
    finally:
        ctx.close()


def _check(frames, pts, offs, t, n, nms):
    for f in range(frames.shape[0]):
        want = oracle.detect(frames[f], t, n, nms)
        assert np.array_equal(pts[offs[f]:offs[f + 1]], want), f


@pytest.fixture(scope="module")
def frames_1080p():
    # S1 at t=16 n=9 (~0.5% keypoints), S1 at t=8 n=12 is denser, S3 (uniform noise, ~28%)
    # overflows the list and the slot of tall bands (the dense tier)
    return np.stack([workloads.s1_frame(2), workloads.s1_frame(9), workloads.s3_frame(3)])


@pytest.mark.parametrize("rows", ROWS)
@pytest.mark.parametrize("t,n,nms", [(16, 9, 1), (16, 9, 2), (8, 12, 2), (8, 12, 1)])
def test_band_rows_1080p(frames_1080p, rows, t, n, nms):
    pts, offs = _detect_rows(frames_1080p, Config(t, n, NonMaximalSuppression(nms)), rows)
    _check(frames_1080p, pts, offs, t, n, nms)


@pytest.mark.parametrize("rows", ROWS)
@pytest.mark.parametrize("nms", [0, 2])
def test_band_rows_4k(rows, nms):
    """4K t=8 n=12 (config 5's settings): 43-row bands of S1 hold 2 048-3 243 keypoints (the
    spill tier), 256-row bands ~10k, and the noise frame's bands the dense tier."""
    frames = np.stack([workloads.s1_frame(0, 3840, 2160), workloads.s3_frame(8, 3840, 2160)])
    pts, offs = _detect_rows(frames, Config(8, 12, NonMaximalSuppression(nms)), rows)
    _check(frames, pts, offs, 8, 12, nms)


def test_config5_batch_repeated():
    """BASELINE config 5's shape on one GPU: the bench's 128-frame 4K t=8 n=12 SAD batch, launched 3
    times (the band height follows the first launch's measured density from launch 2 on).
    All three launches give the same lists, every frame equals the CPU checker, and frame 0
    plus the three densest frames equal the scalar oracle."""
    import torch

    F, W, H = 128, 3840, 2160
    batch = workloads.s1_frames_torch(0, F, W, H)
    cfg = Config(8, 12, NonMaximalSuppression.SumAbsolute)
    out = torch.empty((F * 120_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    ctx = _native.Context(0)
    ctx.lock = __import__("threading").Lock()
    import ctypes
    lib = _native.load()
    c = _native.FdfConfig(8, 12, 2)
    runs = []
    try:
        stream = torch.cuda.current_stream()
        for _ in range(3):
            rc = lib.fdf_detect_device(ctx.handle, batch.data_ptr(), F, W, H, W * H,
                                       ctypes.byref(c), out.data_ptr(), out.shape[0],
                                       offs.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
            _native.check(rc, "fdf_detect_device")
            torch.cuda.synchronize()
            o = offs.cpu().numpy().copy()
            assert o[-1] <= out.shape[0]
            runs.append((o, out[: o[-1]].cpu().numpy().astype(np.uint32)))
    finally:
        ctx.close()
    for o, p in runs[1:]:
        assert np.array_equal(o, runs[0][0]) and np.array_equal(p, runs[0][1])
    o, p = runs[0]
    dens = np.argsort(np.diff(o))[::-1][:3]
    for f in sorted({0, *dens.tolist()}):
        want = oracle.detect(batch[f].cpu().numpy(), 8, 12, 2)
        assert np.array_equal(p[o[f]:o[f + 1]], want), f
    # every frame: the CPU checker (AVX2 port, pinned to the scalar oracle)
    ref_pts, ref_offs = oracle.avx2_detect_batch(batch, 8, 12, 2)
    assert np.array_equal(o.astype(np.uint64), ref_offs) and np.array_equal(p, ref_pts)


@pytest.mark.parametrize("nms", [0, 1, 2])
def test_direct_output_batches(nms):
    """Grids small enough to be resident at once write their points directly (each band's
    output index from a decoupled look-back over the bands before it, no compaction launch):
    an 8-frame 1080p batch (~860 bands) mixing S1, S2 and dense S3 frames, launched 5 times
    on the device path -- every launch equals the first, and every frame equals the oracle."""
    import torch

    host = [workloads.s1_frame(3), workloads.s3_frame(6), workloads.s2_frame(2), workloads.s1_frame(11),
            workloads.s3_frame(7), workloads.s1_frame(20), workloads.s2_frame(5), workloads.s1_frame(0)]
    frames = torch.from_numpy(np.stack(host)).cuda()
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    out = torch.empty((8 * 700_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(9, dtype=torch.int64, device="cuda")
    runs = []
    for _ in range(5):
        out.fill_(-1)
        fast_hip.detect_device(frames, cfg, out, offs)
        torch.cuda.synchronize()
        o = offs.cpu().numpy().copy()
        runs.append((o, out[: o[-1]].cpu().numpy().astype(np.uint32)))
    for o, p in runs[1:]:
        assert np.array_equal(o, runs[0][0]) and np.array_equal(p, runs[0][1])
    o, p = runs[0]
    for f in range(8):
        assert np.array_equal(p[o[f]:o[f + 1]], oracle.detect(host[f], 16, 9, nms)), f


def test_direct_output_4k_frame_and_capacity():
    """One 4K frame (~430 bands at the single-frame geometry) through the direct path with
    the output capacity short of the total: the first `cap` points are written, offsets hold
    the full total, and the host API's two-call pattern returns the whole oracle list."""
    import torch

    img = workloads.s1_frame(4, 3840, 2160)
    want = oracle.detect(img, 8, 12, 0)
    frames = torch.from_numpy(img).cuda().unsqueeze(0).contiguous()
    cap = len(want) // 2
    out = torch.full((cap, 2), -1, dtype=torch.int32, device="cuda")
    offs = torch.zeros(2, dtype=torch.int64, device="cuda")
    fast_hip.detect_device(frames, Config(8, 12, NonMaximalSuppression.Off), out, offs)
    torch.cuda.synchronize()
    assert int(offs[1]) == len(want) and int(offs[0]) == 0
    assert np.array_equal(out.cpu().numpy().astype(np.uint32), want[:cap])
    assert np.array_equal(fast_hip.detect_array(img, Config(8, 12, NonMaximalSuppression.Off)), want)


@pytest.mark.parametrize("nms", [0, 1, 2])
def test_many_band_batches(nms):
    """A grid of more bands than the device holds workgroups at once (8-row bands: ~1 400
    bands, run in rounds), 24 frames of 640x480 mixing S1, S2 and dense S3, launched 4 times
    on one context: every launch equals the first and every frame equals the oracle.  (The
    persistent-grid experiment of round 3, branch exp-persistent-grid, ran this test.)"""
    import ctypes

    import torch

    host = [(workloads.s1_frame, workloads.s2_frame, workloads.s3_frame)[i % 3](i, 640, 480)
            for i in range(24)]
    frames = torch.from_numpy(np.stack(host)).cuda()
    F, H, W = frames.shape
    cfg = _native.FdfConfig(16, 9, nms)
    out = torch.empty((F * 120_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    ctx = _native.Context(0)
    ctx.lock = __import__("threading").Lock()
    lib = _native.load()
    runs = []
    try:
        ctx.set_band_rows(8)
        stream = torch.cuda.current_stream()
        for _ in range(4):
            out.fill_(-1)
            rc = lib.fdf_detect_device(ctx.handle, frames.data_ptr(), F, W, H, W * H,
                                       ctypes.byref(cfg), out.data_ptr(), out.shape[0],
                                       offs.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
            _native.check(rc, "fdf_detect_device")
            torch.cuda.synchronize()
            o = offs.cpu().numpy().copy()
            assert o[-1] <= out.shape[0]
            runs.append((o, out[: o[-1]].cpu().numpy().astype(np.uint32)))
    finally:
        ctx.close()
    for o, p in runs[1:]:
        assert np.array_equal(o, runs[0][0]) and np.array_equal(p, runs[0][1])
    o, p = runs[0]
    for f in range(F):
        assert np.array_equal(p[o[f]:o[f + 1]], oracle.detect(host[f], 16, 9, nms)), f
