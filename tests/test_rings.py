"""Ring-level helpers of the C ABI (the reference's pub items of src/fast_simd.rs:69-110, :623,
:722): fdf_circle / fdf_calculate_offsets (host, no GPU) and fdf_score_rings on the GPU
against the oracle's ring scores, at the reference's own test scale (10M SAD rings,
src/fast_simd.rs:1185-1236) plus rings with planted arcs so the detector's max-threshold
path (segment test + score_max_threshold<N>) carries most max-t cases."""
import ctypes

import numpy as np
import pytest

from feature_detector_fast_amd import NonMaximalSuppression, _native, fast_hip
from oracle import oracle

MAXT, SAD = NonMaximalSuppression.MaxThreshold, NonMaximalSuppression.SumAbsolute


def test_circle_and_offsets_match_reference():
    lib = _native.load()
    dx = (ctypes.c_int32 * 16)()
    dy = (ctypes.c_int32 * 16)()
    lib.fdf_circle(dx, dy)
    # src/fast_simd.rs:79-98, index 0 north then clockwise
    assert list(zip(dx, dy)) == [(0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2),
                                 (1, 3), (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1),
                                 (-2, -2), (-1, -3)]
    assert list(zip(dx, dy)) == [tuple(p) for p in fast_hip.circle()]
    lib.fdf_circle(dx, None)                         # either output may be NULL
    for w in (1, 7, 640, 1920, 3840, 65535):
        off = (ctypes.c_int32 * 16)()
        lib.fdf_calculate_offsets(w, off)
        assert list(off) == [y * w + x for x, y in fast_hip.circle()]
        assert list(off) == list(fast_hip.calculate_offsets(w))
    # cardinal indices (src/fast_simd.rs:69-72)
    assert (fast_hip.NORTH, fast_hip.EAST, fast_hip.SOUTH, fast_hip.WEST) == (0, 4, 8, 12)
    assert [tuple(fast_hip.circle()[i]) for i in (0, 4, 8, 12)] == [(0, -3), (3, 0), (0, 3), (-3, 0)]


def test_oracle_ring_scores_match_scalar():
    rng = np.random.default_rng(3)
    c = rng.integers(0, 256, 200, dtype=np.uint8)
    r = rng.integers(0, 256, (200, 16), dtype=np.uint8)
    for n in (9, 12, 16):
        want = [oracle.score_max_threshold(int(c[k]), r[k].tolist(), n) for k in range(200)]
        assert oracle.score_rings(c, r, 1, 0, n).tolist() == want
    want = [oracle.score_sum_abs(int(c[k]), r[k].tolist(), 20) for k in range(200)]
    assert oracle.score_rings(c, r, 2, 20, 9).tolist() == want


def planted_rings(rng, k, n):
    """Rings with an arc of >= n pixels strictly brighter (or darker) than the centre at a
    random start -- keypoints at t = 0 of either polarity -- plus unrestricted rings."""
    c = rng.integers(1, 255, k).astype(np.int32)
    r = rng.integers(0, 256, (k, 16)).astype(np.int32)
    length = rng.integers(n, 17, k)
    start = rng.integers(0, 16, k)
    dark = rng.random(k) < 0.5
    idx = (start[:, None] + np.arange(16)[None, :]) % 16
    in_arc = np.arange(16)[None, :] < length[:, None]
    hi = rng.integers(0, 256, (k, 16))
    bright_v = c[:, None] + 1 + hi % np.maximum(255 - c[:, None], 1)
    dark_v = c[:, None] - 1 - hi % np.maximum(c[:, None], 1)
    vals = np.where(dark[:, None], dark_v, bright_v)
    rows = np.arange(k)[:, None]
    arc_pos = idx[in_arc.nonzero()[0], in_arc.nonzero()[1]]
    r[rows.repeat(16, 1)[in_arc], arc_pos] = vals[in_arc]
    plain = rng.random(k) < 0.2                  # a fifth stays unrestricted
    r[plain] = rng.integers(0, 256, (int(plain.sum()), 16))
    return np.clip(c, 0, 255).astype(np.uint8), np.clip(r, 0, 255).astype(np.uint8)


@pytest.mark.gpu
def test_score_rings_max_threshold_all_n():
    """Max-threshold on 8 x 512k rings (n = 9..16) -- planted arcs of both polarities and
    unrestricted rings -- equal to the oracle (src/opencv_compat.rs:172-209)."""
    rng = np.random.default_rng(21)
    checked = 0
    for n in range(9, 17):
        c, r = planted_rings(rng, 1 << 19, n)
        got = fast_hip.score_rings(c, r, MAXT, consecutive=n)
        want = oracle.score_rings(c, r, 1, 0, n)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (n, int(bad[0]), c[bad[0]], r[bad[0]].tolist(), got[bad[0]],
                               want[bad[0]])
        checked += c.size
    assert checked >= 4_000_000


@pytest.mark.gpu
def test_score_rings_sum_abs_10m():
    """SAD on 10M random (ring, centre, t) cases, as the reference's own test
    (src/fast_simd.rs:1185-1236): every t = 0..255 with 40k rings each."""
    rng = np.random.default_rng(22)
    checked = 0
    for t in range(256):
        c = rng.integers(0, 256, 40_000, dtype=np.uint8)
        r = rng.integers(0, 256, (40_000, 16), dtype=np.uint8)
        got = fast_hip.score_rings(c, r, SAD, threshold=t)
        want = oracle.score_rings(c, r, 2, t, 9)
        assert np.array_equal(got, want), t
        checked += c.size
    assert checked >= 10_000_000


@pytest.mark.gpu
def test_score_rings_single_and_edges():
    # KAT of test_47_115_score_calc (src/fast_simd.rs:919-948)
    kat = [37, 37, 39, 39, 37, 42, 43, 16, 14, 13, 15, 16, 15, 38, 37, 38]
    assert fast_hip.keypoint_score_max_threshold(17, kat, 9) == 20
    ring = [200] * 9 + [10] * 7
    assert fast_hip.keypoint_score_max_threshold(100, ring, 9) == \
        oracle.score_max_threshold(100, ring, 9)
    assert fast_hip.keypoint_score_sum_abs_difference(ring, 100, 16) == \
        oracle.score_sum_abs(100, ring, 16)
    for c in (0, 255):                                # saturating bounds (test :1213-1222)
        for v in (0, 255):
            for t in (0, 1, 254, 255):
                assert fast_hip.keypoint_score_sum_abs_difference([v] * 16, c, t) == \
                    oracle.score_sum_abs(c, [v] * 16, t)
            for n in (9, 16):
                assert fast_hip.keypoint_score_max_threshold(c, [v] * 16, n) == \
                    oracle.score_max_threshold(c, [v] * 16, n)
    assert fast_hip.score_rings(np.zeros(0, np.uint8), np.zeros((0, 16), np.uint8), SAD).size == 0
    with pytest.raises(_native.FdfError):
        fast_hip.score_rings([1], [[0] * 16], MAXT, consecutive=8)
    with pytest.raises(_native.FdfError):
        fast_hip.score_rings([1], [[0] * 16], NonMaximalSuppression.Off)


@pytest.mark.gpu
def test_score_rings_device():
    import torch
    rng = np.random.default_rng(23)
    c, r = planted_rings(rng, 100_000, 12)
    dc = torch.from_numpy(c).cuda()
    dr = torch.from_numpy(r).cuda()
    out = torch.zeros(c.size, dtype=torch.int16, device="cuda")
    fast_hip.score_rings_device(dc, dr, out, MAXT, consecutive=12)
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, oracle.score_rings(c, r, 1, 0, 12))
    fast_hip.score_rings_device(dc, dr, out, SAD, threshold=30)
    assert np.array_equal(out.cpu().numpy().view(np.uint16), oracle.score_rings(c, r, 2, 30, 9))
    lib = _native.load()
    cfg = _native.FdfConfig(30, 9, int(SAD))
    ctx = fast_hip.context(0)
    flat = torch.zeros(16 * 4 + 1, dtype=torch.uint8, device="cuda")
    assert lib.fdf_score_rings_device(ctx.handle, dc.data_ptr(), flat.data_ptr() + 1, 4,
                                      ctypes.byref(cfg), out.data_ptr(), None) != 0   # unaligned


def test_score_rings_device_argument_checks():
    """score_rings_device names the failed check before any device call:
    non-uint8 centres or rings, and tensors that are not CUDA tensors, raise ValueError."""
    import torch
    c = torch.zeros(4, dtype=torch.uint8)
    r = torch.zeros((4, 16), dtype=torch.uint8)
    s = torch.zeros(4, dtype=torch.int16)
    with pytest.raises(ValueError, match="uint8"):
        fast_hip.score_rings_device(c.to(torch.int32), r, s, SAD)
    with pytest.raises(ValueError, match="uint8"):
        fast_hip.score_rings_device(c, r.to(torch.int16), s, SAD)
    with pytest.raises(ValueError, match="CUDA"):
        fast_hip.score_rings_device(c, r, s, SAD)


@pytest.mark.gpu
def test_score_rings_device_runs_in_stream_order():
    """Round 6: score_rings_device on torch's default stream (handle NULL) runs in that stream's
    order -- after the work enqueued before it, before the copy back.  The default stream first
    spins ~20 ms and then fills ``out`` with -1: a launch on any other stream would score first
    and have its scores overwritten by the fill."""
    import torch
    rng = np.random.default_rng(29)
    c, r = planted_rings(rng, 50_000, 9)
    dc = torch.from_numpy(c).cuda()
    dr = torch.from_numpy(r).cuda()
    out = torch.zeros(c.size, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0       # the HIP null stream
    for score, t, n, mode in ((SAD, 30, 9, 2), (MAXT, 0, 9, 1)):
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(50_000_000)
        out.fill_(-1)
        fast_hip.score_rings_device(dc, dr, out, score, threshold=t, consecutive=n)
        assert np.array_equal(out.cpu().numpy().view(np.uint16), oracle.score_rings(c, r, mode, t, n))
