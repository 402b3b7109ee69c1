"""(x, y, score) output: fdf_detect_scored, fdf_detect_batch_scored and
fdf_score_device against the oracle.  Points are bit-exact to the plain detector; scores are
the oracle's NMS score for the configured mode (the u16 the reference's NMS compares,
src/fast_simd.rs:623-718 / :722-749), or its max-threshold score when NMS is off."""
import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu


def expected(img, t, n, nms):
    pts, scores = oracle.detect(img, t, n, nms, with_scores=True)
    if nms == 0:   # NMS off: the max-threshold score of each keypoint
        ring = fast_hip.circle()
        xy = [(int(x), int(y)) for x, y in pts]
        scores = np.array([oracle.score_max_threshold(
            int(img[y, x]), [int(img[y + dy, x + dx]) for dx, dy in ring], n)
            for x, y in xy], dtype=np.uint16)
    return pts, scores


@pytest.mark.parametrize("nms", [0, 1, 2])
@pytest.mark.parametrize("t,n", [(16, 9), (30, 12), (8, 16)])
def test_scored_matches_oracle(nms, t, n):
    img = workloads.s1_frame(2, 320, 200)
    pts, scores = fast_hip.detect_scored_array(img, Config(t, n, NonMaximalSuppression(nms)))
    want_pts, want_scores = expected(img, t, n, nms)
    assert np.array_equal(pts, want_pts)
    assert np.array_equal(scores, want_scores)


def test_scored_golden(golden):
    img, off, maxt = golden
    for nms, want in ((0, off), (1, maxt)):
        pts, scores = fast_hip.detect_scored_array(img, Config(16, 9, NonMaximalSuppression(nms)))
        assert np.array_equal(pts, want)
        assert np.array_equal(scores, expected(img, 16, 9, nms)[1])


def test_scored_list_and_empty():
    img = workloads.s1_frame(0, 64, 48)
    got = fast_hip.detector_scored(img, Config(16, 9, NonMaximalSuppression.MaxThreshold))
    want_pts, want_scores = expected(img, 16, 9, 1)
    assert [(p.x, p.y) for p, _ in got] == [tuple(map(int, p)) for p in want_pts]
    assert [s for _, s in got] == [int(s) for s in want_scores]
    pts, scores = fast_hip.detect_scored_array(np.zeros((5, 40), np.uint8), Config(16, 9))
    assert pts.shape == (0, 2) and scores.shape == (0,)


def test_batch_scored_matches_per_frame():
    frames = np.stack([workloads.s1_frame(i, 200, 120) for i in range(4)])
    for nms in (0, 2):
        cfg = Config(16, 9, NonMaximalSuppression(nms))
        pts, scores, offs = fast_hip.detector_batch_scored(frames, cfg)
        for f in range(frames.shape[0]):
            wp, ws = expected(frames[f], 16, 9, nms)
            assert np.array_equal(pts[offs[f]:offs[f + 1]], wp)
            assert np.array_equal(scores[offs[f]:offs[f + 1]], ws)


def test_score_device_after_detect_device():
    torch = pytest.importorskip("torch")
    frames = workloads.s1_frames_torch(4, 5, 256, 160)
    host = frames.cpu().numpy()
    for nms, cap in ((1, 100_000), (0, 100_000), (2, 40)):
        cfg = Config(16, 9, NonMaximalSuppression(nms))
        out = torch.zeros((cap, 2), dtype=torch.int32, device="cuda")
        offs = torch.zeros(6, dtype=torch.int64, device="cuda")
        scores = torch.full((cap,), -1, dtype=torch.int16, device="cuda")
        fast_hip.detect_device(frames, cfg, out, offs)
        fast_hip.score_device(frames, cfg, out, offs, scores)
        torch.cuda.synchronize()
        want = [expected(host[f], 16, 9, nms) for f in range(5)]
        wp = np.concatenate([w[0] for w in want])
        ws = np.concatenate([w[1] for w in want])
        k = min(cap, len(wp))
        assert int(offs[-1]) == len(wp)
        assert np.array_equal(out[:k].cpu().numpy().astype(np.uint32), wp[:k])
        assert np.array_equal(scores[:k].cpu().numpy().view(np.uint16), ws[:k])


def _ring_grid(cells_x, cells_y, seed):
    """An image of 7x7 cells, one centre each at (7i+3, 7j+3): every centre's ring and
    centre byte lie inside its own cell.  Half the cells are uniform bytes; the other half
    are centre +- small offsets (rings near the threshold, long arcs)."""
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (7 * cells_y, 7 * cells_x), dtype=np.uint8)
    near = rng.integers(0, 2, (cells_y, cells_x), dtype=bool)
    cells = img.reshape(cells_y, 7, cells_x, 7).transpose(0, 2, 1, 3)
    centre = cells[:, :, 3, 3].astype(np.int32)
    noise = rng.integers(-40, 41, (cells_y, cells_x, 7, 7))
    mixed = np.clip(centre[:, :, None, None] + noise, 0, 255).astype(np.uint8)
    cells[near] = mixed[near]
    cells[:, :, 3, 3] = centre
    img = cells.transpose(0, 2, 1, 3).reshape(7 * cells_y, 7 * cells_x).copy()
    ys, xs = np.mgrid[0:cells_y, 0:cells_x]
    pts = np.stack([7 * xs.ravel() + 3, 7 * ys.ravel() + 3], axis=1).astype(np.uint32)
    return img, pts


def test_score_points_at_scale():
    """>= 1M random (ring, centre, t, n) cases through fdf_score_points against the oracle,
    both scores, every n = 9..16 (max-t) and every t = 0..255 (SAD); the reference runs 10M
    SAD and 20k max-t random triples (src/fast_simd.rs:1185-1236, :919-948)."""
    img, pts = _ring_grid(512, 256, 7)             # 131072 rings per pass
    checked = 0
    for n in range(9, 17):                          # max-t: 8 x 131072
        got = fast_hip.keypoint_scores(img, pts, Config(16, n, NonMaximalSuppression.MaxThreshold))
        want = oracle.score_points(img, pts, 1, 16, n)
        assert np.array_equal(got, want), n
        checked += len(pts)
    rng = np.random.default_rng(11)
    order = rng.permutation(len(pts))
    for t in range(256):                            # SAD: every threshold, 512 rings each
        sel = pts[order[(t * 512) % len(pts):(t * 512) % len(pts) + 512]]
        got = fast_hip.keypoint_scores(img, sel, Config(t, 9, NonMaximalSuppression.SumAbsolute))
        assert np.array_equal(got, oracle.score_points(img, sel, 2, t, 9)), t
        checked += len(sel)
    for t in (0, 8, 16, 40):                        # SAD: all rings at the bench thresholds
        got = fast_hip.keypoint_scores(img, pts, Config(t, 12, NonMaximalSuppression.SumAbsolute))
        assert np.array_equal(got, oracle.score_points(img, pts, 2, t, 12)), t
        checked += len(pts)
    assert checked >= 1_000_000
