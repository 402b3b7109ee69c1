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
