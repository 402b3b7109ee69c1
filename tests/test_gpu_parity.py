"""Parity of the HIP path (through the C ABI) with the CPU oracle and the reference's
golden fixtures.  Bit-exact: keypoint lists are compared as ordered arrays, the way
tests/compare.rs:59 of the reference compares Vec<Point>.  Needs an MI355X."""
import ctypes
import os
import subprocess
import threading

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import (Config, FdfError, GrayImage, NonMaximalSuppression,
                                       Point, detect, fast_hip)
from feature_detector_fast_amd import _native
from oracle import oracle

pytestmark = pytest.mark.gpu

NMS = (NonMaximalSuppression.Off, NonMaximalSuppression.MaxThreshold,
       NonMaximalSuppression.SumAbsolute)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(img, t, n, nms):
    return fast_hip.detect_array(img, Config(t, n, NonMaximalSuppression(nms)))


def assert_same(img, t, n, nms):
    got = run(img, t, n, nms)
    want = oracle.detect(img, t, n, nms)
    assert got.shape == want.shape, (img.shape, t, n, nms, got.shape, want.shape)
    assert np.array_equal(got, want), (img.shape, t, n, nms)
    return len(got)


# --- the reference's own fixtures ------------------------------------------------------

def test_golden_lists(golden):
    img, off, maxt = golden
    assert np.array_equal(run(img, 16, 9, 0), off)      # 309, == OpenCV 3.2
    assert np.array_equal(run(img, 16, 9, 1), maxt)     # 131, == OpenCV 3.2


def test_crate_api_returns_points(golden):
    img, off, _ = golden
    pts = detect(img, Config(16, 9, NonMaximalSuppression.Off))
    assert pts == [Point(int(x), int(y)) for x, y in off]
    gi = GrayImage.from_array(img)
    assert Config(16, 9).detect(gi) == pts


@pytest.fixture(scope="module")
def compare_input(golden):
    """The image of tests/compare.rs: $INPUT_FILE when set (any PNG/PGM: opened as RGB8 and
    converted with image 0.24.6's to_luma8, compare.rs:24-33), else the reference's test image
    (the golden fixture, already grey)."""
    path = os.environ.get("INPUT_FILE")
    if not path:
        return golden[0], None
    return workloads.input_image(path)


@pytest.mark.parametrize("t,n,nms", [(16, 9, 0), (16, 9, 1), (16, 9, 2), (16, 12, 2),
                                     (32, 12, 2)])
def test_compare_rs_configs(compare_input, t, n, nms):
    """tests/compare.rs:66-114: the five configurations of the reference's parity test, on
    $INPUT_FILE when set.  With max-t, the reference's hash guard (compare.rs:83-89): on its
    own test image (RGB bytes hashing to 0x8444a9356505ecab) the keypoints must hash to
    0x8bf9cd0f9ca9ebec (Rust's DefaultHasher, workloads.rust_hash_points)."""
    img, rgb = compare_input
    assert_same(img, t, n, nms)
    if nms == 1 and rgb is not None:
        if workloads.rust_hash_bytes(rgb) == workloads.REF_IMAGE_HASH:
            assert workloads.rust_hash_points(run(img, t, n, nms)) == workloads.REF_MAXT_HASH


def test_hand_kat():
    """src/fast_simd.rs:950-1022 test_47_115_hand: keypoint at (64, 64), max-t score 20."""
    img = np.zeros((128, 128), dtype=np.uint8)
    img[64, 64] = 17
    ring = [37, 37, 39, 39, 37, 42, 43, 16, 14, 13, 15, 16, 15, 38, 37, 38]
    for (dx, dy), v in zip(fast_hip.circle(), ring):
        img[64 + dy, 64 + dx] = v
    pts = run(img, 16, 9, 0)
    assert [64, 64] in pts.tolist()
    score = fast_hip.keypoint_scores(img, [[64, 64]], Config(16, 9, NonMaximalSuppression.MaxThreshold))
    assert score.tolist() == [20]


# --- randomized parity -----------------------------------------------------------------

def _images(rng, w, h):
    yield rng.integers(0, 256, (h, w), dtype=np.uint8)                        # dense corners
    blocks = rng.integers(0, 256, ((h + 5) // 6, (w + 5) // 6), dtype=np.uint8)
    img = np.repeat(np.repeat(blocks, 6, 0), 6, 1)[:h, :w]
    yield np.clip(img.astype(int) + rng.integers(0, 8, (h, w)), 0, 255).astype(np.uint8)
    yield (rng.integers(100, 140, (h, w))).astype(np.uint8)                   # low contrast


SIZES = [(7, 7), (8, 7), (7, 12), (9, 9), (15, 11), (16, 16), (17, 13), (19, 8), (31, 20),
         (33, 17), (64, 9), (65, 33), (100, 21), (257, 14), (300, 200), (1023, 12),
         (1024, 10), (1025, 19), (1027, 9), (1031, 24), (2050, 13), (1920, 18)]


@pytest.mark.parametrize("w,h", SIZES)
def test_random_sizes_all_modes(w, h):
    rng = np.random.default_rng(w * 1000 + h)
    for img in _images(rng, w, h):
        for nms in (0, 1, 2):
            for t, n in ((16, 9), (int(rng.integers(0, 60)), int(rng.integers(9, 17)))):
                assert_same(img, t, n, nms)


@pytest.mark.parametrize("n", range(9, 17))
def test_every_count(n):
    rng = np.random.default_rng(n)
    for img in _images(rng, 333, 77):
        for nms in (0, 1, 2):
            for t in (0, 1, 10, 25, 60):
                assert_same(img, t, n, nms)


@pytest.mark.parametrize("t", [0, 1, 2, 127, 128, 200, 254, 255])
def test_threshold_saturation(t):
    """c + t > 255 and c < t exercise the reference's saturating bounds (:224-231)."""
    rng = np.random.default_rng(1000 + t)
    img = rng.integers(0, 256, (40, 90), dtype=np.uint8)
    img[::7] = 255
    img[:, ::5] = 0
    for n in (9, 12, 16):
        for nms in (0, 1, 2):
            assert_same(img, t, n, nms)


def test_border_rows_and_tail_columns():
    """Rows 3 and h-4 under NMS, and columns in the reference's scalar tail (:559-586)."""
    rng = np.random.default_rng(7)
    for w in (22, 38, 300, 1040):
        h = 15
        img = np.full((h, w), 128, dtype=np.uint8)
        for y in (3, 4, h - 5, h - 4):
            for x in range(3, w - 3, 5):
                img[y, x] = 250 if rng.integers(2) else 5
        for nms in (0, 1, 2):
            assert_same(img, 20, 9, nms)


def test_plateau_ties():
    """Equal neighbour scores suppress both (strict '>', src/fast_simd.rs:605-607)."""
    img = np.full((40, 60), 50, dtype=np.uint8)
    img[10:30, 10:50] = 200
    for nms in (0, 1, 2):
        for n in (9, 12):
            assert_same(img, 30, n, nms)


# --- full-size frames ------------------------------------------------------------------

@pytest.mark.parametrize("gen", ["s1", "s2", "s3"])
def test_1080p(gen):
    img = {"s1": workloads.s1_frame(3), "s2": workloads.s2_frame(0),
           "s3": workloads.s3_frame(0)}[gen]
    for t, n, nms in ((16, 9, 0), (16, 9, 1), (16, 9, 2)):
        assert_same(img, t, n, nms)


@pytest.fixture
def full_geometry():
    """Run small jobs with the full-size geometry (tall bands, long units, pipelined batches
    and FIFO overflow) that large batches get: fdf_ctx_set_geometry(ctx, 1) on the shared
    device-0 context, restored afterwards."""
    ctx = fast_hip.context(0)
    ctx.set_geometry(1)
    yield
    ctx.set_geometry(0)


@pytest.mark.parametrize("gen", ["s1", "s2", "s3"])
def test_1080p_full_geometry(full_geometry, gen):
    img = {"s1": workloads.s1_frame(5), "s2": workloads.s2_frame(1),
           "s3": workloads.s3_frame(2)}[gen]
    for t, n, nms in ((16, 9, 0), (16, 9, 1), (16, 9, 2), (10, 12, 1)):
        assert_same(img, t, n, nms)


def test_batch_full_geometry(full_geometry):
    frames = np.stack([workloads.s1_frame(i) for i in range(3)] + [workloads.s3_frame(7)])
    cfg = Config(16, 9, NonMaximalSuppression.MaxThreshold)
    pts, offs = fast_hip.detector_batch(frames, cfg)
    for f in range(frames.shape[0]):
        assert np.array_equal(pts[offs[f]:offs[f + 1]], oracle.detect(frames[f], 16, 9, 1)), f


def test_4k_full_geometry(full_geometry):
    img = workloads.s1_frame(3, 3840, 2160)
    assert_same(img, 8, 12, 2)
    assert_same(img, 16, 9, 0)


@pytest.mark.parametrize("nms", [0, 1, 2])
def test_full_geometry_every_n(full_geometry, nms):
    """Dense candidates (noise with 2-row structure, low threshold) keep the FIFO near full in every unit,
    so the overflow path runs inside issue steps for every circle count."""
    rng = np.random.default_rng(77)
    img = rng.integers(0, 256, (1080, 1920), dtype=np.uint8)
    img[::2] = img[1::2]                                   # some 2-row structure
    for n in range(9, 17):
        assert_same(img, 6 if n < 13 else 3, n, nms)


@pytest.mark.parametrize("shape", [(613, 1001), (1500, 37), (9, 2000), (1079, 1919)])
def test_full_geometry_ragged(full_geometry, shape):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    img = (rng.integers(0, 256, shape, dtype=np.uint8) // 3 * 3).astype(np.uint8)
    for nms in (0, 1, 2):
        assert_same(img, 12, 9, nms)


def test_4k_t8_n12_sad():
    """BASELINE config 5 shape: 3840x2160 t=8 n=12 SAD."""
    assert_same(workloads.s1_frame(1, 3840, 2160), 8, 12, 2)


# --- errors, edge shapes, capacity -----------------------------------------------------

@pytest.mark.parametrize("w,h", [(w, h) for h in range(0, 9) for w in (0, 1, 5, 6, 7, 9)])
def test_edge_shapes_match_reference_rules(w, h):
    img = np.random.default_rng(w + 17 * h).integers(0, 256, (h, w), dtype=np.uint8)
    for nms in (0, 1):
        status, empty = oracle.check(w, h, 9, nms)
        if status < 0:
            with pytest.raises(FdfError) as e:
                run(img, 10, 9, nms)
            assert e.value.status == _native.FDF_ERR_SIZE
        else:
            got = run(img, 10, 9, nms)
            assert np.array_equal(got, oracle.detect(img, 10, 9, nms))
            if empty:
                assert len(got) == 0


@pytest.mark.parametrize("n,code", [(0, _native.FDF_ERR_COUNT), (8, _native.FDF_ERR_COUNT),
                                    (17, _native.FDF_ERR_COUNT), (255, _native.FDF_ERR_COUNT)])
def test_bad_count(golden, n, code):
    with pytest.raises(FdfError) as e:
        run(golden[0], 16, n, 0)
    assert e.value.status == code


def test_bad_nms_and_capacity(golden):
    img = golden[0]
    lib = _native.load()
    ctx = fast_hip.context(0)
    cfg = _native.FdfConfig(16, 9, 3)
    n = ctypes.c_size_t(0)
    assert lib.fdf_detect(ctx.handle, img.ctypes.data, 300, 200, 300, ctypes.byref(cfg), None, 0,
                          ctypes.byref(n)) == _native.FDF_ERR_NMS
    cfg = _native.FdfConfig(16, 9, 0)
    out = np.zeros((100, 2), dtype=np.uint32)
    rc = lib.fdf_detect(ctx.handle, img.ctypes.data, 300, 200, 300, ctypes.byref(cfg),
                        out.ctypes.data, 100, ctypes.byref(n))
    assert rc == _native.FDF_ERR_CAPACITY and n.value == 309
    assert np.array_equal(out, golden[1][:100])


def test_strided_input(golden):
    img = golden[0]
    wide = np.zeros((200, 320), dtype=np.uint8)
    wide[:, :300] = img
    view = wide[:, :300]
    assert not view.flags.c_contiguous
    assert np.array_equal(fast_hip.detect_array(view, Config(16, 9)), golden[1])


# --- batches, device path, repeatability -----------------------------------------------

def test_batch_matches_per_frame():
    frames = np.stack([workloads.s1_frame(i, 640, 360) for i in range(5)] +
                      [workloads.s3_frame(1, 640, 360)])
    for nms in (0, 1, 2):
        pts, offs = fast_hip.detector_batch(frames, Config(16, 9, NonMaximalSuppression(nms)))
        assert offs[-1] == len(pts)
        for f in range(frames.shape[0]):
            want = oracle.detect(frames[f], 16, 9, nms)
            assert np.array_equal(pts[offs[f]:offs[f + 1]], want), (nms, f)


def test_device_batch_torch():
    torch = pytest.importorskip("torch")
    frames = workloads.s1_frames_torch(10, 6)
    out = torch.zeros((200_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(7, dtype=torch.int64, device="cuda")
    for nms in (0, 1):
        cfg = Config(16, 9, NonMaximalSuppression(nms))
        fast_hip.detect_device(frames, cfg, out, offs)
        torch.cuda.synchronize()
        o = offs.cpu().numpy()
        got = out[: int(o[-1])].cpu().numpy().astype(np.uint32)
        host = frames.cpu().numpy()
        for f in range(6):
            assert np.array_equal(got[o[f]:o[f + 1]], oracle.detect(host[f], 16, 9, nms))


def test_device_capacity_overflow_reports_total():
    torch = pytest.importorskip("torch")
    frames = workloads.s1_frames_torch(0, 3, 640, 480)
    out = torch.full((50, 2), -1, dtype=torch.int32, device="cuda")
    offs = torch.zeros(4, dtype=torch.int64, device="cuda")
    fast_hip.detect_device(frames, Config(16, 9), out, offs)
    torch.cuda.synchronize()
    want = [oracle.detect(frames[f].cpu().numpy(), 16, 9, 0) for f in range(3)]
    total = sum(len(w) for w in want)
    assert int(offs[-1]) == total > 50
    assert np.array_equal(out.cpu().numpy().astype(np.uint32), np.concatenate(want)[:50])


@pytest.mark.parametrize("nms", [0, 1])
def test_bitmap_and_list_bands_mixed(full_geometry, nms):
    """Bands with more keypoints than their slot holds are written as keep-bitmaps and
    expanded by compact_kernel.  Frames whose top half is noise and bottom half S1 put bitmap
    and point-list bands in the same compaction group; a device capacity that cuts inside the
    first frame's bitmap bands keeps exactly the first `cap` points."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5 + nms)
    host = np.stack([workloads.s1_frame(i) for i in range(3)])
    host[:, :540] = rng.integers(0, 256, (3, 540, 1920), dtype=np.uint8)
    want = [oracle.detect(host[f], 6, 9, nms) for f in range(3)]
    cfg = Config(6, 9, NonMaximalSuppression(nms))
    pts, offs = fast_hip.detector_batch(host, cfg)
    for f in range(3):
        assert np.array_equal(pts[offs[f]:offs[f + 1]], want[f]), f
    frames = torch.from_numpy(host).cuda()
    cap = len(want[0]) // 2 + 17
    out = torch.full((cap, 2), -1, dtype=torch.int32, device="cuda")
    offs_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    fast_hip.detect_device(frames, cfg, out, offs_d)
    torch.cuda.synchronize()
    assert int(offs_d[-1]) == sum(len(w) for w in want)
    assert np.array_equal(out.cpu().numpy().astype(np.uint32), np.concatenate(want)[:cap])


@pytest.mark.parametrize("nms", [1, 2])
def test_dense_nms_batch_deterministic(nms):
    """A 512-frame 1080p batch at t=8 n=12 (BASELINE config 5's setting; many bands with
    more neighbouring keypoints than the LDS list holds): repeated launches give identical
    points, and the densest frames equal the oracle's."""
    torch = pytest.importorskip("torch")
    F = 512
    frames = workloads.s1_frames_torch(0, F, 1920, 1080)
    cfg = Config(8, 12, NonMaximalSuppression(nms))
    out = torch.empty((F * 60_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    runs = []
    for _ in range(4):
        fast_hip.detect_device(frames, cfg, out, offs)
        torch.cuda.synchronize()
        n = int(offs[-1])
        assert n <= out.shape[0]
        runs.append((offs.cpu().numpy().copy(), out[:n].cpu().numpy().copy()))
    for o, p in runs[1:]:
        assert np.array_equal(o, runs[0][0])
        assert np.array_equal(p, runs[0][1])
    o, p = runs[0]
    counts = np.diff(o)
    for f in sorted(np.argsort(counts)[-3:].tolist() + [0]):
        want = oracle.detect(frames[f].cpu().numpy(), 8, 12, nms)
        assert np.array_equal(p[o[f]:o[f + 1]].astype(np.uint32), want), f


def test_repeat_launches_identical():
    """The context's buffers (slots, counts, score map) are reused across launches and never
    cleared; results must not drift."""
    img = workloads.s2_frame(5)
    first = run(img, 16, 9, 1)
    for _ in range(5):
        assert np.array_equal(run(img, 16, 9, 1), first)
    assert np.array_equal(first, oracle.detect(img, 16, 9, 1))


def test_two_contexts_two_threads():
    frames = [workloads.s1_frame(i, 800, 600) for i in range(4)]
    want = [oracle.detect(f, 16, 9, 2) for f in frames]
    errors = []

    def work(k):
        try:
            ctx = _native.Context(0)
            lib = _native.load()
            cfg = _native.FdfConfig(16, 9, 2)
            for _ in range(3):
                for f, w in zip(frames, want):
                    out = np.zeros((len(w) + 10, 2), dtype=np.uint32)
                    n = ctypes.c_size_t(0)
                    _native.check(lib.fdf_detect(ctx.handle, f.ctypes.data, 800, 600, 800,
                                                 ctypes.byref(cfg), out.ctypes.data,
                                                 out.shape[0], ctypes.byref(n)))
                    assert np.array_equal(out[: n.value], w)
            ctx.close()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors


def test_scores_match_oracle():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (60, 70), dtype=np.uint8)
    ys, xs = np.mgrid[3:57, 3:67]
    pts = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.uint32)
    ring = fast_hip.circle()
    for n in (9, 12, 16):
        for t in (0, 16, 90):
            mt = fast_hip.keypoint_scores(img, pts, Config(t, n, NonMaximalSuppression.MaxThreshold))
            sad = fast_hip.keypoint_scores(img, pts, Config(t, n, NonMaximalSuppression.SumAbsolute))
            for k in range(0, len(pts), 37):
                x, y = int(pts[k][0]), int(pts[k][1])
                circ = [int(img[y + dy, x + dx]) for dx, dy in ring]
                c = int(img[y, x])
                assert mt[k] == oracle.score_max_threshold(c, circ, n)
                assert sad[k] == oracle.score_sum_abs(c, circ, t)


def test_cpp_api_binary(golden):
    exe = os.path.join(ROOT, "tests", "cpp", "test_cpp_api")
    g = os.path.join(ROOT, "tests", "golden")
    res = subprocess.run([exe, os.path.join(g, "screenshot315_grey.pgm"),
                          os.path.join(g, "kp_t16_n9_off.txt"),
                          os.path.join(g, "kp_t16_n9_maxt.txt")],
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "off=309 maxt=131" in res.stdout
