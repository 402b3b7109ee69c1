"""ctypes front-end of the CPU checker (oracle/fast_oracle.c) and of the AVX2 port of the
reference path (oracle/fast_avx2.cpp).  TEST INFRASTRUCTURE ONLY.

Parity status: pinned -- fast_oracle.c reproduces the reference's committed golden vectors
(tests/golden/, 309 keypoints NMS off and 131 max-t on media/Screenshot315_torch_grey.png,
identical for the Rust crate and OpenCV 3.2) and the reference unit-test KATs; see
tests/test_oracle.py.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(_HERE, "liboracle.so")
AVX2_LIB = os.path.join(_HERE, "libfast_avx2.so")

ERR_COUNT = -1
ERR_SIZE = -2
ERR_NMS = -4


class OracleError(ValueError):
    def __init__(self, code):
        self.code = code
        super().__init__({ERR_COUNT: "count", ERR_SIZE: "size", ERR_NMS: "nms"}.get(code, str(code)))


_lib = None
_avx = None


def _load():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(ORACLE_LIB)
        u8 = ctypes.c_uint8
        lib.fdf_oracle_is_corner.restype = ctypes.c_int
        lib.fdf_oracle_is_corner.argtypes = [u8, ctypes.c_void_p, u8, u8]
        lib.fdf_oracle_score_max_threshold.restype = ctypes.c_uint16
        lib.fdf_oracle_score_max_threshold.argtypes = [u8, ctypes.c_void_p, u8]
        lib.fdf_oracle_score_sum_abs.restype = ctypes.c_uint16
        lib.fdf_oracle_score_sum_abs.argtypes = [u8, ctypes.c_void_p, u8]
        lib.fdf_oracle_check.restype = ctypes.c_int
        lib.fdf_oracle_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u8, u8,
                                         ctypes.POINTER(ctypes.c_int)]
        lib.fdf_oracle_rgb_to_luma.restype = None
        lib.fdf_oracle_rgb_to_luma.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_size_t, ctypes.c_void_p]
        lib.fdf_oracle_detect.restype = ctypes.c_int64
        lib.fdf_oracle_detect.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_size_t, u8, u8, u8, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p]
        lib.fdf_oracle_score_points.restype = None
        lib.fdf_oracle_score_points.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                ctypes.c_size_t, u8, u8, u8, ctypes.c_void_p]
        lib.fdf_oracle_score_rings.restype = None
        lib.fdf_oracle_score_rings.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                               u8, u8, u8, ctypes.c_void_p]
        _lib = lib
    return _lib


def _load_avx2():
    global _avx
    if _avx is None:
        lib = ctypes.CDLL(AVX2_LIB)
        u8 = ctypes.c_uint8
        u32 = ctypes.c_uint32
        lib.fdf_avx2_detect.restype = ctypes.c_int64
        lib.fdf_avx2_detect.argtypes = [ctypes.c_void_p, u32, u32, u8, u8, u8, ctypes.c_void_p,
                                        ctypes.c_size_t]
        lib.fdf_avx2_time.restype = ctypes.c_double
        lib.fdf_avx2_time.argtypes = [ctypes.c_void_p, u32, ctypes.c_size_t, u32, u32, u8, u8,
                                      u8, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_uint64)]
        lib.fdf_avx2_time_pinned.restype = ctypes.c_double
        lib.fdf_avx2_time_pinned.argtypes = [ctypes.c_void_p, u32, ctypes.c_size_t, u32, u32, u8,
                                             u8, u8, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_uint64)]
        lib.fdf_avx2_detect_batch.restype = ctypes.c_int64
        lib.fdf_avx2_detect_batch.argtypes = [ctypes.c_void_p, u32, ctypes.c_size_t, u32, u32, u8,
                                              u8, u8, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_void_p]
        lib.fdf_avx2_samples.restype = ctypes.c_int64
        lib.fdf_avx2_samples.argtypes = [ctypes.c_void_p, u32, u32, u8, u8, u8, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_void_p]
        _avx = lib
    return _avx


def _circle_buf(circle):
    arr = (ctypes.c_uint8 * 16)(*[int(v) for v in circle])
    return arr


def is_corner(center, circle, t, n):
    return bool(_load().fdf_oracle_is_corner(center, _circle_buf(circle), t, n))


def score_max_threshold(center, circle, n):
    return int(_load().fdf_oracle_score_max_threshold(center, _circle_buf(circle), n))


def score_sum_abs(center, circle, t):
    return int(_load().fdf_oracle_score_sum_abs(center, _circle_buf(circle), t))


def score_points(img, points, kind, t, n):
    """Oracle scores (uint16) of centres `points` ((K, 2) x, y): kind 1 max-threshold with
    window n, kind 2 SAD with threshold t."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.uint32).reshape(-1, 2))
    out = np.zeros(pts.shape[0], dtype=np.uint16)
    if pts.shape[0]:
        _load().fdf_oracle_score_points(img.ctypes.data, img.shape[1], pts.ctypes.data,
                                        pts.shape[0], int(kind), int(t), int(n), out.ctypes.data)
    return out


def score_rings(centers, rings, kind, t, n):
    """Oracle scores (uint16) of rings ((K, 16) uint8, circle order) around `centers` (K,):
    kind 1 max-threshold with window n, kind 2 SAD with threshold t."""
    c = np.ascontiguousarray(np.asarray(centers, dtype=np.uint8).reshape(-1))
    r = np.ascontiguousarray(np.asarray(rings, dtype=np.uint8).reshape(-1, 16))
    out = np.zeros(c.shape[0], dtype=np.uint16)
    if c.shape[0]:
        _load().fdf_oracle_score_rings(c.ctypes.data, r.ctypes.data, c.shape[0], int(kind),
                                       int(t), int(n), out.ctypes.data)
    return out


def rgb_to_luma(rgb):
    """image 0.24.6 to_luma8 restated (fast_oracle.c): (H, W, 3) uint8 -> (H, W) uint8."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    if rgb.ndim != 3 or rgb.shape[2] != 3:
        raise ValueError("(H, W, 3) image expected")
    h, w = rgb.shape[:2]
    out = np.empty((h, w), dtype=np.uint8)
    if out.size:
        _load().fdf_oracle_rgb_to_luma(rgb.ctypes.data, w, h, 3 * w, out.ctypes.data)
    return out


def check(w, h, n, nms):
    """(status, empty) with the reference's size/count rules; status < 0 means it panics."""
    empty = ctypes.c_int(0)
    rc = _load().fdf_oracle_check(w, h, n, nms, ctypes.byref(empty))
    return rc, bool(empty.value)


def detect(img, t, n, nms, with_scores=False):
    """Keypoints (K, 2) uint32 (x, y) in raster order; raises OracleError where the
    reference panics."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim != 2:
        raise ValueError("2-D image expected")
    h, w = img.shape
    lib = _load()
    ptr = img.ctypes.data if img.size else None
    cnt = lib.fdf_oracle_detect(ptr, w, h, w, t, n, int(nms), None, 0, None)
    if cnt < 0:
        raise OracleError(cnt)
    out = np.empty((cnt, 2), dtype=np.uint32)
    scores = np.empty(cnt, dtype=np.uint16)
    if cnt:
        lib.fdf_oracle_detect(ptr, w, h, w, t, n, int(nms), out.ctypes.data, cnt,
                              scores.ctypes.data)
    return (out, scores) if with_scores else out


def _padded(img):
    """Copy into a buffer with 16 readable bytes after the last pixel (the reference's
    gathers read up to 3 bytes past the end)."""
    flat = np.zeros(img.size + 16, dtype=np.uint8)
    flat[: img.size] = img.reshape(-1)
    return flat


def avx2_detect(img, t, n, nms):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    buf = _padded(img)
    lib = _load_avx2()
    cnt = lib.fdf_avx2_detect(buf.ctypes.data, w, h, t, n, int(nms), None, 0)
    if cnt < 0:
        raise OracleError(cnt)
    out = np.empty((cnt, 2), dtype=np.uint32)
    if cnt:
        lib.fdf_avx2_detect(buf.ctypes.data, w, h, t, n, int(nms), out.ctypes.data, cnt)
    return out


def checker_threads():
    """Worker threads for whole-batch checks: the CPUs this process may use, at most the
    cgroup quota and at most 16 (the GPU box's CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return max(1, min(16, n))


def avx2_detect_batch(frames, t, n, nms, threads=None):
    """Every frame of a (F, H, W) stack (numpy, or a torch tensor on any device) through the
    AVX2 port (pinned to the scalar oracle: tests/test_oracle.py), frame f on worker
    f % threads.  Returns (points (K, 2) uint32, offsets (F+1,) uint64) in frame order -- the
    layout of fdf_detect_batch / detect_device -- for whole-batch parity checks."""
    if hasattr(frames, "cpu"):
        frames = frames.cpu().numpy()
    frames = np.asarray(frames, dtype=np.uint8)
    if frames.ndim != 3:
        raise ValueError("(F, H, W) stack expected")
    f, h, w = frames.shape
    buf = np.zeros(frames.size + 16, dtype=np.uint8)
    buf[: frames.size] = frames.reshape(-1)
    lib = _load_avx2()
    offsets = np.zeros(f + 1, dtype=np.uint64)
    th = checker_threads() if threads is None else int(threads)
    # one keypoint per 32 pixels first (real images: ~1 per 100); a denser batch runs again
    # with the exact size
    cap = max(1024, frames.size // 32)
    out = np.empty((cap, 2), dtype=np.uint32)
    cnt = lib.fdf_avx2_detect_batch(buf.ctypes.data, f, h * w, w, h, t, n, int(nms), th,
                                    out.ctypes.data, cap, offsets.ctypes.data)
    if cnt < 0:
        raise OracleError(cnt)
    if cnt > cap:
        out = np.empty((cnt, 2), dtype=np.uint32)
        lib.fdf_avx2_detect_batch(buf.ctypes.data, f, h * w, w, h, t, n, int(nms), th,
                                  out.ctypes.data, cnt, offsets.ctypes.data)
    return out[:cnt], offsets


def avx2_time(frames, t, n, nms, threads=1, reps=1, cpus=None):
    """Wall seconds for `reps` passes over a (F, H, W) stack with `threads` workers (frame f
    on worker f % threads; worker i pinned to CPU cpus[i] when `cpus` is given), and the
    keypoint total of one pass."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    f, h, w = frames.shape
    buf = np.zeros(frames.size + 16, dtype=np.uint8)
    buf[: frames.size] = frames.reshape(-1)
    total = ctypes.c_uint64(0)
    lib = _load_avx2()
    if cpus is None:
        secs = lib.fdf_avx2_time(buf.ctypes.data, f, h * w, w, h, t, n, int(nms), threads,
                                 reps, ctypes.byref(total))
    else:
        cpu_arr = np.ascontiguousarray(np.asarray(cpus, dtype=np.int32)[:threads])
        assert cpu_arr.size == threads
        secs = lib.fdf_avx2_time_pinned(buf.ctypes.data, f, h * w, w, h, t, n, int(nms), threads,
                                        reps, cpu_arr.ctypes.data, ctypes.byref(total))
    return secs, int(total.value)


def avx2_samples(img, t, n, nms, warmup=10, samples=100):
    """Per-call wall times (ms, float64 array) of the AVX2 port on one frame after `warmup`
    untimed calls (the reference's criterion protocol), and the keypoint count."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    buf = _padded(img)
    out = np.zeros(samples, dtype=np.float64)
    cnt = _load_avx2().fdf_avx2_samples(buf.ctypes.data, w, h, t, n, int(nms), warmup, samples,
                                        out.ctypes.data)
    return out, int(cnt)
