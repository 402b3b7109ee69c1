"""The HIP detector: drop-in for the reference's ``fast_simd`` module (src/fast_simd.rs).

``detector(img, config)`` replaces ``fast_simd::detector`` (src/fast_simd.rs:847-859) and
returns ``list[Point]`` in raster order.  Array and batched variants return numpy arrays;
``detect_device`` keeps everything in HBM (torch CUDA tensors) for throughput.
"""
import collections
import ctypes
import threading

import numpy as np

from . import _native
from ._native import FdfConfig, FdfError, check
from .types import Config, GrayImage, NonMaximalSuppression, Point

# src/fast_simd.rs:69-72
NORTH = 0
EAST = 4
SOUTH = 8
WEST = 12

_CIRCLE = ((0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3),
           (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3))


def circle():
    """The 16-pixel Bresenham circle, index 0 north then clockwise (src/fast_simd.rs:79-98)."""
    return list(_CIRCLE)


def calculate_offsets(width):
    """Row-major memory offsets of the circle points (src/fast_simd.rs:104-110)."""
    return [dy * int(width) + dx for dx, dy in _CIRCLE]


_ctx_lock = threading.Lock()
_contexts = {}
_shard_contexts = {}


def context(device=0):
    """The process-wide :class:`_native.Context` for ``device`` (created on first use)."""
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = _native.Context(device)
            ctx.lock = threading.Lock()     # holds a two-call pattern together
            _contexts[device] = ctx
        return ctx


def shard_contexts(devices):
    """One distinct context per entry of ``devices`` (a device listed twice gets two
    contexts), for :func:`detector_batch` over several devices."""
    out, seen = [], {}
    with _ctx_lock:
        for dev in devices:
            k = seen.get(dev, 0)
            seen[dev] = k + 1
            ctx = _shard_contexts.get((dev, k))
            if ctx is None:
                ctx = _native.Context(dev)
                ctx.lock = threading.Lock()
                _shard_contexts[(dev, k)] = ctx
            out.append(ctx)
    return out


def _to_c_config(config):
    if not isinstance(config, Config):
        raise TypeError("config must be a feature_detector_fast_amd.Config")
    for name, v in (("threshold", config.threshold), ("count", config.count)):
        if not 0 <= int(v) <= 255:
            raise ValueError(f"{name} must fit in u8")
    nms = int(config.non_maximal_supression)
    if not 0 <= nms <= 255:
        raise FdfError(_native.FDF_ERR_NMS, "config")
    return FdfConfig(int(config.threshold), int(config.count), nms)


def _as_pixels(img):
    if isinstance(img, GrayImage):
        arr = img.array()
    else:
        arr = np.asarray(img)
    if arr.ndim != 2:
        raise ValueError("expected a 2-D grayscale image (H, W)")
    if arr.dtype != np.uint8:
        raise TypeError("expected uint8 pixels")
    if arr.strides[1] != 1:
        arr = np.ascontiguousarray(arr)
    return arr


def capacity_guess(pixels):
    """First output capacity of the two-call pattern: 1 keypoint per 64 pixels (real images
    have 0.5-1.5 per 100; denser results are fetched with fdf_fetch_last, not recomputed)."""
    return max(4096, int(pixels) // 64)


def _two_call(ctx, pixels, call, where, scored=False):
    """Run ``call(out_ptr, scores_ptr, cap, n_ref)`` with a guessed capacity; on
    FDF_ERR_CAPACITY copy the retained device result out with fdf_fetch_last (the detection
    runs once either way)."""
    lib = _native.load()
    cap = capacity_guess(pixels)
    out = np.empty((cap, 2), dtype=np.uint32)
    scores = np.empty(cap, dtype=np.uint16) if scored else None
    n = ctypes.c_size_t(0)
    with ctx.lock:
        rc = call(out.ctypes.data, scores.ctypes.data if scored else None, cap, n)
        if rc == _native.FDF_ERR_CAPACITY:
            out = np.empty((n.value, 2), dtype=np.uint32)
            scores = np.empty(n.value, dtype=np.uint16) if scored else None
            rc = lib.fdf_fetch_last(ctx.handle, out.ctypes.data,
                                    scores.ctypes.data if scored else None, n.value,
                                    ctypes.byref(n))
            where = "fdf_fetch_last"
    check(rc, where)
    k = n.value
    return (out[:k], scores[:k]) if scored else out[:k]


def detect_array(img, config, device=0):
    """Keypoints as a (K, 2) uint32 array of (x, y) rows in raster order."""
    arr = _as_pixels(img)
    cfg = _to_c_config(config)
    h, w = arr.shape
    ctx = context(device)
    lib = _native.load()
    stride = arr.strides[0] if arr.size else w
    ptr = arr.ctypes.data if arr.size else None
    return _two_call(ctx, w * h, lambda o, _s, cap, n: lib.fdf_detect(
        ctx.handle, ptr, w, h, stride, ctypes.byref(cfg), o, cap, ctypes.byref(n)), "fdf_detect")


def detector(img, config):
    """Drop-in for fast_simd::detector: ``list[Point]`` in raster order."""
    return [Point(int(x), int(y)) for x, y in detect_array(img, config)]


def detect_rgb_array(rgb, config, device=0):
    """Keypoints of an RGB8 (H, W, 3) image: converted on the device as image 0.24.6's
    to_luma8 (what the reference's callers do, src/main.rs:58), then detected."""
    arr = np.asarray(rgb)
    if arr.ndim != 3 or arr.shape[2] != 3 or arr.dtype != np.uint8:
        raise ValueError("expected an (H, W, 3) uint8 RGB image")
    if arr.strides[1] != 3 or arr.strides[2] != 1:
        arr = np.ascontiguousarray(arr)
    cfg = _to_c_config(config)
    h, w = arr.shape[:2]
    ctx = context(device)
    lib = _native.load()
    stride = arr.strides[0] if arr.size else 3 * w
    ptr = arr.ctypes.data if arr.size else None
    return _two_call(ctx, w * h, lambda o, _s, cap, n: lib.fdf_detect_rgb(
        ctx.handle, ptr, w, h, stride, ctypes.byref(cfg), o, cap, ctypes.byref(n)),
        "fdf_detect_rgb")


def detector_rgb(rgb, config):
    """``list[Point]`` for an RGB8 image (luma conversion on the device)."""
    return [Point(int(x), int(y)) for x, y in detect_rgb_array(rgb, config)]


def rgb_to_luma(frames, out, stream=None, device=None):
    """Device-side RGB8 -> grey of torch uint8 CUDA tensors: ``frames`` (F, H, W, 3)
    contiguous, ``out`` (F, H, W).  Asynchronous on ``stream`` (default: torch's current)."""
    import torch

    if frames.dim() != 4 or frames.shape[3] != 3 or frames.dtype != torch.uint8 or \
            not frames.is_contiguous():
        raise ValueError("frames must be a contiguous (F, H, W, 3) uint8 tensor")
    if out.shape != frames.shape[:3] or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("out must be a contiguous (F, H, W) uint8 tensor")
    if not frames.is_cuda or not out.is_cuda:
        raise ValueError("rgb_to_luma needs CUDA (HIP) tensors")
    dev = frames.device.index if device is None else device
    ctx = context(dev)
    if stream is None:
        stream = torch.cuda.current_stream(frames.device)
    f, h, w = frames.shape[:3]
    lib = _native.load()
    check(lib.fdf_rgb_to_luma_device(ctx.handle, frames.data_ptr(), f, w, h, 3 * w * h,
                                     out.data_ptr(), ctypes.c_void_p(stream.cuda_stream)),
          "fdf_rgb_to_luma_device")


def detector_batch(frames, config, device=0, devices=None):
    """Detect on a (F, H, W) uint8 stack.  Returns (points (K, 2) uint32, offsets (F+1,))
    where frame f's keypoints are points[offsets[f]:offsets[f+1]].

    ``devices``: a list of HIP device ids to shard the frames over (contiguous shards, one
    host thread and context per entry, results in frame order: fdf_detect_batch_multi).  A
    device may be listed more than once (several contexts on one GPU)."""
    frames = np.ascontiguousarray(np.asarray(frames), dtype=np.uint8)
    if frames.ndim != 3:
        raise ValueError("expected a (F, H, W) uint8 stack")
    f, h, w = frames.shape
    cfg = _to_c_config(config)
    lib = _native.load()
    offsets = np.zeros(f + 1, dtype=np.uint64)
    ptr = frames.ctypes.data if frames.size else None
    if devices is None:
        ctx = context(device)
        pts = _two_call(ctx, f * h * w, lambda o, _s, cap, n: lib.fdf_detect_batch(
            ctx.handle, ptr, f, w, h, h * w, ctypes.byref(cfg), o, cap, offsets.ctypes.data,
            ctypes.byref(n)), "fdf_detect_batch")
        return pts, offsets
    ctxs = shard_contexts(list(devices))
    handles = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    cap = capacity_guess(f * h * w)
    out = np.empty((cap, 2), dtype=np.uint32)
    n = ctypes.c_size_t(0)
    # one global lock order (by handle), whatever order the caller lists the devices in:
    # detector_batch(devices=[0, 1]) and devices=[1, 0] from two threads cannot deadlock
    locked = sorted(ctxs, key=lambda c: c.handle.value)
    for c in locked:
        c.lock.acquire()
    try:
        rc = lib.fdf_detect_batch_multi(handles, len(ctxs), ptr, f, w, h, h * w,
                                        ctypes.byref(cfg), out.ctypes.data, cap,
                                        offsets.ctypes.data, ctypes.byref(n))
        where = "fdf_detect_batch_multi"
        if rc == _native.FDF_ERR_CAPACITY:
            out = np.empty((n.value, 2), dtype=np.uint32)
            rc = lib.fdf_fetch_last_multi(handles, len(ctxs), out.ctypes.data, n.value,
                                          ctypes.byref(n))
            where = "fdf_fetch_last_multi"
    finally:
        for c in reversed(locked):
            c.lock.release()
    check(rc, where)
    return out[: n.value], offsets


def detect_device(frames, config, out, offsets, stream=None, device=None, ctx=None):
    """Enqueue detection on device-resident frames; nothing crosses PCIe.

    ``frames``: torch uint8 CUDA tensor (F, H, W), contiguous.  ``out``: int32/uint32 CUDA
    tensor (cap, 2).  ``offsets``: int64 CUDA tensor (F+1,).  Asynchronous on ``stream``
    (a torch.cuda.Stream; default: torch's current stream).  On completion
    offsets[F] holds the total (even when it exceeds ``cap``).  ``ctx``: the context whose
    workspace the call uses (default: the device's process-wide one; see :class:`Lanes`)."""
    import torch

    if frames.dim() != 3 or frames.dtype != torch.uint8 or not frames.is_contiguous():
        raise ValueError("frames must be a contiguous (F, H, W) uint8 tensor")
    if not frames.is_cuda or not out.is_cuda or not offsets.is_cuda:
        raise ValueError("detect_device needs CUDA (HIP) tensors")
    if offsets.dtype != torch.int64 or offsets.numel() < frames.shape[0] + 1:
        raise ValueError("offsets must be int64 with F+1 entries")
    if out.dim() != 2 or out.shape[1] != 2 or out.element_size() != 4 or not out.is_contiguous():
        raise ValueError("out must be a contiguous (cap, 2) 32-bit tensor")
    dev = frames.device.index if device is None else device
    cfg = _to_c_config(config)
    if ctx is None:
        ctx = context(dev)
    if stream is None:
        stream = torch.cuda.current_stream(frames.device)
    f, h, w = frames.shape
    rc = _native.load().fdf_detect_device(
        ctx.handle, frames.data_ptr(), f, w, h, h * w, ctypes.byref(cfg), out.data_ptr(),
        out.shape[0], offsets.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    check(rc, "fdf_detect_device")


class Lanes:
    """``n`` launch lanes on one device for back-to-back device-resident batches: lane i is a
    context of its own (workspace: band slots, counts, sums) and the HIP stream that context
    created.  Call k goes to lane k % n with no dependency on the other lanes, so one call's
    detector runs beside the previous calls' last workgroups and compaction: with n = 3, 512
    1080p frames take 0.391 ms per call against 0.442 ms on one stream.

    Ordering: with ``after_current=True`` (default) each call first makes its lane wait for
    the work already enqueued on torch's current stream (the producer of ``frames``), and
    :meth:`wait` makes the current stream wait for a lane's last call (before reading its
    ``out`` / ``offsets``).  Each lane needs its own ``out`` / ``offsets`` buffers while its
    call may still run."""

    def __init__(self, n=3, device=0):
        if n < 1:
            raise ValueError("at least one lane")
        self.device = int(device)
        # every lane a context of its own, the process-wide context(device) included: no
        # state of other callers' calls (workspace sizes, ticket counters, completion stream)
        # reaches a lane, and close() destroys them all
        self.ctxs = []
        for _ in range(n):
            ctx = _native.Context(self.device)
            ctx.lock = threading.Lock()
            self.ctxs.append(ctx)
        self._ext = [None] * n
        # per lane: (event recorded after a call, the tensors that call borrows), oldest first
        self._held = [collections.deque() for _ in range(n)]

    def __len__(self):
        return len(self.ctxs)

    def stream(self, lane):
        """Lane ``lane``'s HIP stream as a torch.cuda.ExternalStream (events, waits)."""
        import torch

        if self._ext[lane] is None:
            self._ext[lane] = torch.cuda.ExternalStream(self.ctxs[lane].stream,
                                                        device=torch.device("cuda", self.device))
        return self._ext[lane]

    def _hold(self, lane, tensors):
        """Keep `tensors` referenced until the lane's stream has passed the call just enqueued
        (an event recorded after it), and drop the references of earlier calls it has passed.
        (Not Tensor.record_stream: the caching allocator would then record events on the lane's
        stream when the tensor is freed, which may be after the context -- and its stream --
        is gone.)"""
        import torch

        q = self._held[lane]
        while q and q[0][0].query():
            q.popleft()
        ev = torch.cuda.Event()
        ev.record(self.stream(lane))
        q.append((ev, tensors))

    def detect_device(self, k, frames, config, out, offsets, after_current=True):
        """detect_device on lane k % n (asynchronous on that lane's stream).

        The call borrows ``frames``, ``out`` and ``offsets`` until the lane's work is done,
        as the reference's detector borrows its image for the call (src/fast_simd.rs:847):
        the lane keeps a reference to each until its stream has passed the call, so torch's
        caching allocator cannot hand their memory to another tensor while the lane still
        reads or writes it, even when the caller drops its last reference right after this
        call."""
        import torch

        lane = k % len(self.ctxs)
        s = self.stream(lane)
        if after_current:
            s.wait_stream(torch.cuda.current_stream(frames.device))
        detect_device(frames, config, out, offsets, stream=s, device=self.device,
                      ctx=self.ctxs[lane])
        self._hold(lane, (frames, out, offsets))
        return lane

    def wait(self, lane=None):
        """Make torch's current stream wait for lane ``lane`` (every lane when None)."""
        import torch

        cur = torch.cuda.current_stream(torch.device("cuda", self.device))
        for i in (range(len(self.ctxs)) if lane is None else [lane]):
            cur.wait_stream(self.stream(i))

    def close(self):
        """Wait for every lane, release the borrowed tensors, destroy the lanes' contexts."""
        try:
            for q in self._held:
                if q:
                    q[-1][0].synchronize()
        finally:
            # also after a device error: drop the borrows and the lanes' contexts (each
            # context's destroy drains its own stream first)
            for ctx in self.ctxs:
                ctx.close()
            for q in self._held:
                q.clear()
            self.ctxs = []
            self._ext = []
            self._held = []


def detect_device_rgb(frames, config, out, offsets, stream=None, device=None):
    """detect_device for RGB8 frames: ``frames`` a contiguous (F, H, W, 3) uint8 CUDA tensor;
    the detector converts pixels to luma (image 0.24.6 to_luma8) as it loads them
    (fdf_detect_device_rgb), so no grey copy is written."""
    import torch

    if frames.dim() != 4 or frames.shape[3] != 3 or frames.dtype != torch.uint8 or \
            not frames.is_contiguous():
        raise ValueError("frames must be a contiguous (F, H, W, 3) uint8 tensor")
    if not frames.is_cuda or not out.is_cuda or not offsets.is_cuda:
        raise ValueError("detect_device_rgb needs CUDA (HIP) tensors")
    if offsets.dtype != torch.int64 or offsets.numel() < frames.shape[0] + 1:
        raise ValueError("offsets must be int64 with F+1 entries")
    if out.dim() != 2 or out.shape[1] != 2 or out.element_size() != 4 or not out.is_contiguous():
        raise ValueError("out must be a contiguous (cap, 2) 32-bit tensor")
    dev = frames.device.index if device is None else device
    cfg = _to_c_config(config)
    ctx = context(dev)
    if stream is None:
        stream = torch.cuda.current_stream(frames.device)
    f, h, w = frames.shape[:3]
    rc = _native.load().fdf_detect_device_rgb(
        ctx.handle, frames.data_ptr(), f, w, h, 3 * h * w, ctypes.byref(cfg), out.data_ptr(),
        out.shape[0], offsets.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    check(rc, "fdf_detect_device_rgb")


def keypoint_scores(img, points, config, device=0):
    """u16 NMS scores of the given centres (extension: the reference's Point has no score).
    ``config.non_maximal_supression`` picks MaxThreshold (src/fast_simd.rs:623-718, window =
    count) or SumAbsolute (:722-749, uses threshold)."""
    arr = _as_pixels(img)
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.uint32).reshape(-1, 2))
    cfg = _to_c_config(config)
    h, w = arr.shape
    scores = np.zeros(pts.shape[0], dtype=np.uint16)
    ctx = context(device)
    # fdf_score_points reuses the context's retained result buffers: hold the lock that keeps
    # a two-call pattern (detect, then fdf_fetch_last) of another thread together
    with ctx.lock:
        rc = _native.load().fdf_score_points(
            ctx.handle, arr.ctypes.data, w, h, arr.strides[0], ctypes.byref(cfg),
            pts.ctypes.data, pts.shape[0], scores.ctypes.data)
    check(rc, "fdf_score_points")
    return scores


def _ring_config(score, t, n):
    return _native.FdfConfig(t, n, int(score))


def score_rings(centers, rings, score, threshold=0, consecutive=9, device=0):
    """u16 scores of (centre, 16 circle pixels) rings on the GPU (fdf_score_rings).
    ``score`` is NonMaximalSuppression.MaxThreshold (src/fast_simd.rs:623, window
    ``consecutive``) or SumAbsolute (:722, ``threshold``); ``rings`` is (K, 16) uint8 in
    circle() order, ``centers`` (K,) uint8."""
    c = np.ascontiguousarray(np.asarray(centers, dtype=np.uint8).reshape(-1))
    r = np.ascontiguousarray(np.asarray(rings, dtype=np.uint8).reshape(-1, 16))
    if r.shape[0] != c.shape[0]:
        raise ValueError("centers and rings differ in length")
    if not 0 <= int(threshold) <= 255:
        raise ValueError("threshold must fit u8")
    cfg = _ring_config(score, threshold, consecutive)
    out = np.zeros(c.shape[0], dtype=np.uint16)
    ctx = context(device)
    with ctx.lock:   # reuses the retained result buffers, see keypoint_scores
        rc = _native.load().fdf_score_rings(ctx.handle, c.ctypes.data, r.ctypes.data,
                                            c.shape[0], ctypes.byref(cfg), out.ctypes.data)
    check(rc, "fdf_score_rings")
    return out


def keypoint_score_max_threshold(base_v, pixels, consecutive):
    """src/fast_simd.rs:623 on one ring (16 circle pixels), computed on the GPU."""
    return int(score_rings([base_v], [pixels], NonMaximalSuppression.MaxThreshold,
                           consecutive=consecutive)[0])


def keypoint_score_sum_abs_difference(pixels, center, threshold):
    """src/fast_simd.rs:722 on one ring with the masks its callers build from ``threshold``
    (:1213-1222), computed on the GPU."""
    return int(score_rings([center], [pixels], NonMaximalSuppression.SumAbsolute,
                           threshold=threshold)[0])


def score_rings_device(centers, rings, scores, score, threshold=0, consecutive=9,
                       stream=None, device=None):
    """Device-resident fdf_score_rings_device: torch uint8 (K,) centres and (K, 16) rings,
    int16/uint16-sized (K,) scores tensor, all on one GPU; asynchronous on ``stream``."""
    import torch
    if rings.dim() != 2 or rings.shape[1] != 16 or centers.numel() != rings.shape[0] \
            or scores.numel() < rings.shape[0]:
        raise ValueError("rings must be (K, 16) with K centres and K scores")
    if centers.dtype != torch.uint8 or rings.dtype != torch.uint8:
        raise ValueError("centers and rings must be uint8 tensors")
    if not (centers.is_cuda and rings.is_cuda and scores.is_cuda):
        raise ValueError("score_rings_device needs CUDA (HIP) tensors")
    if not (centers.device == rings.device == scores.device):
        raise ValueError("centers, rings and scores must be on the same device")
    if not (centers.is_contiguous() and rings.is_contiguous() and scores.is_contiguous()):
        raise ValueError("tensors must be contiguous")
    if scores.element_size() != 2:
        raise ValueError("scores must be a 16-bit tensor")
    if rings.numel() and rings.data_ptr() % 16 != 0:
        raise ValueError("rings must start on a 16-byte boundary (one 16-byte load per ring)")
    dev = rings.device.index if device is None else device
    cfg = _ring_config(score, threshold, consecutive)
    if stream is None:
        stream = torch.cuda.current_stream(rings.device)
    rc = _native.load().fdf_score_rings_device(
        context(dev).handle, centers.data_ptr(), rings.data_ptr(), rings.shape[0],
        ctypes.byref(cfg), scores.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    check(rc, "fdf_score_rings_device")


def detect_scored_array(img, config, device=0):
    """Keypoints with scores: ((K, 2) uint32 (x, y) in raster order, (K,) uint16 scores).
    The score is the one the configured NMS suppresses with, max-threshold when NMS is off
    (fdf_detect_scored)."""
    arr = _as_pixels(img)
    cfg = _to_c_config(config)
    h, w = arr.shape
    ctx = context(device)
    lib = _native.load()
    stride = arr.strides[0] if arr.size else w
    ptr = arr.ctypes.data if arr.size else None
    return _two_call(ctx, w * h, lambda o, sc, cap, n: lib.fdf_detect_scored(
        ctx.handle, ptr, w, h, stride, ctypes.byref(cfg), o, sc, cap, ctypes.byref(n)),
        "fdf_detect_scored", scored=True)


def detector_scored(img, config):
    """``list[(Point, score)]`` in raster order (the (x, y, score) output)."""
    pts, scores = detect_scored_array(img, config)
    return [(Point(int(x), int(y)), int(s)) for (x, y), s in zip(pts, scores)]


def detector_batch_scored(frames, config, device=0):
    """detector_batch with scores: (points (K, 2), scores (K,) uint16, offsets (F+1,))."""
    frames = np.ascontiguousarray(np.asarray(frames), dtype=np.uint8)
    if frames.ndim != 3:
        raise ValueError("expected a (F, H, W) uint8 stack")
    f, h, w = frames.shape
    cfg = _to_c_config(config)
    ctx = context(device)
    lib = _native.load()
    offsets = np.zeros(f + 1, dtype=np.uint64)
    ptr = frames.ctypes.data if frames.size else None
    pts, scores = _two_call(ctx, f * h * w, lambda o, sc, cap, n: lib.fdf_detect_batch_scored(
        ctx.handle, ptr, f, w, h, h * w, ctypes.byref(cfg), o, sc, cap, offsets.ctypes.data,
        ctypes.byref(n)), "fdf_detect_batch_scored", scored=True)
    return pts, scores, offsets


def score_device(frames, config, points, offsets, scores, stream=None, device=None):
    """Scores of detect_device's output, on the device: ``points`` (cap, 2) and ``offsets``
    as detect_device filled them, ``scores`` a (cap,) int16/uint16 CUDA tensor.
    Asynchronous on ``stream`` (default: torch's current stream)."""
    import torch

    if frames.dim() != 3 or frames.dtype != torch.uint8 or not frames.is_contiguous():
        raise ValueError("frames must be a contiguous (F, H, W) uint8 tensor")
    if not (frames.is_cuda and points.is_cuda and offsets.is_cuda and scores.is_cuda):
        raise ValueError("score_device needs CUDA (HIP) tensors")
    if scores.element_size() != 2 or not scores.is_contiguous() or \
            scores.numel() < points.shape[0]:
        raise ValueError("scores must be a contiguous 16-bit tensor with cap entries")
    if offsets.dtype != torch.int64 or offsets.numel() < frames.shape[0] + 1:
        raise ValueError("offsets must be int64 with F+1 entries")
    dev = frames.device.index if device is None else device
    cfg = _to_c_config(config)
    ctx = context(dev)
    if stream is None:
        stream = torch.cuda.current_stream(frames.device)
    f, h, w = frames.shape
    rc = _native.load().fdf_score_device(
        ctx.handle, frames.data_ptr(), f, w, h, h * w, ctypes.byref(cfg), points.data_ptr(),
        points.shape[0], offsets.data_ptr(), scores.data_ptr(),
        ctypes.c_void_p(stream.cuda_stream))
    check(rc, "fdf_score_device")


__all__ = ["NORTH", "EAST", "SOUTH", "WEST", "circle", "calculate_offsets", "context",
           "shard_contexts", "capacity_guess", "Lanes",
           "detect_array", "detector", "detector_batch", "detect_device", "keypoint_scores",
           "detect_scored_array", "detector_scored", "detector_batch_scored", "score_device",
           "detect_rgb_array", "detector_rgb", "rgb_to_luma", "detect_device_rgb",
           "score_rings", "score_rings_device", "keypoint_score_max_threshold",
           "keypoint_score_sum_abs_difference", "NonMaximalSuppression"]
