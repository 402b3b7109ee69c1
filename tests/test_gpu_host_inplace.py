"""fdf_detect on a frame in pinned host memory: the detector reads it in place over PCIe (no
copy before the launch; fdf_ctx_set_upload_chunks, include/fdf.h).

The buffer is reused across calls with different contents -- an L2 line cached from the
previous call's frame would show as a wrong list (the launch's system-scope acquire must make
the host's writes visible) -- at an aligned and an odd offset inside the allocation, and every list
equals the CPU oracle (oracle/fast_oracle.c, pinned to the reference's goldens; the image
contract is src/fast_simd.rs:307-330).  The two-call pattern keeps the frame for
fdf_fetch_last's scores; a result that fit asks for fdf_detect_scored instead."""
import ctypes

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import _native
from oracle import oracle

pytestmark = pytest.mark.gpu


def _pinned(nbytes):
    import torch

    return torch.empty(nbytes, dtype=torch.uint8).pin_memory()


def _detect(lib, ctx, ptr, w, h, t, n, nms, cap=None):
    cfg = _native.FdfConfig(t, n, nms)
    cap = w * h if cap is None else cap
    out = np.zeros((max(cap, 1), 2), dtype=np.uint32)
    got = ctypes.c_size_t(0)
    rc = lib.fdf_detect(ctx.handle, ctypes.c_void_p(ptr), w, h, w, ctypes.byref(cfg),
                        out.ctypes.data if cap else None, cap, ctypes.byref(got))
    return rc, out[: min(got.value, cap)], got.value


@pytest.mark.parametrize("offset", [0, 4096 + 13])
def test_in_place_frames_alternate(offset):
    W, H = 1920, 1080
    frames = [workloads.s1_frame(31), workloads.s3_frame(12), workloads.s2_frame(9),
              workloads.s1_frame(77)]
    buf = _pinned(W * H + 8192)
    view = buf.numpy()
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 3
                view[offset: offset + W * H] = f.reshape(-1)
                rc, got, _ = _detect(lib, ctx, buf.data_ptr() + offset, W, H, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(f, 16, 9, nms)), (rep, i, nms)
        # the same frames through one copy (chunks = 1) give the same lists
        ctx.set_upload_chunks(1)
        view[offset: offset + W * H] = frames[1].reshape(-1)
        rc, got, _ = _detect(lib, ctx, buf.data_ptr() + offset, W, H, 16, 9, 1)
        _native.check(rc, "fdf_detect")
        assert np.array_equal(got, oracle.detect(frames[1], 16, 9, 1))
    finally:
        ctx.close()


def test_in_place_small_and_ragged_frames():
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for (w, h) in [(7, 7), (33, 20), (641, 479), (1000, 7)]:
            img = workloads.s3_frame(5)[:h, :w].copy()
            buf = _pinned(w * h)
            buf.numpy()[:] = img.reshape(-1)
            for nms in (0, 1, 2):
                rc, got, _ = _detect(lib, ctx, buf.data_ptr(), w, h, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(img, 16, 9, nms)), (w, h, nms)
    finally:
        ctx.close()


def test_in_place_two_call_pattern_keeps_scores():
    """cap 0 -> FDF_ERR_CAPACITY; fdf_fetch_last then returns the points and their scores (the
    frame was copied for it).  A result that fit has no retained frame: scores -> FDF_ERR_ARG,
    points still fine."""
    W, H = 640, 480
    img = workloads.s1_frame(1, W, H)
    want, want_sc = oracle.detect(img, 16, 9, 1, with_scores=True)
    buf = _pinned(W * H)
    buf.numpy()[:] = img.reshape(-1)
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        rc, _, n = _detect(lib, ctx, buf.data_ptr(), W, H, 16, 9, 1, cap=0)
        assert rc == _native.FDF_ERR_CAPACITY and n == len(want)
        buf.numpy()[:] = 0          # the caller may reuse its buffer after the call
        out = np.zeros((n, 2), dtype=np.uint32)
        sc = np.zeros(n, dtype=np.uint16)
        got = ctypes.c_size_t(0)
        _native.check(lib.fdf_fetch_last(ctx.handle, out.ctypes.data, sc.ctypes.data, n,
                                         ctypes.byref(got)), "fdf_fetch_last")
        assert np.array_equal(out, want) and np.array_equal(sc, want_sc)

        buf.numpy()[:] = img.reshape(-1)
        rc, pts, n = _detect(lib, ctx, buf.data_ptr(), W, H, 16, 9, 1)
        _native.check(rc, "fdf_detect")
        assert np.array_equal(pts, want)
        assert lib.fdf_fetch_last(ctx.handle, out.ctypes.data, sc.ctypes.data, n,
                                  ctypes.byref(got)) == _native.FDF_ERR_ARG
        out[:] = 0
        _native.check(lib.fdf_fetch_last(ctx.handle, out.ctypes.data, None, n,
                                         ctypes.byref(got)), "fdf_fetch_last")
        assert np.array_equal(out, want)
    finally:
        ctx.close()


def _hip():
    """The HIP runtime already in the process (the one libfdf.so and torch use), never a
    second copy."""
    import os

    _native.load()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for fn in ("hipHostMalloc", "hipHostRegister", "hipHostFree", "hipHostUnregister"):
        getattr(hip, fn).restype = ctypes.c_int
    return hip


@pytest.mark.parametrize("kind", ["coherent", "registered"])
def test_in_place_other_pinned_kinds(kind):
    """Fine-grained (coherent) pinned memory is copied, not read in place; memory registered
    with hipHostRegister is read in place.  Either way the lists equal the oracle, across
    frames written into the same buffer."""
    W, H = 1280, 720
    frames = [workloads.s1_frame(3, W, H), workloads.s3_frame(7)[:H, :W].copy(),
              workloads.s1_frame(40, W, H)]
    hip = _hip()
    ptr = ctypes.c_void_p()
    keep = None
    if kind == "coherent":
        assert hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(W * H),
                                 ctypes.c_uint(0x40000000)) == 0
        view = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
    else:
        keep = np.zeros(W * H + 4096, dtype=np.uint8)
        base = keep.ctypes.data + (-keep.ctypes.data) % 4096   # page-aligned start
        view = np.ctypeslib.as_array(ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
        assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(W * H),
                                   ctypes.c_uint(0)) == 0
        ptr = ctypes.c_void_p(base)
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 3
                view[:] = f.reshape(-1)
                rc, got, _ = _detect(lib, ctx, ptr.value, W, H, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(f, 16, 9, nms)), (kind, rep, i, nms)
    finally:
        ctx.close()
        if kind == "coherent":
            assert hip.hipHostFree(ptr) == 0
        else:
            assert hip.hipHostUnregister(ptr) == 0


@pytest.mark.parametrize("chunks", [0, 4])
def test_in_place_registered_range_shorter_than_frame(chunks):
    """a frame whose first bytes sit in a hipHostRegister'ed range that ends before
    the frame does is copied, not read in place (reading it in place would read past the
    registration over PCIe).  The frame's last byte must map to the same contiguous device
    range as its first (fdf_api.cpp run_host).  ADVICE r05: the overlapped chunked upload
    (chunks = 4) stages such a frame as well, so no chunk copy is rejected and no fallback is
    counted."""
    W, H = 1280, 720
    img = workloads.s1_frame(11, W, H)
    hip = _hip()
    keep = np.zeros(W * H + 4096, dtype=np.uint8)
    base = keep.ctypes.data + (-keep.ctypes.data) % 4096
    view = np.ctypeslib.as_array(ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
    view[:] = img.reshape(-1)
    half = (W * H // 2) & ~4095                       # whole pages, half the frame
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(half), ctypes.c_uint(0)) == 0
    lib = _native.load()
    ctx = _native.Context(0)
    ctx.set_upload_chunks(chunks)
    try:
        for nms in (0, 1, 2):
            rc, got, _ = _detect(lib, ctx, base, W, H, 16, 9, nms)
            _native.check(rc, "fdf_detect")
            assert np.array_equal(got, oracle.detect(img, 16, 9, nms)), nms
        assert ctx.recoveries() == (0, 0)
    finally:
        ctx.close()
        assert hip.hipHostUnregister(ctypes.c_void_p(base)) == 0
